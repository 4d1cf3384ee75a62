// rdo_kern.h -- C4: fused per-block TX-type RDO kernels for gfx950, and the
// 64-point forward transform sizes (instantiated per mode in rdo_m0..3.hip,
// driven by rdo.hip).
//
// Per TX block and candidate TX type (the body of
// search_tx_type, av1/encoder/tx_search.c:2148-2312, with TX-domain
// distortion):
//   aom_highbd_subtract_block (aom_dsp/subtract.c:38-54)
//   -> av1_fwd_txfm2d_WxH (av1/encoder/av1_fwd_txfm2d.c:56-312, 64-point
//      sizes zeroed + re-packed to the 32x32 quadrant)
//   -> av1_highbd_quantize_fp (av1/encoder/av1_quantize.c:125-198,565-577)
//   -> aom_satd on the coefficients (aom_dsp/avg.c:509-516)
//   -> dist_block_tx_domain: av1_highbd_block_error, RIGHT_SIGNED_SHIFT by
//      (MAX_TX_SCALE - tx_scale) * 2 (tx_search.c:1077-1116)
//   -> rate_estimator (av1/encoder/tpl_model.c:214-226, DCT_DCT scan)
//   -> RDCOST(rdmult, rate, dist) (av1/encoder/rd.h:31-33)
// and the block keeps the first type with the strictly smallest cost (the
// `<` test of tx_search.c:2246).  Output per block: the decision record and
// the winning qcoeff / dqcoeff.
//
// Mode 0 of the same kernel is the plain lavish_txq_plane contract (every
// type's qcoeff / dqcoeff / eob) for the 64-point sizes, which txq.hip does
// not instantiate.
//
// Layout per wave: P = 64 / min(W,H) blocks.  Column pass: one column per
// lane (registers) -> LDS.  Row pass: only the KH = min(H,32) rows that
// survive the 64-point zeroing are transformed, one per lane; the lane then
// holds the row's KW = min(W,32) kept coefficients, quantizes them and
// contributes to the block reductions (xor shuffles over the KH lanes of the
// block).  The FAST 24-bit path is certified for |residual| <= 1023 for every
// size including the 64-point ones (tools/range_analysis.py).
#include <type_traits>

#include "coeffcost_dev.h"
#include "lane_red.h"
#include "lavish_internal.h"
#include "quant_dev.h"
#pragma once

namespace lavish {

struct RdoArgs {
  const int16_t* res;    // mode 0: residual plane
  const uint16_t* src;   // mode 1: source / prediction planes (u16)
  const uint16_t* pred;
  int stride;
  int bw, nblocks;
  int ntypes;
  int types[16];
  int bd;
  int quant_kind;  // mode 0
  int highbd;      // mode 0
  int rdmult;      // mode 1
  QP qp;
  const int16_t* iscan_type[16];  // per slot: inverse scan of the type (n)
  int scan_kind[16];              // per slot: its scan kind (0 default, 1 mcol, 2 mrow)
  const int16_t* scan_rows;       // the 3 kinds' inverse scans in lane-row order
                                  // ([kind][KH][KW], dev_iscan_rows)
  // evaluation order: slots grouped by vertical 1-D kind (one column pass per
  // group); newcol[i] = 1 where order[i] starts a group
  int order[16];
  int newcol[16];
  // decision modes, optional: per-block allowed_tx_mask and search order
  // (txk_map, [block][16]) as prune_tx_2D leaves them
  const uint16_t* block_mask;
  const uint8_t* block_map;
  const int16_t* iscan_dct;       // DCT_DCT inverse scan (rate_estimator)
  // MODE 3: the coefficient rate (av1_cost_coeffs_txb) replaces
  // rate_estimator: the size's luma LV_MAP_COEFF_COST / LV_MAP_EOB_COST,
  // per-block TXB_CTX (nullable: {0, 0}), get_tx_type_cost per tx type, and
  // the av1_nz_map_ctx_offset shape of the unadjusted size
  const int32_t* cc_cost;
  const int32_t* cc_eob;
  const LavishTxbCtx* txb_ctx;
  int tx_type_cost[16];
  int nz_wlt, nz_wgt;
  int32_t* qcoeff;
  int32_t* dqcoeff;
  uint16_t* eob;
  int32_t* coeff;
  LavishRdoBlock* out;
};

// The TX-domain decision (mode 1) of the 16x16, 8x8 and 4x4 sizes of one
// rectangle in one launch, for small rectangles (every present size would
// take the split form: fewer than kRdoSplitTiles tiles, four vertical-kind
// groups): workgroups [first[k], first[k + 1]) run size slot k (0: 16x16,
// 1: 8x8, 2: 4x4; the longest-lived first), four waves per tile as in the
// split form.  Replaces three launches on three streams and the cross-queue
// waits between them (~15-35 us each at these sizes).
struct RdoSmall {
  RdoArgs a[3];
  int first[4];
};
constexpr int kRdoSplitTiles = 2048;  // below this many tiles a mode-1 launch splits
int rdo_small_launch_m1(const RdoSmall& m, hipStream_t s);

// per mode: one size's launch (rdo_m<MODE>.hip); -2 for a size the mode
// does not instantiate
int rdo_launch_m0(int tx_size, const RdoArgs& a, hipStream_t s);
int rdo_launch_m1(int tx_size, const RdoArgs& a, hipStream_t s);
int rdo_launch_m2(int tx_size, const RdoArgs& a, hipStream_t s);
int rdo_launch_m3(int tx_size, const RdoArgs& a, hipStream_t s);

#ifdef LAVISH_RDO_KERNELS
namespace {

template <int W, int H>
struct RTile {
  static constexpr int MN = W < H ? W : H;
  static constexpr int P = 64 / MN;
  static constexpr int CPT = W / MN;
  static constexpr int KW = W > 32 ? 32 : W;
  static constexpr int KH = H > 32 ? 32 : H;
  static constexpr int NC = KW * KH;                 // coefficients kept per block
  static constexpr int RPT = (P * KH + 63) / 64;     // kept rows per lane
  static constexpr int T1S = W + 1;
  static constexpr int T1 = P * KH * T1S;
  static constexpr int T2 = P * NC;
};

__device__ __forceinline__ int get_msb(uint32_t n) { return 31 - __builtin_clz(n); }

// Waves per tile of the split form of the TX-domain decision (mode 1): the
// types of a block are split by vertical 1-D kind (one column pass each)
// over up to this many waves of one workgroup, which then pick each block's
// winner across waves (tx_search.c:2246's first type of strictly lowest
// cost, in search order).  The sizes' valid types give at most 4 kinds
// (<= 16 points), 2 (32 points: DCT_DCT, IDTX) or 1 (64 points: DCT_DCT).
// A launch takes the split form only when its grid would leave the SIMDs
// short of waves (small rectangles: the C5 shard's rows and tail segments),
// where a wave's lifetime -- every type of its blocks in sequence -- is the
// kernel's duration; a full frame has waves enough and keeps one wave per
// tile (measured: the split form is slower there, C4 0.81 -> 1.08 ms).
template <int W, int H, int MODE, bool SPLIT>
constexpr int rdo_nvmax() {
  if (!SPLIT || MODE != 1) return 1;
  constexpr int M = W > H ? W : H;
  return M >= 64 ? 1 : (M == 32 ? 2 : 4);
}

// Per-tile LDS of the pixel-domain mode (MODE 2): the prediction pixels, the
// inverse transform's transposition buffer, and per-block sums.
template <int W, int H>
struct PxLds {
  static constexpr int P = RTile<W, H>::P;
  static constexpr int T1S = W + 1;
  uint16_t pred[P * H * W];
  int32_t tx[P * H * T1S];
  int64_t bsse[P];  // block_sse (rounded, x16)
  uint64_t psse[P]; // this type's sum of (src - recon)^2
};

// The LDS of one workgroup of rdo_kernel<W, H, MODE, ., NVM waves> as one
// carved buffer (byte offsets), so a kernel running several sizes
// (rdo_small_kernel) can overlay them: the column-pass output per wave, the
// MODE 0 per-type coefficients, the per-wave winners, the MODE 2 pixel
// state, and the per-block bookkeeping of rdo_types.
constexpr int lds_align(int v, int a) { return (v + a - 1) / a * a; }
// The mode-1 decision of the 32-point sizes keeps the tile's residual in LDS
// (int16: any residual of bit depth <= 12) rather than in a lane's 32 VGPRs,
// which stayed live through every type's row pass (two vertical kinds, DCT
// and IDTX, so the second column pass needs it after the first row pass):
// the 32x32 kernel spilled at its 2-wave register budget.
// Measured slower and off (LAVISH_RDO_RES_LDS=1 builds it): spill-free
// (32x32: 256 VGPRs with 24 spilled -> 227, none) but its 27 KB of LDS fits
// 6 workgroups per CU instead of 7, 61 -> 73 us for the 4K frame's 32x32
// leg (profiles/r06_ab_same_box.txt).
#ifndef LAVISH_RDO_RES_LDS
#define LAVISH_RDO_RES_LDS 0
#endif
template <int W, int H, int MODE>
constexpr bool rdo_res_lds() {
  return LAVISH_RDO_RES_LDS && MODE == 1 && W != 64 && H != 64 && (W == 32 || H == 32);
}

template <int W, int H, int MODE, int NVM>
struct RdoLds {
  using T = RTile<W, H>;
  static constexpr int t1 = 0;
  static constexpr int t2 = lds_align(t1 + 4 * NVM * T::T1, 16);
  static constexpr int tb = lds_align(t2 + 4 * (MODE == 0 ? T::T2 : 4), 16);
  static constexpr int px = lds_align(tb + 4 * (MODE >= 1 ? NVM * T::T2 : 4), 16);
  static constexpr int rank = lds_align(px + (MODE == 2 ? (int)sizeof(PxLds<W, H>) : 0), 16);
  static constexpr int ok = lds_align(rank + 16 * T::P, 4);
  static constexpr int cc = lds_align(ok + 2 * T::P, 16);
  static constexpr int dead = lds_align(cc + 4 * (MODE == 3 ? cc::kTabCells : 1), 4);
  static constexpr int win = lds_align(dead + T::P, 4);
  static constexpr int brd = lds_align(win + T::P, 8);
  static constexpr int brk = lds_align(brd + 8 * NVM * T::P, 4);
  static constexpr int scan = lds_align(brk + NVM * T::P, 16);  // int16 [3][KH][KW]
  // the 32-point sizes' residual (int16 [CPT][H][64 lanes], rdo_res_lds)
  static constexpr int rs = lds_align(scan + 2 * 3 * T::NC, 16);
  static constexpr int bytes =
      lds_align(rs + (rdo_res_lds<W, H, MODE>() ? 2 * T::CPT * H * 64 : 0), 16);
};

// dist_block_tx_domain's finish of a block sum of squares
// (tx_search.c:1077-1116): av1_highbd_block_error's rounding by 2 (bd - 8)
// bits, then the TX-domain shift (MAX_TX_SCALE - tx_scale) * 2
template <int LS>
__device__ __forceinline__ int64_t tx_dist(int64_t v, int bd) {
  const int sh = 2 * (bd - 8);
  if (sh > 0) v = (v + ((int64_t)1 << (sh - 1))) >> sh;
  constexpr int dshift = (1 - LS) * 2;
  if constexpr (dshift >= 0) return v >> dshift;
  else return v << -dshift;
}

template <int W, int H, int MODE, bool FAST, int QK, bool HBD, int BDI, int NVM>
__device__ __forceinline__ void rdo_types(const RdoArgs& a, const int32_t (&res)[RTile<W, H>::CPT][H],
                                          int32_t* t1, int32_t* t2, int32_t* tb0, PxLds<W, H>* px,
                                          int lane, int blk0, int nvalid, int wave, int nv,
                                          char* lds) {
  using LY = RdoLds<W, H, MODE, NVM>;
  using C = TxCfg<W, H>;
  using T = RTile<W, H>;
  using B = Bd<BDI>;
  constexpr int NC = T::NC, KW = T::KW, KH = T::KH, T1S = T::T1S;
  constexpr int LS = C::log_scale;
  constexpr bool DEC = MODE >= 1;  // decision modes (1: TX-domain, 2: pixel-domain distortion)
  constexpr bool RATE = MODE == 3;  // TX-domain distortion, coefficient rate
  int32_t* const tb = tb0 + wave * T::T2;  // this wave's winners' coefficients
  // per (row-pass slot k) running best of the block that slot belongs to
  int64_t best_rd[T::RPT], best_dist[T::RPT], best_sse[T::RPT];
  int best_type[T::RPT], best_eob[T::RPT], best_rate[T::RPT], best_satd[T::RPT];
#pragma unroll
  for (int k = 0; k < T::RPT; ++k) {
    best_rd[k] = INT64_MAX;
    best_dist[k] = best_sse[k] = 0;
    best_type[k] = best_eob[k] = best_rate[k] = best_satd[k] = 0;
  }
  // per block (LDS, read at each decision): the allowed types that also
  // appear in the block's search order, and each type's position in that
  // order; identity without per-block data.  A zero mask means DCT_DCT only
  // (get_tx_mask's rule, tx_search.c:1885-1888).
  uint8_t(*const s_rank)[16] = reinterpret_cast<uint8_t(*)[16]>(lds + LY::rank);
  uint16_t* const s_ok = reinterpret_cast<uint16_t*>(lds + LY::ok);
  // the three scan kinds' inverse scans in lane-row order, staged once per
  // tile: a lane's KW positions of kept row r are one contiguous LDS read
  // per type (global loads per coefficient had been VMEM requests and
  // waits in the middle of the quantizer)
  int16_t* const s_scan = reinterpret_cast<int16_t*>(lds + LY::scan);
  {
    constexpr int NV4 = 3 * NC / 8;  // 16-byte chunks (NC >= 16)
    const int tid = NVM > 1 ? (int)threadIdx.x : lane;
    const int nth = NVM > 1 ? 64 * NVM : 64;
    for (int i = tid; i < NV4; i += nth)
      reinterpret_cast<v4i*>(s_scan)[i] = reinterpret_cast<const v4i*>(a.scan_rows)[i];
    if constexpr (!DEC) wave_sync();  // (DEC: the barrier below covers it)
  }
  if constexpr (DEC) {
    if ((NVM > 1 ? (int)threadIdx.x : lane) < T::P) {  // (wave 0 for the workgroup)
      uint32_t ok = 0xFFFFu;
      if (lane < nvalid) {
        const int blk = blk0 + lane;
        if (a.block_mask) {
          const uint32_t m = a.block_mask[blk];
          ok = m ? m : 1u;
        }
        if (a.block_map) {
          uint32_t present = 0;
          for (int i = 0; i < 16; ++i) s_rank[lane][i] = 16;
          for (int i = 0; i < 16; ++i) {
            const int t = a.block_map[(size_t)blk * 16 + i];
            if (t < 16 && !((present >> t) & 1)) {
              present |= 1u << t;
              s_rank[lane][t] = (uint8_t)i;
            }
          }
          ok &= present;
        } else {
          for (int i = 0; i < 16; ++i) s_rank[lane][i] = (uint8_t)i;
        }
      }
      s_ok[lane] = (uint16_t)ok;
    }
    if constexpr (NVM > 1) __syncthreads();
    else wave_sync();
  }
  // MODE 3: the cost tables
  int32_t* const s_cc = reinterpret_cast<int32_t*>(lds + LY::cc);
  if constexpr (RATE) {  // (mode 3: one wave per tile)
    for (int i = lane; i < cc::kCostCells; i += 64) s_cc[i] = a.cc_cost[i];
    if (lane < cc::kEobCells) s_cc[cc::kCostCells + lane] = a.cc_eob[lane];
    wave_sync();
  }

  // MODE 1, FAST: highbd quantize_fp with uniform per-(dc, ac) constants
  // (quant_one / dequant_one restated in the cheap instruction classes; see
  // coef_fast): rounding, quant << 16, the pass threshold
  // ceil(dequant / 2^(1 + LS)) - 1, dequant
  int qf_rnd[2], qf_thr1[2], qf_deq[2];
  uint32_t qf_qsh[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    qf_rnd[i] = (a.qp.round[i] + ((1 << LS) >> 1)) >> LS;
    qf_qsh[i] = (uint32_t)(uint16_t)a.qp.quant[i] << 16;
    qf_deq[i] = a.qp.dequant[i];
    qf_thr1[i] = ((qf_deq[i] + (1 << (1 + LS)) - 1) >> (1 + LS)) - 1;
  }

  // the 64-point sizes have one candidate type (EXT_TX_SET_DCTONLY,
  // tx_type_valid): with a constant trip count the residual columns die at
  // the column pass instead of staying live through every row pass
  constexpr bool ONE_TYPE = W == 64 || H == 64;
  const int ntypes = ONE_TYPE ? 1 : a.ntypes;
  int grp = -1;  // vertical-kind group of order[oi]; group g runs on wave g % nv
  for (int oi = 0; oi < ntypes; ++oi) {
    if constexpr (NVM > 1) {
      grp += __builtin_amdgcn_readfirstlane(a.newcol[oi]);
      if (grp % nv != wave) continue;
    }
    const int ti = __builtin_amdgcn_readfirstlane(a.order[oi]);
    const int t = __builtin_amdgcn_readfirstlane(a.types[ti]);
    const int vt = (kVtxPacked >> (2 * t)) & 3, ht = (kHtxPacked >> (2 * t)) & 3;
    const int kc = vt == 3 ? 2 : (vt == 0 ? 0 : 1);
    const int kr = ht == 3 ? 2 : (ht == 0 ? 0 : 1);
    const bool ud = vt == 2;
    const bool lr = ht == 2;  // FLIPADST rows: the column results read right to left
    const int skind = __builtin_amdgcn_readfirstlane(a.scan_kind[ti]);
    const int16_t* const srow = s_scan + skind * NC;

    // ---- columns (av1_fwd_txfm2d.c:88-106), once per vertical kind; only
    // rows < KH are kept ----
    if (__builtin_amdgcn_readfirstlane(a.newcol[oi])) {
#pragma unroll
      for (int k = 0; k < T::CPT; ++k) {
        const int j = k * 64 + lane;
        const int b = j / W, c = j % W;
        int32_t in[H], out[H];
        auto col_in = [&](int r, int32_t x) {
          if constexpr (FAST) in[r] = x * (1 << C::s0);
          else in[r] = round_shift_1<-C::s0>(x);
        };
        if constexpr (rdo_res_lds<W, H, MODE>()) {
          const int16_t* const rl = reinterpret_cast<const int16_t*>(lds + LY::rs) + k * H * 64 + lane;
#pragma unroll
          for (int r = 0; r < H; ++r) col_in(r, rl[(ud ? H - 1 - r : r) * 64]);
        } else if (ud) {  // FLIPADST columns: rows bottom to top (a uniform branch:
                          // the select per row had compiled to VGPR-indexed moves)
#pragma unroll
          for (int r = 0; r < H; ++r) col_in(r, res[k][H - 1 - r]);
        } else {
#pragma unroll
          for (int r = 0; r < H; ++r) col_in(r, res[k][r]);
        }
        fwd_1d<H, C::cos_bit_col, FAST>(kc, in, out);
#pragma unroll
        for (int r = 0; r < KH; ++r) t1[(b * KH + r) * T1S + c] = round_shift_1<-C::s1>(out[r]);
      }
      wave_sync();
    }

    // ---- kept rows + quantization + per-block statistics ----
    int st_last[T::RPT], st_rate[T::RPT], st_satd[T::RPT];
    int64_t st_dist[T::RPT], st_sse[T::RPT];
    int32_t st_q[DEC ? T::RPT : 1][DEC ? KW : 1];
#pragma unroll
    for (int k = 0; k < T::RPT; ++k) {
      const int j = k * 64 + lane;
      const int b = j / KH, r = j % KH;
      const bool live = b < T::P;
      const int bb = live ? b : 0;
      int32_t in[W], out[W];
      const int32_t* row = t1 + (bb * KH + r) * T1S;
      if (lr) {
#pragma unroll
        for (int c = 0; c < W; ++c) in[c] = row[W - 1 - c];
      } else {
#pragma unroll
        for (int c = 0; c < W; ++c) in[c] = row[c];
      }
      fwd_1d<W, C::cos_bit_row, FAST>(kr, in, out);
      int32_t q[KW];
      int last = 0, satd = 0, rall = 0;
      int64_t err = 0, sse = 0;
      const size_t obase = ((size_t)ti * a.nblocks + blk0 + bb) * NC;
      // the type's inverse scan of this lane's row (LDS, lane-row order:
      // the KW positions contiguous)
      const int16_t* const isc = srow + r * KW;
      // (the rows of 32-point sizes keep the generic form: 32 unrolled
      // coefficients of this one spill at the 32x32 kernel's 2-wave budget)
      constexpr bool CHEAP = MODE == 1 && FAST && KW <= 16;
      if constexpr (CHEAP) {
        // quantize_fp (highbd, av1_quantize.c:174-194) + dequantisation +
        // block error / sse / SATD / eob / rate_estimator terms on the
        // certified range (|v| < 2^19, tools/range_analysis.py), in the
        // VALU's cheap classes (tools/microbench/valu_rates.hip: add / sub /
        // xor / and / ashr issue in ~2 cycles, multiplies, max, cndmask,
        // 64-bit ops and DPP in ~4): with a = |v|,
        //   pass  <=> a << (1 + LS) >= dequant <=> a > thr1 (uniform): a mask
        //   |q|   = ((a + rnd) * quant) >> (16 - LS) = mulhi((a + rnd) << LS,
        //           quant << 16) (exact: the product stays below 2^64)
        //   |dq|  = (|q| * dequant) >> LS (24-bit multiply)
        //   v - dq = sign(v) (a - |dq|): err += (a - |dq|)^2, sse += a^2
        //   eob   = max over nonzero |q| of iscan + 1, nonzero = (|q| + 2^23 - 1) >> 23
        //   rate_estimator term msb(|q| + 1) + 1 + (|q| > 0) = 32 - clz(|q| + 1) + nz
        // bit-exact with quant_one / dequant_one (the same integers).
        const bool dcl = r == 0;  // column 0 of row 0 is the DC coefficient
        const int rnd0 = dcl ? qf_rnd[0] : qf_rnd[1];
        const uint32_t qsh0 = dcl ? qf_qsh[0] : qf_qsh[1];
        const int thr0 = dcl ? qf_thr1[0] : qf_thr1[1];
        const int deq0 = dcl ? qf_deq[0] : qf_deq[1];
#pragma unroll
        for (int c = 0; c < KW; ++c) {
          int32_t v = round_shift_1<-C::s2>(out[c]);
          if constexpr (C::rect2) v = rshift64((int64_t)v * 5793, 12);
          const int rnd = c ? qf_rnd[1] : rnd0;
          const uint32_t qsh = c ? qf_qsh[1] : qsh0;
          const int thr1 = c ? qf_thr1[1] : thr0;
          const int deq = c ? qf_deq[1] : deq0;
          const int32_t sgn = v >> 31;
          const int32_t av = (v ^ sgn) - sgn;
          const int32_t pass = (thr1 - av) >> 31;  // -1 where the coefficient is kept
          const int32_t qa = (int32_t)__umulhi((uint32_t)(av + rnd) << LS, qsh) & pass;
          const int32_t dqa = mul_i24(qa, deq) >> LS;
          const int32_t e = av - dqa;
          err += (int64_t)e * e;
          sse += (int64_t)av * av;
          satd += av;
          const int32_t nz = (qa + 0x7FFFFF) >> 23;
          last = max(last, ((int)isc[c] + 1) & -nz);
          rall += 32 - __builtin_clz((uint32_t)qa + 1u) + nz;
          q[c] = (qa ^ sgn) - sgn;
        }
      } else {
#pragma unroll
      for (int c = 0; c < KW; ++c) {
        int32_t v = round_shift_1<-C::s2>(out[c]);
        if constexpr (C::rect2) v = rshift64((int64_t)v * 5793, 12);
        const int rc = c * KH + r;
        const bool ac = c != 0 || r != 0;
        if constexpr (MODE == 0 && QK == LAVISH_QUANT_NONE) {
          q[c] = 0;
          if (live && bb < nvalid) a.coeff[obase + rc] = v;
        } else {
          if constexpr (MODE == 0) {
            if (a.coeff != nullptr && live && bb < nvalid) a.coeff[obase + rc] = v;
          }
          q[c] = quant_one<LS, QK, HBD, FAST>(v, ac, a.qp);
        }
        if constexpr (DEC) {
          const int32_t dq = dequant_one<LS, FAST>(q[c], ac, a.qp);
          if constexpr (FAST) {
            // the certified range: |v| < 2^19 (tools/range_analysis.py
            // max|coeff|), |dq| <= |v| + dequant (int16), so v - dq and v
            // fit 24 signed bits and each square is one v_mul_i32_i24 +
            // v_mul_hi_i32_i24 pair (the int64 forms were three quarter-rate
            // 64-bit multiplies per coefficient)
            const int32_t d = v - dq;
            err += (int64_t)sext24(d) * (int64_t)sext24(d);
            sse += (int64_t)sext24(v) * (int64_t)sext24(v);
          } else {
            const int64_t d = (int64_t)v - dq;
            err += d * d;
            sse += (int64_t)v * v;
          }
          satd += abs(v);
        }
        if constexpr (MODE == 0) {
          if (live) t2[bb * NC + rc] = q[c];
        }
        last = q[c] != 0 ? max(last, isc[c] + 1) : last;
      }
      }
      last = lane_max<KH>(last);
      if constexpr (MODE == 0) {
        if (r == 0 && live && bb < nvalid && a.eob != nullptr)
          a.eob[(size_t)ti * a.nblocks + blk0 + bb] = (uint16_t)last;
      } else {
        int rate = 0;
        if constexpr (RATE) {
          // av1_cost_coeffs_txb (txb_rdopt.c:599-624) on this type's
          // quantized block.  Lane = row r of its block, so the |level| map
          // neighbours of get_nz_mag / get_br_ctx are this lane's own
          // columns c+1.. and the same columns of rows r+1.. (lanes below):
          // levels clipped to 15 as nibbles, 8 per word, shifted down the
          // wave a word at a time; rows past the block read as the zero pad.
          constexpr int NW = (KW + 7) / 8;
          const int cls = cc::tx_class(t);
          const int nrow = cls == 2 ? 4 : 2;  // rows below that a context reads
          uint32_t pk[5][NW];
#pragma unroll
          for (int w = 0; w < NW; ++w) pk[0][w] = 0u;
#pragma unroll
          for (int c = 0; c < KW; ++c)
            pk[0][c >> 3] |= (uint32_t)min(abs(q[c]), 15) << (4 * (c & 7));
#pragma unroll
          for (int d = 1; d <= 4; ++d) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
              const uint32_t x = d <= nrow ? (uint32_t)__shfl_down((int)pk[0][w], d) : 0u;
              pk[d][w] = r + d < KH ? x : 0u;
            }
          }
          auto nib = [&](int d, int c) -> int {
            return c < KW ? (int)((pk[d][c >> 3] >> (4 * (c & 7))) & 15u) : 0;
          };
          // get_nz_mag for 8 positions per word at once (SWAR on the
          // nibbles): every neighbour clipped to 3 -- x & 3, or 3 where bit
          // 2 or 3 is set -- then the class's five neighbours, each a
          // nibble shift of a row word, summed without carries (<= 15)
          uint32_t m3[5][NW];
#pragma unroll
          for (int d = 0; d < 5; ++d)
#pragma unroll
            for (int w = 0; w < NW; ++w) {
              const uint32_t x = pk[d][w];
              const uint32_t f = ((x >> 2) | (x >> 3)) & 0x11111111u;
              m3[d][w] = (x & 0x33333333u) | f | (f << 1);
            }
          auto sh = [&](int d, int w, int k) -> uint32_t {  // nibble c + k of row d, word w
            return (m3[d][w] >> (4 * k)) | (w + 1 < NW ? m3[d][w + 1] << (32 - 4 * k) : 0u);
          };
          uint32_t nzs[NW];
#pragma unroll
          for (int w = 0; w < NW; ++w) {
            const uint32_t base = sh(0, w, 1) + m3[1][w];
            nzs[w] = cls == 0 ? base + sh(1, w, 1) + sh(0, w, 2) + m3[2][w]
                   : cls == 1 ? base + sh(0, w, 2) + sh(0, w, 3) + sh(0, w, 4)
                              : base + m3[2][w] + m3[3][w] + m3[4][w];
          }
          const bool has_ctx = a.txb_ctx != nullptr && live && bb < nvalid;
          const LavishTxbCtx tc = has_ctx ? a.txb_ctx[blk0 + bb] : LavishTxbCtx{0, 0};
#pragma unroll
          for (int c = 0; c < KW; ++c) {
            const int rc = c * KH + r;
            const int i = isc[c];
            if (i < last) {
              const int nzmag = (int)((nzs[c >> 3] >> (4 * (c & 7))) & 15u);
              // get_br_ctx's raw sum, needed only above level 2
              int brmag = 0;
              if (abs(q[c]) > 2)
                brmag = nib(0, c + 1) + nib(1, c) +
                        (cls == 0 ? nib(1, c + 1) : cls == 1 ? nib(0, c + 2) : nib(2, c));
              rate += cc::coeff_term_mag(s_cc, cls, a.nz_wlt, a.nz_wgt, NC, rc, c, r, i, last,
                                         q[c], tc.dc_sign_ctx, nzmag, brmag);
            }
          }
          rate = lane_sum<KH>(rate);
          rate = cc::txb_rate(s_cc, cls, tc.txb_skip_ctx, last, a.tx_type_cost[t], rate);
        } else if (CHEAP && skind == 0) {
          // rate_estimator over the DCT_DCT scan below eob: for a type of the
          // default scan (the 2-D classes) eob comes from that same scan, so
          // every position at or past it is zero and costs 1 -- the sum is
          // the whole block's minus (n - eob), no per-position test
          rate = lane_sum<KH>(rall) - (NC - last);
          rate = (rate + 1) << 9;  // AV1_PROB_COST_SHIFT
        } else {
          // rate_estimator: positions of the DCT_DCT scan below eob
          const int16_t* const dct = s_scan + r * KW;
#pragma unroll
          for (int c = 0; c < KW; ++c) {
            const uint32_t al = (uint32_t)abs(q[c]);
            if (dct[c] < last) rate += get_msb(al + 1) + 1 + (al > 0);
          }
          rate = lane_sum<KH>(rate);
          rate = (rate + 1) << 9;  // AV1_PROB_COST_SHIFT
        }
        // only the block error enters the cost: the SATD and the sse are
        // record fields of the winner, so each lane keeps its unreduced
        // partial sums of them and they are reduced once, after the type
        // loop (every lane of a block takes the same winner)
        err = lane_sum64<KH>(err);
        st_dist[k] = tx_dist<LS>(err, a.bd);
        st_sse[k] = sse;
        st_last[k] = last;
        st_rate[k] = rate;
        st_satd[k] = satd;
#pragma unroll
        for (int c = 0; c < KW; ++c) st_q[k][c] = q[c];
      }
      if constexpr (MODE == 2) {
        // inverse rows (inv_txfm2d_add_c "Rows") straight from this lane's
        // quantized row: dequantize, x NewInvSqrt2 for 2:1, clamp, 1-D, shift
        int32_t vin[W], vout[W];
#pragma unroll
        for (int c = 0; c < W; ++c) {
          int32_t v = dequant_one<LS, FAST>(q[c], c != 0 || r != 0, a.qp);
          if constexpr (C::rect2) v = rshift64((int64_t)v * 2896, 12);
          vin[c] = clamp_bits<B::clamp_in_row>(v);
        }
        inv_1d<W, 12, B::rng_row>(kr, vin, vout);
        if (live) {
#pragma unroll
          for (int c = 0; c < W; ++c) px->tx[(bb * H + r) * T1S + c] = rshift_r(vout[c], -C::is0);
        }
      }
    }

    if constexpr (MODE == 2) {
      wave_sync();
      // ---- inverse columns + reconstruction + pixel SSE against src ----
      constexpr int maxv = (1 << B::bd) - 1;
#pragma unroll
      for (int k = 0; k < T::CPT; ++k) {
        const int j = k * 64 + lane;
        const int b = j / W, c = j % W;
        const int cc = lr ? W - 1 - c : c;
        int32_t in[H], out[H];
#pragma unroll
        for (int r = 0; r < H; ++r)
          in[r] = clamp_bits<B::clamp_in_col>(px->tx[(b * H + r) * T1S + cc]);
        inv_1d<H, 12, B::rng_col>(kc, in, out);
        uint64_t ps = 0;
#pragma unroll
        for (int r = 0; r < H; ++r) {
          const int p = px->pred[(b * H + r) * W + c];
          const int v = p + rshift_r(ud ? out[H - 1 - r] : out[r], -C::is1);
          const int rec = v < 0 ? 0 : (v > maxv ? maxv : v);
          const int d = p + res[k][r] - rec;  // src - recon
          ps += (uint64_t)(d * d);
        }
        ps = (uint64_t)lane_sum64<W>((int64_t)ps);
        if (c == 0) px->psse[b] = ps;
      }
      wave_sync();
    }

    if constexpr (DEC) {
      // ---- distortion, RDCOST and the running best per block ----
#pragma unroll
      for (int k = 0; k < T::RPT; ++k) {
        const int j = k * 64 + lane;
        const int b = j / KH, r = j % KH;
        const bool live = b < T::P;
        const int bb = live ? b : 0;
        int64_t dist = st_dist[k], dsse = st_sse[k];
        if constexpr (MODE == 2) {
          // search_tx_type with pixel-domain distortion (tx_search.c:2187-2231);
          // sizes here are <= 32x32, never TX_64X64
          const int64_t bsse = px->bsse[bb];
          if (st_last[k] == 0) {
            dist = bsse;
          } else {
            const int sh = 2 * (a.bd - 8);
            uint64_t ps = px->psse[bb];
            if (sh > 0) ps = (ps + ((uint64_t)1 << (sh - 1))) >> sh;
            // 16 * pixel_dist(): an unsigned 32-bit product
            const int64_t pxd = (int64_t)(uint32_t)(16u * (uint32_t)ps);
            const bool high = bsse >= (int64_t)128 * 128 * W * H;
            dist = (high && pxd < dist) ? dist : pxd;
          }
          dsse = bsse;
        }
        const int64_t rd = (((int64_t)st_rate[k] * a.rdmult + 256) >> 9) + dist * 128;
        // the reference keeps the first type of strictly smallest cost in
        // its search order (txk_map; ascending without one); types are
        // visited here grouped by vertical kind, so equal costs resolve by
        // that order's rank
        if (((s_ok[bb] >> t) & 1) &&
            (rd < best_rd[k] ||
             (rd == best_rd[k] && s_rank[bb][t] < s_rank[bb][best_type[k]]))) {
          best_rd[k] = rd;
          best_dist[k] = dist;
          best_sse[k] = dsse;
          best_type[k] = t;
          best_eob[k] = st_last[k];
          best_rate[k] = st_rate[k];
          best_satd[k] = st_satd[k];
#pragma unroll
          for (int c = 0; c < KW; ++c)
            if (live) tb[bb * NC + c * KH + r] = st_q[k][c];
        }
      }
    }
    wave_sync();

    if constexpr (MODE == 0) {
      // coalesced copy-out of this type's qcoeff / dqcoeff
      if (a.qcoeff != nullptr) {
        const int total = nvalid * NC;
        const size_t gbase = ((size_t)ti * a.nblocks + blk0) * NC;
        for (int i = lane * 4; i < total; i += 64 * 4) {
          const v4i q4 = *reinterpret_cast<const v4i*>(&t2[i]);
          __builtin_nontemporal_store(q4, reinterpret_cast<v4i*>(&a.qcoeff[gbase + i]));
          if (a.dqcoeff != nullptr) {
            const int rc0 = i % NC;
            v4i d4;
            d4.x = dequant_one<LS, FAST>(q4.x, rc0 != 0, a.qp);
            d4.y = dequant_one<LS, FAST>(q4.y, 1, a.qp);
            d4.z = dequant_one<LS, FAST>(q4.z, 1, a.qp);
            d4.w = dequant_one<LS, FAST>(q4.w, 1, a.qp);
            __builtin_nontemporal_store(d4, reinterpret_cast<v4i*>(&a.dqcoeff[gbase + i]));
          }
        }
      }
      wave_sync();
    }
  }

  if constexpr (DEC) {
    // the winners' SATD and (TX-domain modes) sse, reduced once (see the
    // type loop)
#pragma unroll
    for (int k = 0; k < T::RPT; ++k) {
      best_satd[k] = lane_sum<KH>(best_satd[k]);
      if constexpr (MODE != 2) best_sse[k] = tx_dist<LS>(lane_sum64<KH>(best_sse[k]), a.bd);
    }
  }
  if constexpr (DEC && NVM == 1) {
    // decision records (one lane per block) and the winner's coefficients.
    // A block none of whose allowed types is in the evaluated set (possible
    // only with caller masks) has no candidate: record best_type
    // TX_TYPE_INVALID (255), eob 0, rdcost INT64_MAX, zero coefficients.
    uint8_t* const s_dead = reinterpret_cast<uint8_t*>(lds + LY::dead);
#pragma unroll
    for (int k = 0; k < T::RPT; ++k) {
      const int j = k * 64 + lane;
      const int b = j / KH, r = j % KH;
      if (b < T::P && b < nvalid && r == 0) {
        const bool dead = best_rd[k] == INT64_MAX;
        LavishRdoBlock o;
        o.best_type = dead ? 255 : best_type[k];
        o.eob = best_eob[k];
        o.rate = best_rate[k];
        o.satd = best_satd[k];
        o.dist = best_dist[k];
        o.sse = best_sse[k];
        o.rdcost = best_rd[k];
        a.out[blk0 + b] = o;
        s_dead[b] = dead;
      }
    }
    wave_sync();
    const int total = nvalid * NC;
    const size_t gbase = (size_t)blk0 * NC;
    for (int i = lane * 4; i < total; i += 64 * 4) {
      v4i q4 = *reinterpret_cast<const v4i*>(&tb[i]);
      if (s_dead[i / NC]) q4 = v4i{0, 0, 0, 0};
      __builtin_nontemporal_store(q4, reinterpret_cast<v4i*>(&a.qcoeff[gbase + i]));
      const int rc0 = i % NC;
      v4i d4;
      d4.x = dequant_one<LS, FAST>(q4.x, rc0 != 0, a.qp);
      d4.y = dequant_one<LS, FAST>(q4.y, 1, a.qp);
      d4.z = dequant_one<LS, FAST>(q4.z, 1, a.qp);
      d4.w = dequant_one<LS, FAST>(q4.w, 1, a.qp);
      __builtin_nontemporal_store(d4, reinterpret_cast<v4i*>(&a.dqcoeff[gbase + i]));
    }
  }
  if constexpr (DEC && NVM > 1) {
    // decision records (one lane per block) and the winner's coefficients.
    // A block none of whose allowed types is in the evaluated set (possible
    // only with caller masks) has no candidate: record best_type
    // TX_TYPE_INVALID (255), eob 0, rdcost INT64_MAX, zero coefficients.
    // With the types over nv waves, each block's winner is the lowest
    // (rdcost, search rank) over the waves' bests: the sequential scan's
    // first type of strictly lowest cost, as every rank is distinct.
    // winning wave per block (255: none), each wave's best cost and rank
    uint8_t* const s_win = reinterpret_cast<uint8_t*>(lds + LY::win);
    int64_t(*const s_brd)[T::P] = reinterpret_cast<int64_t(*)[T::P]>(lds + LY::brd);
    uint8_t(*const s_brk)[T::P] = reinterpret_cast<uint8_t(*)[T::P]>(lds + LY::brk);
    {
#pragma unroll
      for (int k = 0; k < T::RPT; ++k) {
        const int j = k * 64 + lane;
        const int b = j / KH, r = j % KH;
        if (b < T::P && r == 0) {
          s_brd[wave][b] = best_rd[k];
          s_brk[wave][b] = best_rd[k] == INT64_MAX ? 255 : s_rank[b][best_type[k]];
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < T::RPT; ++k) {
      const int j = k * 64 + lane;
      const int b = j / KH, r = j % KH;
      if (b < T::P && b < nvalid && r == 0) {
        int win = 0;
        int64_t wrd = best_rd[k];
        {
          int wrk = 256;
          wrd = INT64_MAX;
          for (int q = 0; q < nv; ++q) {
            const int64_t rd = s_brd[q][b];
            const int rk = s_brk[q][b];
            if (rd < wrd || (rd == wrd && rk < wrk)) {
              wrd = rd;
              wrk = rk;
              win = q;
            }
          }
        }
        const bool dead = wrd == INT64_MAX;
        if (win == wave) {  // (a dead block: wave 0 writes its record)
          LavishRdoBlock o;
          o.best_type = dead ? 255 : best_type[k];
          o.eob = best_eob[k];
          o.rate = best_rate[k];
          o.satd = best_satd[k];
          o.dist = best_dist[k];
          o.sse = best_sse[k];
          o.rdcost = best_rd[k];
          a.out[blk0 + b] = o;
          s_win[b] = dead ? 255 : (uint8_t)win;
        }
      }
    }
    __syncthreads();
    const int total = nvalid * NC;
    const size_t gbase = (size_t)blk0 * NC;
    for (int i = (wave * 64 + lane) * 4; i < total; i += nv * 64 * 4) {
      const int w = s_win[i / NC];
      v4i q4 = *reinterpret_cast<const v4i*>(&tb0[(w == 255 ? 0 : w) * T::T2 + i]);
      if (w == 255) q4 = v4i{0, 0, 0, 0};
      __builtin_nontemporal_store(q4, reinterpret_cast<v4i*>(&a.qcoeff[gbase + i]));
      const int rc0 = i % NC;
      v4i d4;
      d4.x = dequant_one<LS, FAST>(q4.x, rc0 != 0, a.qp);
      d4.y = dequant_one<LS, FAST>(q4.y, 1, a.qp);
      d4.z = dequant_one<LS, FAST>(q4.z, 1, a.qp);
      d4.w = dequant_one<LS, FAST>(q4.w, 1, a.qp);
      __builtin_nontemporal_store(d4, reinterpret_cast<v4i*>(&a.dqcoeff[gbase + i]));
    }
  }
}

// one wave = one tile of P blocks; 64-thread workgroups (LDS per tile is up
// to ~20 KB for the 64-point sizes).  MODE 0: per-type coefficients (the
// txq_plane contract), 1: decision with TX-domain distortion, 2: decision
// with pixel-domain distortion (sizes <= 32x32; BDI = bit-depth index), 3:
// mode 1 ranked by the coefficient rate (av1_cost_coeffs_txb) instead of
// rate_estimator.
// Occupancy: a rdo_kernel wave holds a column (or row) of its block per lane
// through each 1-D transform, so the large sizes sit just above a VGPR
// step of the unified 512-register file (32x32 TX-domain: 266 registers =
// 1 wave per SIMD, latency bound at 14% of the VALU peak).  The TX-domain
// decision kernels of the sizes of 512+ coefficients ask for 2 waves per
// SIMD (<= 256 registers), the 16x16 one for 4 (<= 128).
#ifndef LAVISH_RDO_WV16
#define LAVISH_RDO_WV16 4
#endif
#ifndef LAVISH_RDO_WV32
#define LAVISH_RDO_WV32 2
#endif
#ifndef LAVISH_RDO_WV64
#define LAVISH_RDO_WV64 2
#endif
// (The 64-point sizes fit the 2-wave request without spills since their
// type loop has a constant trip count (rdo_types' ONE_TYPE: 256 VGPRs with
// 426 spilled -> 216, none); until round 6 they ran a one-wave-per-SIMD
// build below 2048 tiles -- the 4K frame's 2040 64x64 blocks included -- to
// avoid the spills.)
template <int W, int H, int MODE, bool SPLIT = false>
constexpr int rdo_waves() {
  if (MODE != 1) return 1;
  if (W == 16 && H == 16) return LAVISH_RDO_WV16;
  if (W * H >= 2048) return LAVISH_RDO_WV64;
  return W * H >= 512 ? LAVISH_RDO_WV32 : 1;
}

// one tile (P blocks) of rdo_kernel: tile index `tile`, the workgroup's
// wave `wave` of nv sharing it (NVM > 1), its LDS (RdoLds bytes)
template <int W, int H, int MODE, int BDI, int NVM>
__device__ __forceinline__ void rdo_tile(const RdoArgs& a, int tile, int lane, int wave, int nv,
                                         char* lds) {
  using T = RTile<W, H>;
  using LY = RdoLds<W, H, MODE, NVM>;
  int32_t* const t2 = reinterpret_cast<int32_t*>(lds + LY::t2);
  int32_t* const tb = reinterpret_cast<int32_t*>(lds + LY::tb);
  PxLds<W, H>* px = MODE == 2 ? reinterpret_cast<PxLds<W, H>*>(lds + LY::px) : nullptr;
  int32_t* const t1 = reinterpret_cast<int32_t*>(lds + LY::t1) + wave * T::T1;
  const int blk0 = tile * T::P;
  if (blk0 >= a.nblocks) return;
  const int nvalid = min(T::P, a.nblocks - blk0);

  int32_t res[T::CPT][H];
  int32_t amax = 0;
#pragma unroll
  for (int k = 0; k < T::CPT; ++k) {
    const int j = k * 64 + lane;
    const int b = j / W, c = j % W;
    const int blk = blk0 + b;
    int64_t ss = 0;
    if (b < nvalid) {
      const int by = blk / a.bw, bx = blk - by * a.bw;
      const size_t off = (size_t)by * H * a.stride + (size_t)bx * W + c;
#pragma unroll
      for (int r = 0; r < H; ++r) {
        int32_t v;
        if constexpr (MODE == 0) {
          v = a.res[off + (size_t)r * a.stride];
        } else {
          const int32_t p = a.pred[off + (size_t)r * a.stride];
          v = (int32_t)a.src[off + (size_t)r * a.stride] - p;
          if constexpr (MODE == 2) px->pred[(b * H + r) * W + c] = (uint16_t)p;
        }
        res[k][r] = v;
        if constexpr (rdo_res_lds<W, H, MODE>())
          reinterpret_cast<int16_t*>(lds + LY::rs)[(k * H + r) * 64 + lane] = (int16_t)v;
        amax = max(amax, abs(v));
        ss += (int64_t)v * v;
      }
    } else {
#pragma unroll
      for (int r = 0; r < H; ++r) {
        res[k][r] = 0;
        if constexpr (rdo_res_lds<W, H, MODE>())
          reinterpret_cast<int16_t*>(lds + LY::rs)[(k * H + r) * 64 + lane] = 0;
        if constexpr (MODE == 2) px->pred[(b * H + r) * W + c] = 0;
      }
    }
    if constexpr (MODE == 2) {
      // block_sse (tx_search.c:2079-2094): sum of squares of the residual,
      // highbd-rounded by 2 (bd - 8) bits, x 16
      ss = lane_sum64<W>(ss);
      constexpr int sh = 2 * (Bd<BDI>::bd - 8);
      if constexpr (sh > 0) ss = (ss + ((int64_t)1 << (sh - 1))) >> sh;
      if (c == 0) px->bsse[b] = ss * 16;
    }
  }
  if constexpr (MODE == 2) wave_sync();
  const bool fast = __builtin_amdgcn_ballot_w64(amax > kFastResidualMax) == 0;
  if constexpr (MODE >= 1) {
    if (fast)
      rdo_types<W, H, MODE, true, LAVISH_QUANT_FP, true, BDI, NVM>(a, res, t1, t2, tb, px, lane,
                                                                   blk0, nvalid, wave, nv, lds);
    else
      rdo_types<W, H, MODE, false, LAVISH_QUANT_FP, true, BDI, NVM>(a, res, t1, t2, tb, px, lane,
                                                                    blk0, nvalid, wave, nv, lds);
  } else {
#define LAVISH_RDO_RUN(F, Q, HB) \
  rdo_types<W, H, 0, F, Q, HB, 0, 1>(a, res, t1, t2, tb, px, lane, blk0, nvalid, 0, 1, lds)
    if (a.quant_kind == LAVISH_QUANT_NONE) {
      if (fast) LAVISH_RDO_RUN(true, LAVISH_QUANT_NONE, false);
      else LAVISH_RDO_RUN(false, LAVISH_QUANT_NONE, false);
    } else if (a.quant_kind == LAVISH_QUANT_FP) {
      if (a.highbd) {
        if (fast) LAVISH_RDO_RUN(true, LAVISH_QUANT_FP, true);
        else LAVISH_RDO_RUN(false, LAVISH_QUANT_FP, true);
      } else {
        if (fast) LAVISH_RDO_RUN(true, LAVISH_QUANT_FP, false);
        else LAVISH_RDO_RUN(false, LAVISH_QUANT_FP, false);
      }
    } else {
      if (a.highbd) {
        if (fast) LAVISH_RDO_RUN(true, LAVISH_QUANT_B, true);
        else LAVISH_RDO_RUN(false, LAVISH_QUANT_B, true);
      } else {
        if (fast) LAVISH_RDO_RUN(true, LAVISH_QUANT_B, false);
        else LAVISH_RDO_RUN(false, LAVISH_QUANT_B, false);
      }
    }
#undef LAVISH_RDO_RUN
  }
}

template <int W, int H, int MODE, int BDI, bool SPLIT = false>
__global__ __launch_bounds__(64 * (rdo_nvmax<W, H, MODE, SPLIT>()))
__attribute__((amdgpu_waves_per_eu(rdo_waves<W, H, MODE, SPLIT>())))
void rdo_kernel(RdoArgs a) {
  constexpr int NVM = rdo_nvmax<W, H, MODE, SPLIT>();
  __shared__ __attribute__((aligned(16))) char lds[RdoLds<W, H, MODE, NVM>::bytes];
  // NVM > 1: the workgroup's waves share one tile, each a share of the types
  // (threadIdx.x & 63 for the lane made the compiler spill ~2x more in
  // these register-bound kernels; the mbcnt lane id does not)
  const int lane = NVM > 1 ? __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u))
                           : (int)threadIdx.x;
  const int wave = NVM > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  const int nv = NVM > 1 ? (int)(blockDim.x >> 6) : 1;
  rdo_tile<W, H, MODE, BDI, NVM>(a, blockIdx.x, lane, wave, nv, lds);
}

template <int MODE>
constexpr int rdo_small_lds() {
  constexpr int a = RdoLds<16, 16, MODE, 4>::bytes, b = RdoLds<8, 8, MODE, 4>::bytes,
                c = RdoLds<4, 4, MODE, 4>::bytes;
  return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LAVISH_RDO_WV16)))
void rdo_small_kernel(RdoSmall m) {
  __shared__ __attribute__((aligned(16))) char lds[rdo_small_lds<MODE>()];
  const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x;
  if (b < m.first[1]) rdo_tile<16, 16, MODE, 0, 4>(m.a[0], b - m.first[0], lane, wave, 4, lds);
  else if (b < m.first[2]) rdo_tile<8, 8, MODE, 0, 4>(m.a[1], b - m.first[1], lane, wave, 4, lds);
  else rdo_tile<4, 4, MODE, 0, 4>(m.a[2], b - m.first[2], lane, wave, 4, lds);
}

template <int W, int H, int MODE>
void launch_rdo(const RdoArgs& a, hipStream_t s) {
  const int grid = (a.nblocks + RTile<W, H>::P - 1) / RTile<W, H>::P;
  if (grid == 0) return;
  // split form (mode 1, small grids): one wave per vertical-kind group of
  // the mask, at most NVM
  int groups = 0;
  for (int i = 0; i < a.ntypes; ++i) groups += a.newcol[i];
  constexpr int NVM = rdo_nvmax<W, H, MODE, true>();
  const int nv = groups < NVM ? groups : NVM;
  if constexpr (NVM > 1) {
    if (nv > 1 && grid < kRdoSplitTiles) {
      hipLaunchKernelGGL((rdo_kernel<W, H, MODE, 0, true>), dim3(grid), dim3(64 * nv), 0, s, a);
      LAVISH_CHECK(hipGetLastError());
      return;
    }
  }
  if constexpr (MODE == 2) {
    if (a.bd == 8)
      hipLaunchKernelGGL((rdo_kernel<W, H, 2, 0>), dim3(grid), dim3(64), 0, s, a);
    else if (a.bd == 10)
      hipLaunchKernelGGL((rdo_kernel<W, H, 2, 1>), dim3(grid), dim3(64), 0, s, a);
    else
      hipLaunchKernelGGL((rdo_kernel<W, H, 2, 2>), dim3(grid), dim3(64), 0, s, a);
  } else {
    hipLaunchKernelGGL((rdo_kernel<W, H, MODE, 0>), dim3(grid), dim3(64), 0, s, a);
  }
  LAVISH_CHECK(hipGetLastError());
}

template <int MODE>
int launch_size(int tx_size, const RdoArgs& a, hipStream_t s) {
  if constexpr (MODE <= 1 || MODE == 3) {
    switch (tx_size) {
      case 4: launch_rdo<64, 64, MODE>(a, s); return 0;
      case 11: launch_rdo<32, 64, MODE>(a, s); return 0;
      case 12: launch_rdo<64, 32, MODE>(a, s); return 0;
      case 17: launch_rdo<16, 64, MODE>(a, s); return 0;
      case 18: launch_rdo<64, 16, MODE>(a, s); return 0;
      default: break;
    }
  }
  if constexpr (MODE >= 1) {
    switch (tx_size) {
      case 0: launch_rdo<4, 4, MODE>(a, s); return 0;
      case 1: launch_rdo<8, 8, MODE>(a, s); return 0;
      case 2: launch_rdo<16, 16, MODE>(a, s); return 0;
      case 3: launch_rdo<32, 32, MODE>(a, s); return 0;
      case 5: launch_rdo<4, 8, MODE>(a, s); return 0;
      case 6: launch_rdo<8, 4, MODE>(a, s); return 0;
      case 7: launch_rdo<8, 16, MODE>(a, s); return 0;
      case 8: launch_rdo<16, 8, MODE>(a, s); return 0;
      case 9: launch_rdo<16, 32, MODE>(a, s); return 0;
      case 10: launch_rdo<32, 16, MODE>(a, s); return 0;
      case 13: launch_rdo<4, 16, MODE>(a, s); return 0;
      case 14: launch_rdo<16, 4, MODE>(a, s); return 0;
      case 15: launch_rdo<8, 32, MODE>(a, s); return 0;
      case 16: launch_rdo<32, 8, MODE>(a, s); return 0;
      default: break;
    }
  }
  return -2;
}

}  // namespace
#endif  // LAVISH_RDO_KERNELS

}  // namespace lavish
