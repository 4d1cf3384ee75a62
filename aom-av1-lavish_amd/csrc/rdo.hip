// rdo.hip -- C4: fused per-block TX-type RDO for gfx950, and the 64-point
// forward transform sizes.
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
#include "lavish_internal.h"
#include "quant_dev.h"

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

template <int W, int H, int MODE, bool FAST, int QK, bool HBD, int BDI>
__device__ __forceinline__ void rdo_types(const RdoArgs& a, const int32_t (&res)[RTile<W, H>::CPT][H],
                                          int32_t* t1, int32_t* t2, int32_t* tb, PxLds<W, H>* px,
                                          int lane, int blk0, int nvalid) {
  using C = TxCfg<W, H>;
  using T = RTile<W, H>;
  using B = Bd<BDI>;
  constexpr int NC = T::NC, KW = T::KW, KH = T::KH, T1S = T::T1S;
  constexpr int LS = C::log_scale;
  constexpr bool DEC = MODE >= 1;  // decision modes (1: TX-domain, 2: pixel-domain distortion)
  constexpr bool RATE = MODE == 3;  // TX-domain distortion, coefficient rate
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
  __shared__ uint8_t s_rank[T::P][16];
  __shared__ uint16_t s_ok[T::P];
  if constexpr (DEC) {
    if (lane < T::P) {
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
    wave_sync();
  }
  // MODE 3: the cost tables
  __shared__ int32_t s_cc[RATE ? cc::kTabCells : 1];
  if constexpr (RATE) {
    for (int i = lane; i < cc::kCostCells; i += 64) s_cc[i] = a.cc_cost[i];
    if (lane < cc::kEobCells) s_cc[cc::kCostCells + lane] = a.cc_eob[lane];
    wave_sync();
  }

  for (int oi = 0; oi < a.ntypes; ++oi) {
    const int ti = __builtin_amdgcn_readfirstlane(a.order[oi]);
    const int t = __builtin_amdgcn_readfirstlane(a.types[ti]);
    const int vt = (kVtxPacked >> (2 * t)) & 3, ht = (kHtxPacked >> (2 * t)) & 3;
    const int kc = vt == 3 ? 2 : (vt == 0 ? 0 : 1);
    const int kr = ht == 3 ? 2 : (ht == 0 ? 0 : 1);
    const bool ud = vt == 2;
    const bool lr = ht == 2;  // FLIPADST rows: the column results read right to left
    const int16_t* iscan = a.iscan_type[ti];

    // ---- columns (av1_fwd_txfm2d.c:88-106), once per vertical kind; only
    // rows < KH are kept ----
    if (__builtin_amdgcn_readfirstlane(a.newcol[oi])) {
#pragma unroll
      for (int k = 0; k < T::CPT; ++k) {
        const int j = k * 64 + lane;
        const int b = j / W, c = j % W;
        int32_t in[H], out[H];
#pragma unroll
        for (int r = 0; r < H; ++r) {
          const int32_t x = ud ? res[k][H - 1 - r] : res[k][r];
          if constexpr (FAST) in[r] = x * (1 << C::s0);
          else in[r] = round_shift_1<-C::s0>(x);
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
      int last = 0, satd = 0;
      int64_t err = 0, sse = 0;
      const size_t obase = ((size_t)ti * a.nblocks + blk0 + bb) * NC;
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
          q[c] = quant_one<LS, QK, HBD>(v, ac, a.qp);
        }
        if constexpr (DEC) {
          const int32_t dq = dequant_one<LS>(q[c], ac, a.qp);
          const int64_t d = (int64_t)v - dq;
          err += d * d;
          sse += (int64_t)v * v;
          satd += abs(v);
        }
        if constexpr (MODE == 0) {
          if (live) t2[bb * NC + rc] = q[c];
        }
        last = q[c] != 0 ? max(last, iscan[rc] + 1) : last;
      }
#pragma unroll
      for (int m = 1; m < KH; m <<= 1) last = max(last, __shfl_xor(last, m));
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
            const int i = iscan[rc];
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
#pragma unroll
          for (int m = 1; m < KH; m <<= 1) rate += __shfl_xor(rate, m);
          rate = cc::txb_rate(s_cc, cls, tc.txb_skip_ctx, last, a.tx_type_cost[t], rate);
        } else {
          // rate_estimator: positions of the DCT_DCT scan below eob
#pragma unroll
          for (int c = 0; c < KW; ++c) {
            const int rc = c * KH + r;
            const uint32_t al = (uint32_t)abs(q[c]);
            if (a.iscan_dct[rc] < last) rate += get_msb(al + 1) + 1 + (al > 0);
          }
#pragma unroll
          for (int m = 1; m < KH; m <<= 1) rate += __shfl_xor(rate, m);
          rate = (rate + 1) << 9;  // AV1_PROB_COST_SHIFT
        }
#pragma unroll
        for (int m = 1; m < KH; m <<= 1) {
          satd += __shfl_xor(satd, m);
          err += __shfl_xor(err, m);
          sse += __shfl_xor(sse, m);
        }
        // av1_highbd_block_error rounding, then the TX-domain shift
        const int sh = 2 * (a.bd - 8);
        if (sh > 0) {
          const int64_t rnd = (int64_t)1 << (sh - 1);
          err = (err + rnd) >> sh;
          sse = (sse + rnd) >> sh;
        }
        constexpr int dshift = (1 - LS) * 2;  // (MAX_TX_SCALE - tx_scale) * 2
        if constexpr (dshift >= 0) {
          st_dist[k] = err >> dshift;
          st_sse[k] = sse >> dshift;
        } else {
          st_dist[k] = err << -dshift;
          st_sse[k] = sse << -dshift;
        }
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
          int32_t v = dequant_one<LS>(q[c], c != 0 || r != 0, a.qp);
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
#pragma unroll
        for (int m = 1; m < W; m <<= 1) ps += __shfl_xor(ps, m);
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
            d4.x = dequant_one<LS>(q4.x, rc0 != 0, a.qp);
            d4.y = dequant_one<LS>(q4.y, 1, a.qp);
            d4.z = dequant_one<LS>(q4.z, 1, a.qp);
            d4.w = dequant_one<LS>(q4.w, 1, a.qp);
            __builtin_nontemporal_store(d4, reinterpret_cast<v4i*>(&a.dqcoeff[gbase + i]));
          }
        }
      }
      wave_sync();
    }
  }

  if constexpr (DEC) {
    // decision records (one lane per block) and the winner's coefficients.
    // A block none of whose allowed types is in the evaluated set (possible
    // only with caller masks) has no candidate: record best_type
    // TX_TYPE_INVALID (255), eob 0, rdcost INT64_MAX, zero coefficients.
    __shared__ uint8_t s_dead[T::P];
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
      d4.x = dequant_one<LS>(q4.x, rc0 != 0, a.qp);
      d4.y = dequant_one<LS>(q4.y, 1, a.qp);
      d4.z = dequant_one<LS>(q4.z, 1, a.qp);
      d4.w = dequant_one<LS>(q4.w, 1, a.qp);
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
template <int W, int H, int MODE>
constexpr int rdo_waves() {
  if (MODE != 1) return 1;
  if (W == 16 && H == 16) return LAVISH_RDO_WV16;
  if (W * H >= 2048) return LAVISH_RDO_WV64;
  return W * H >= 512 ? LAVISH_RDO_WV32 : 1;
}

template <int W, int H, int MODE, int BDI>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(rdo_waves<W, H, MODE>())))
void rdo_kernel(RdoArgs a) {
  using T = RTile<W, H>;
  __shared__ int32_t t1[T::T1];
  __shared__ __attribute__((aligned(16))) int32_t t2[MODE == 0 ? T::T2 : 4];
  __shared__ __attribute__((aligned(16))) int32_t tb[MODE >= 1 ? T::T2 : 4];
  __shared__ typename std::conditional<MODE == 2, PxLds<W, H>, int>::type pxs;
  PxLds<W, H>* px = MODE == 2 ? reinterpret_cast<PxLds<W, H>*>(&pxs) : nullptr;

  const int lane = threadIdx.x;
  const int blk0 = blockIdx.x * T::P;
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
        amax = max(amax, abs(v));
        ss += (int64_t)v * v;
      }
    } else {
#pragma unroll
      for (int r = 0; r < H; ++r) {
        res[k][r] = 0;
        if constexpr (MODE == 2) px->pred[(b * H + r) * W + c] = 0;
      }
    }
    if constexpr (MODE == 2) {
      // block_sse (tx_search.c:2079-2094): sum of squares of the residual,
      // highbd-rounded by 2 (bd - 8) bits, x 16
#pragma unroll
      for (int m = 1; m < W; m <<= 1) ss += __shfl_xor(ss, m);
      constexpr int sh = 2 * (Bd<BDI>::bd - 8);
      if constexpr (sh > 0) ss = (ss + ((int64_t)1 << (sh - 1))) >> sh;
      if (c == 0) px->bsse[b] = ss * 16;
    }
  }
  if constexpr (MODE == 2) wave_sync();
  const bool fast = __builtin_amdgcn_ballot_w64(amax > kFastResidualMax) == 0;
  if constexpr (MODE >= 1) {
    if (fast)
      rdo_types<W, H, MODE, true, LAVISH_QUANT_FP, true, BDI>(a, res, t1, t2, tb, px, lane, blk0,
                                                              nvalid);
    else
      rdo_types<W, H, MODE, false, LAVISH_QUANT_FP, true, BDI>(a, res, t1, t2, tb, px, lane, blk0,
                                                               nvalid);
  } else {
#define LAVISH_RDO_RUN(F, Q, HB) \
  rdo_types<W, H, 0, F, Q, HB, 0>(a, res, t1, t2, tb, px, lane, blk0, nvalid)
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

template <int W, int H, int MODE>
void launch_rdo(const RdoArgs& a, hipStream_t s) {
  const int grid = (a.nblocks + RTile<W, H>::P - 1) / RTile<W, H>::P;
  if (grid == 0) return;
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

int fill_types(RdoArgs& a, int tx_size, uint32_t type_mask) {
  a.ntypes = 0;
  for (int t = 0; t < 16; ++t) {
    if (!((type_mask >> t) & 1)) continue;
    if (!tx_type_valid(tx_size, t)) return -5;
    a.iscan_type[a.ntypes] = dev_iscan(tx_size, t);
    a.types[a.ntypes++] = t;
  }
  int n = 0;
  for (int vk = 0; vk < 4; ++vk) {
    bool first = true;
    for (int i = 0; i < a.ntypes; ++i) {
      if (((kVtxPacked >> (2 * a.types[i])) & 3) != (uint32_t)vk) continue;
      a.order[n] = i;
      a.newcol[n++] = first;
      first = false;
    }
  }
  return a.ntypes == 0 ? -5 : 0;
}

QP qp_of(const LavishQuantParams* p) {
  QP q{};
  for (int i = 0; i < 2; ++i) {
    q.zbin[i] = p->zbin[i];
    q.round[i] = p->round[i];
    q.quant[i] = p->quant[i];
    q.quant_shift[i] = p->quant_shift[i];
    q.dequant[i] = p->dequant[i];
  }
  return q;
}

}  // namespace

// lavish_txq_plane for the 64-point sizes (called from txq.hip)
int txq_plane_64(const int16_t* residual, int stride, int width, int height, int tx_size,
                 uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
                 int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff,
                 hipStream_t s) {
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  RdoArgs a{};
  a.res = residual;
  a.stride = stride;
  a.bw = width / W;
  a.nblocks = (width / W) * (height / H);
  const int rc = fill_types(a, tx_size, type_mask);
  if (rc) return rc;
  a.bd = bd;
  a.quant_kind = quant_kind;
  a.highbd = bd > 8;
  if (qp) a.qp = qp_of(qp);
  a.qcoeff = qcoeff;
  a.dqcoeff = dqcoeff;
  a.eob = eob;
  a.coeff = coeff;
  return launch_size<0>(tx_size, a, s);
}

// 64-point sizes with pixel-domain distortion (one candidate type: DCT_DCT):
// the TX-domain decision kernel, then the inverse of its winner into a
// scratch copy of the prediction, the pixel SSE and the reference's
// TX_64X64 / high-energy rules (px64_finish_kernel).
int rdo_plane_px64(RdoArgs& a, int tx_size, int width, int height, hipStream_t s);

int rdo_plane(const uint16_t* src, const uint16_t* pred, int stride, int width, int height,
              int tx_size, uint32_t type_mask, int bd, const LavishQuantParams* qp, int rdmult,
              LavishRdoBlock* out, int32_t* qcoeff, int32_t* dqcoeff, hipStream_t s, int px,
              const uint16_t* block_mask, const uint8_t* block_map, const RateCfg* rate) {
  if (tx_size < 0 || tx_size >= 19) return -1;
  if (qp == nullptr || out == nullptr || qcoeff == nullptr || dqcoeff == nullptr) return -3;
  if (bd != 8 && bd != 10 && bd != 12) return -3;
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  if (width <= 0 || height <= 0 || stride < width) return -4;
  RdoArgs a{};
  a.src = src;
  a.pred = pred;
  a.stride = stride;
  a.bw = width / W;
  a.nblocks = (width / W) * (height / H);
  const int rc = fill_types(a, tx_size, type_mask);
  if (rc) return rc;
  a.bd = bd;
  a.rdmult = rdmult;
  a.qp = qp_of(qp);
  a.iscan_dct = dev_iscan(tx_size, 0);
  a.out = out;
  a.qcoeff = qcoeff;
  a.dqcoeff = dqcoeff;
  a.block_mask = block_mask;
  a.block_map = block_map;
  if (rate != nullptr) {
    if (px) return -7;  // the coefficient rate is built for TX-domain distortion
    if (rate->costs == nullptr) return -3;
    const int txw = W, txh = H;
    const int w = txw > 32 ? 32 : txw, h = txh > 32 ? 32 : txh;
    const int mn = txw < txh ? txw : txh, mx = txw < txh ? txh : txw;
    const int lg_mn = 31 - __builtin_clz(mn), lg_mx = 31 - __builtin_clz(mx);
    const int txs_ctx = (lg_mn - 2 + lg_mx - 2 + 1) >> 1;        // get_txsize_entropy_ctx
    const int eob_multi = 31 - __builtin_clz(w * h) - 4;         // txsize_log2_minus4
    a.cc_cost = &rate->costs->coeff_costs[txs_ctx][0].txb_skip_cost[0][0];
    a.cc_eob = &rate->costs->eob_costs[eob_multi][0].eob_cost[0][0];
    a.txb_ctx = rate->txb_ctx;
    for (int t = 0; t < 16; ++t) a.tx_type_cost[t] = rate->tx_type_costs ? rate->tx_type_costs[t] : 0;
    a.nz_wlt = txw < txh;
    a.nz_wgt = txw > txh;
    return launch_size<3>(tx_size, a, s);
  }
  if (px) {
    if (W > 32 || H > 32) {
      if (block_mask || block_map) return -6;  // single-type path
      return rdo_plane_px64(a, tx_size, width, height, s);
    }
    return launch_size<2>(tx_size, a, s);
  }
  return launch_size<1>(tx_size, a, s);
}

// ---------------------------------------------------------------------------
// frame level: every candidate TX size of a frame, the per-superblock TX-size
// decision and the reconstruction
// ---------------------------------------------------------------------------
int rdo_frame(const uint16_t* src, const uint16_t* pred, int stride, int width, int height,
              uint32_t size_mask, const uint32_t* type_masks, int bd,
              const LavishQuantParams* qp, int rdmult, LavishRdoBlock* const* out,
              int32_t* const* qcoeff, int32_t* const* dqcoeff, hipStream_t caller, int px = 0) {
  int order[19], n = 0;
  for (int s = 0; s < 19; ++s)
    if ((size_mask >> s) & 1) order[n++] = s;
  // most work first, dealt round-robin over the internal streams (measured
  // against least work first, so the few-wave, latency-bound large sizes
  // start beside the small sizes' kernels: that was slower, 0.821-0.840 vs
  // 0.811-0.829 ms per 4K step, profiles/r04_v13_ab_notes.txt)
  auto work = [&](int s) {
    return (long)__builtin_popcount(type_masks[s]) * (width / tx_w(s)) * (height / tx_h(s)) *
           max_eob(s);
  };
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && work(order[j]) > work(order[j - 1]); --j) {
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  hipStream_t* fs = fan_out(caller);
  int rc = 0;
  for (int i = 0; i < n && rc == 0; ++i) {
    const int s = order[i];
    rc = rdo_plane(src, pred, stride, width, height, s, type_masks[s], bd, qp, rdmult, out[s],
                   qcoeff[s], dqcoeff[s], fs[i % fan_width()], px);
  }
  fan_in(caller);
  return rc;
}

namespace {

__constant__ uint8_t kTxWd[19] = {4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64};
__constant__ uint8_t kTxHd[19] = {4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16};
__device__ __forceinline__ int tx_w_dev(int s) { return kTxWd[s]; }
__device__ __forceinline__ int tx_h_dev(int s) { return kTxHd[s]; }
// av1_get_max_eob (av1/common/blockd.h:1596-1604)
__device__ __forceinline__ int max_eob_dev(int s) {
  const int w = kTxWd[s], h = kTxHd[s];
  if (w == 64 || h == 64) return (w == 16 || h == 16) ? 512 : 1024;
  return w * h;
}

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
  return a > INT64_MAX - b ? INT64_MAX : a + b;
}

struct SbArgs {
  int nsizes;
  int sizes[19];                       // candidate order: largest area first
  const LavishRdoBlock* rec[19];
  LavishInvJob* jobs[19];              // per size: one slot of `cap` jobs per SB
  uint16_t* cnt[19];                   // per size and SB: its live jobs
  int sbw, sbh;                        // superblocks per row / column
  int width, height, stride;
  uint8_t* sb_tx_size;
};

// per SB64: the candidate TX size whose blocks' summed RD cost is lowest
// (sizes that do not tile the SB with full blocks are skipped; ties keep
// the earlier, larger size), then the inverse-transform jobs of that size's
// blocks with eob > 0 -- a block with eob 0 adds nothing
// (av1_inverse_transform_block, idct.c:308) and the other sizes' blocks are
// not reconstructed at all.
// One wave64 per SB: lanes stride the SB's blocks of a size, a 64-bit xor
// reduction sums their costs; the size scan stays sequential (strict <).
// Jobs go to the SB's own slot of each size's list (no atomics, nothing to
// zero first): the chosen size's coded blocks, compacted by ballot, and a
// count of 0 in every other size's slot.
__global__ __launch_bounds__(256) void sb_decide_kernel(SbArgs a) {
  const int sb = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (sb >= a.sbw * a.sbh) return;
  const int sy = sb / a.sbw, sx = sb - sy * a.sbw;
  const int y1 = min(64, a.height - sy * 64), x1 = min(64, a.width - sx * 64);
  int64_t best = INT64_MAX;
  int best_s = 255;
  for (int i = 0; i < a.nsizes; ++i) {
    const int s = a.sizes[i];
    const int W = tx_w_dev(s), H = tx_h_dev(s);
    if (y1 % H || x1 % W) continue;
    const int bw = a.width / W, nx = x1 / W, nblk = nx * (y1 / H);
    // costs are >= 0; a block without a candidate costs INT64_MAX, so the
    // sums saturate there instead of wrapping
    // (nblk <= 256: the loads of up to 4 blocks per lane in flight together;
    // a sum of non-negative costs saturating at INT64_MAX is order-free)
    int64_t v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = lane + 64 * q;
      const int y = k / nx, x = k - y * nx;
      v[q] = k < nblk ? a.rec[s][(sy * 64 / H + y) * bw + sx * 64 / W + x].rdcost : 0;
    }
    int64_t sum = sat_add(sat_add(v[0], v[1]), sat_add(v[2], v[3]));
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) sum = sat_add(sum, __shfl_xor(sum, m));
    if (sum < best) {
      best = sum;
      best_s = s;
    }
  }
  if (lane == 0) {
    a.sb_tx_size[sb] = (uint8_t)best_s;
    for (int i = 0; i < a.nsizes; ++i)
      if (a.sizes[i] != best_s) a.cnt[a.sizes[i]][sb] = 0;
  }
  if (best_s == 255) return;  // no candidate tiles this SB: recon = pred
  const int s = best_s;
  const int W = tx_w_dev(s), H = tx_h_dev(s);
  const int bw = a.width / W, nx = x1 / W, nblk = nx * (y1 / H), n = max_eob_dev(s);
  LavishInvJob* const slot = a.jobs[s] + (size_t)sb * ((64 / W) * (64 / H));
  int base = 0;
  for (int k0 = 0; k0 < nblk; k0 += 64) {
    const int k = k0 + lane;
    const int y = k / nx, x = k - y * nx;
    const int blk = (sy * 64 / H + y) * bw + sx * 64 / W + x;
    const bool live = k < nblk;
    const LavishRdoBlock r = a.rec[s][live ? blk : 0];
    const bool coded = live && r.eob != 0;
    const uint64_t m = __builtin_amdgcn_ballot_w64(coded);
    if (coded) {
      const int at = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      LavishInvJob j;
      j.dst_off = (int64_t)(sy * 64 + y * H) * a.stride + sx * 64 + x * W;
      j.coeff_off = (int64_t)blk * n;
      j.tx_type = r.best_type;
      j.eob = r.eob;
      slot[at] = j;
    }
    base += __popcll(m);
  }
  if (lane == 0) a.cnt[s][sb] = (uint16_t)base;
}

// inverse-transform job list of lavish_rdo_reconstruct: reused call after
// call, possibly from different streams (e.g. per-band streams of a shard),
// so reuse is ordered by StreamScratch's event
thread_local StreamScratch t_rs;

}  // namespace

namespace {

// px64 helpers: inverse jobs of the TX-domain winners, then per block the
// pixel SSE and the distortion rules of search_tx_type (tx_search.c:2187-2231)
__global__ void px64_jobs_kernel(const LavishRdoBlock* rec, int nblocks, int bw, int W, int H,
                                 int n, int stride, LavishInvJob* jobs) {
  const int blk = blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= nblocks) return;
  const int by = blk / bw, bx = blk - by * bw;
  LavishInvJob j;
  j.dst_off = (int64_t)by * H * stride + (int64_t)bx * W;
  j.coeff_off = (int64_t)blk * n;
  j.tx_type = rec[blk].best_type;
  j.eob = rec[blk].eob;
  jobs[blk] = j;
}

__global__ __launch_bounds__(256) void px64_finish_kernel(const uint16_t* src, const uint16_t* pred,
                                                          const uint16_t* recon, int stride,
                                                          int bw, int W, int H, int is64, int bd,
                                                          int rdmult, LavishRdoBlock* rec) {
  const int blk = blockIdx.x;
  const int by = blk / bw, bx = blk - by * bw;
  const size_t base = (size_t)by * H * stride + (size_t)bx * W;
  uint64_t s1 = 0, s2 = 0;
  for (int i = threadIdx.x; i < W * H; i += 256) {
    const size_t o = base + (size_t)(i / W) * stride + (i % W);
    const int64_t d1 = (int64_t)src[o] - pred[o], d2 = (int64_t)src[o] - recon[o];
    s1 += (uint64_t)(d1 * d1);
    s2 += (uint64_t)(d2 * d2);
  }
  __shared__ uint64_t r1[4], r2[4];
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    s1 += __shfl_xor(s1, m);
    s2 += __shfl_xor(s2, m);
  }
  if ((threadIdx.x & 63) == 0) {
    r1[threadIdx.x >> 6] = s1;
    r2[threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  s1 = r1[0] + r1[1] + r1[2] + r1[3];
  s2 = r2[0] + r2[1] + r2[2] + r2[3];
  const int sh = 2 * (bd - 8);
  if (sh > 0) {
    s1 = (s1 + ((uint64_t)1 << (sh - 1))) >> sh;
    s2 = (s2 + ((uint64_t)1 << (sh - 1))) >> sh;
  }
  const int64_t bsse = (int64_t)s1 * 16;
  LavishRdoBlock o = rec[blk];
  int64_t dist = o.dist;
  if (o.eob == 0) {
    dist = bsse;
  } else {
    const bool high = bsse >= (int64_t)128 * 128 * W * H;
    const int64_t sse_diff = bsse - o.sse;
    if (!is64 || !high || sse_diff * 2 < o.sse) {
      const int64_t pxd = (int64_t)(uint32_t)(16u * (uint32_t)s2);
      dist = (high && pxd < dist) ? dist : pxd;
    } else {
      dist += sse_diff;
    }
  }
  o.dist = dist;
  o.sse = bsse;
  o.rdcost = (((int64_t)o.rate * rdmult + 256) >> 9) + dist * 128;
  rec[blk] = o;
}

// per TX size: rdo_frame_px deals the 64-point sizes over concurrent fan-out
// streams, so each size owns its scratch plane / job list, and reuse across
// calls (any stream) waits for the previous user's event
thread_local StreamScratch t_px_plane[19], t_px_jobs[19];

}  // namespace

int rdo_plane_px64(RdoArgs& a, int tx_size, int width, int height, hipStream_t s) {
  if (a.ntypes != 1) return -6;  // 64-point sizes have one candidate type
  int rc = launch_size<1>(tx_size, a, s);
  if (rc || a.nblocks == 0) return rc;
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  uint16_t* plane = (uint16_t*)t_px_plane[tx_size].acquire(
      (size_t)a.stride * height * sizeof(uint16_t), s);
  LavishInvJob* jobs =
      (LavishInvJob*)t_px_jobs[tx_size].acquire((size_t)a.nblocks * sizeof(LavishInvJob), s);
  LAVISH_CHECK(hipMemcpy2DAsync(plane, (size_t)a.stride * 2, a.pred, (size_t)a.stride * 2,
                                (size_t)width * 2, height, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(px64_jobs_kernel, dim3((a.nblocks + 255) / 256), dim3(256), 0, s, a.out,
                     a.nblocks, a.bw, W, H, max_eob(tx_size), a.stride, jobs);
  LAVISH_CHECK(hipGetLastError());
  rc = inv_txfm_add_batch(a.dqcoeff, tx_size, jobs, a.nblocks, plane, a.stride, a.bd, 1, s);
  if (rc == 0) {
    hipLaunchKernelGGL(px64_finish_kernel, dim3(a.nblocks), dim3(256), 0, s, a.src, a.pred,
                       plane, a.stride, a.bw, W, H, tx_size == 4 ? 1 : 0, a.bd, a.rdmult,
                       a.out);
    LAVISH_CHECK(hipGetLastError());
  }
  // both scratches are released on every path: the copy and the job kernel
  // are already queued on `s`, so a later acquire must wait for them
  t_px_plane[tx_size].release(s);
  t_px_jobs[tx_size].release(s);
  return rc;
}

// reconstruction scratch: per candidate size one slot of (64 / w) x (64 / h)
// jobs per SB, then the SBs' job counts; offsets into it
size_t recon_scratch_layout(const SbArgs& a, int nsb, size_t (&joff)[19], size_t (&coff)[19]) {
  size_t bytes = 0;
  for (int i = 0; i < a.nsizes; ++i) {
    const int t = a.sizes[i];
    joff[t] = bytes;
    bytes += (size_t)nsb * (64 / tx_w(t)) * (64 / tx_h(t)) * sizeof(LavishInvJob);
  }
  for (int i = 0; i < a.nsizes; ++i) {
    const int t = a.sizes[i];
    coff[t] = bytes;
    bytes += ((size_t)nsb * sizeof(uint16_t) + 15) & ~(size_t)15;
  }
  return bytes;
}

// scratch_out: nullptr -> the per-thread stream-ordered scratch; else the
// caller's buffer of recon_scratch_bytes() (a captured graph owns one)
int rdo_reconstruct_impl(uint32_t size_mask, const LavishRdoBlock* const* rec,
                         const int32_t* const* dqcoeff, int width, int height,
                         const uint16_t* pred, uint16_t* recon, int stride, int bd,
                         uint8_t* sb_tx_size, hipStream_t s, char* own_scratch,
                         size_t* scratch_bytes);

int rdo_reconstruct(uint32_t size_mask, const LavishRdoBlock* const* rec,
                    const int32_t* const* dqcoeff, int width, int height, const uint16_t* pred,
                    uint16_t* recon, int stride, int bd, uint8_t* sb_tx_size, hipStream_t s) {
  return rdo_reconstruct_impl(size_mask, rec, dqcoeff, width, height, pred, recon, stride, bd,
                              sb_tx_size, s, nullptr, nullptr);
}

int rdo_reconstruct_impl(uint32_t size_mask, const LavishRdoBlock* const* rec,
                         const int32_t* const* dqcoeff, int width, int height,
                         const uint16_t* pred, uint16_t* recon, int stride, int bd,
                         uint8_t* sb_tx_size, hipStream_t s, char* own_scratch,
                         size_t* scratch_bytes) {
  SbArgs a{};
  for (int t = 0; t < 19; ++t)
    if ((size_mask >> t) & 1) a.sizes[a.nsizes++] = t;
  if (a.nsizes == 0) return -1;
  for (int i = 1; i < a.nsizes; ++i)  // largest area first
    for (int j = i; j > 0 && tx_w(a.sizes[j]) * tx_h(a.sizes[j]) >
                                 tx_w(a.sizes[j - 1]) * tx_h(a.sizes[j - 1]); --j) {
      const int t = a.sizes[j];
      a.sizes[j] = a.sizes[j - 1];
      a.sizes[j - 1] = t;
    }
  for (int i = 0; i < a.nsizes; ++i) a.rec[a.sizes[i]] = rec[a.sizes[i]];
  a.sbw = (width + 63) / 64;
  a.sbh = (height + 63) / 64;
  a.width = width;
  a.height = height;
  a.stride = stride;
  a.sb_tx_size = sb_tx_size;
  const int nsb = a.sbw * a.sbh;
  size_t joff[19] = {}, coff[19] = {};
  const size_t bytes = recon_scratch_layout(a, nsb, joff, coff);
  if (scratch_bytes != nullptr) {  // size query
    *scratch_bytes = bytes;
    if (own_scratch == nullptr) return 0;
  }
  const bool shared = own_scratch == nullptr;
  char* scratch = shared ? (char*)t_rs.acquire(bytes, s) : own_scratch;
  for (int i = 0; i < a.nsizes; ++i) {
    const int t = a.sizes[i];
    a.jobs[t] = (LavishInvJob*)(scratch + joff[t]);
    a.cnt[t] = (uint16_t*)(scratch + coff[t]);
  }
  hipLaunchKernelGGL(sb_decide_kernel, dim3((nsb + 3) / 4), dim3(256), 0, s, a);
  LAVISH_CHECK(hipGetLastError());
  // recon = pred, then add the chosen coded blocks' residuals: the sizes'
  // inverse launches side by side over the fan-out streams (every SB chose
  // one size, so they write disjoint pixels; a size no SB chose still costs a
  // launch of ~6 us, which then overlaps the others instead of following them)
  LAVISH_CHECK(hipMemcpy2DAsync(recon, (size_t)stride * 2, pred, (size_t)stride * 2,
                                (size_t)width * 2, height, hipMemcpyDeviceToDevice, s));
  hipStream_t* fs = fan_out(s);
  int rc = 0, k = 0;
  for (int i = 0; i < a.nsizes && rc == 0; ++i) {
    const int t = a.sizes[i];
    if ((width / tx_w(t)) * (height / tx_h(t)) == 0) continue;
    const int cap = (64 / tx_w(t)) * (64 / tx_h(t));
    rc = inv_txfm_add_batch(dqcoeff[t], t, a.jobs[t], nsb * cap, recon, stride, bd, 1,
                            fs[k++ % fan_width()], a.cnt[t], cap);
  }
  fan_in(s);
  if (shared) t_rs.release(s);
  return rc;
}

}  // namespace lavish

extern "C" int lavish_rdo_plane(const uint16_t* src, const uint16_t* pred, int stride, int width,
                                int height, int tx_size, uint32_t type_mask, int bit_depth,
                                const LavishQuantParams* qp, int rdmult, LavishRdoBlock* out,
                                int32_t* qcoeff, int32_t* dqcoeff, void* stream) {
  return lavish::rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream);
}

extern "C" int lavish_rdo_plane_px(const uint16_t* src, const uint16_t* pred, int stride,
                                   int width, int height, int tx_size, uint32_t type_mask,
                                   int bit_depth, const LavishQuantParams* qp, int rdmult,
                                   LavishRdoBlock* out, int32_t* qcoeff, int32_t* dqcoeff,
                                   void* stream) {
  return lavish::rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream, 1);
}

extern "C" int lavish_rdo_frame(const uint16_t* src, const uint16_t* pred, int stride, int width,
                                int height, uint32_t size_mask, const uint32_t* type_masks,
                                int bit_depth, const LavishQuantParams* qp, int rdmult,
                                LavishRdoBlock* const* out, int32_t* const* qcoeff,
                                int32_t* const* dqcoeff, void* stream) {
  return lavish::rdo_frame(src, pred, stride, width, height, size_mask, type_masks, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream);
}

extern "C" int lavish_rdo_frame_px(const uint16_t* src, const uint16_t* pred, int stride,
                                   int width, int height, uint32_t size_mask,
                                   const uint32_t* type_masks, int bit_depth,
                                   const LavishQuantParams* qp, int rdmult,
                                   LavishRdoBlock* const* out, int32_t* const* qcoeff,
                                   int32_t* const* dqcoeff, void* stream) {
  return lavish::rdo_frame(src, pred, stride, width, height, size_mask, type_masks, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream, 1);
}

extern "C" int lavish_rdo_reconstruct(uint32_t size_mask, const LavishRdoBlock* const* records,
                                      const int32_t* const* dqcoeff, int width, int height,
                                      const uint16_t* pred, uint16_t* recon, int stride,
                                      int bit_depth, uint8_t* sb_tx_size, void* stream) {
  return lavish::rdo_reconstruct(size_mask, records, dqcoeff, width, height, pred, recon, stride,
                                 bit_depth, sb_tx_size, (hipStream_t)stream);
}

extern "C" int lavish_rdo_plane_masked(const uint16_t* src, const uint16_t* pred, int stride,
                                       int width, int height, int tx_size, uint32_t type_mask,
                                       int bit_depth, const LavishQuantParams* qp, int rdmult,
                                       const uint16_t* block_mask, const uint8_t* block_map,
                                       int pixel_domain, LavishRdoBlock* out, int32_t* qcoeff,
                                       int32_t* dqcoeff, void* stream) {
  return lavish::rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream, pixel_domain ? 1 : 0,
                           block_mask, block_map);
}

extern "C" int lavish_rdo_plane_rate(const uint16_t* src, const uint16_t* pred, int stride,
                                     int width, int height, int tx_size, uint32_t type_mask,
                                     int bit_depth, const LavishQuantParams* qp, int rdmult,
                                     const LavishCoeffCosts* costs, const LavishTxbCtx* txb_ctx,
                                     const int32_t* tx_type_costs, const uint16_t* block_mask,
                                     const uint8_t* block_map, LavishRdoBlock* out,
                                     int32_t* qcoeff, int32_t* dqcoeff, void* stream) {
  const lavish::RateCfg rc{costs, txb_ctx, tx_type_costs};
  return lavish::rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream, 0, block_mask,
                           block_map, &rc);
}

// ---------------------------------------------------------------------------
// A captured C4 step: lavish_rdo_frame + lavish_rdo_reconstruct for fixed
// buffers recorded once into a HIP graph, replayed with one launch.  For
// callers that run the step on many small rectangles (the C5 row wavefront's
// chunks), where ~15 kernel launches and the fan-out events per call cost
// more host time than the rectangle's GPU work.  The graph owns the
// reconstruction's job scratch, so replays on any stream are independent of
// the per-thread scratch; two replays of one graph must not overlap.
// ---------------------------------------------------------------------------
struct LavishRdoGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  void* scratch = nullptr;
};

extern "C" int lavish_rdo_graph_create(const uint16_t* src, const uint16_t* pred, int stride,
                                       int width, int height, uint32_t size_mask,
                                       const uint32_t* type_masks, int bit_depth,
                                       const LavishQuantParams* qp, int rdmult,
                                       LavishRdoBlock* const* records, int32_t* const* qcoeff,
                                       int32_t* const* dqcoeff, uint16_t* recon,
                                       uint8_t* sb_tx_size, void* stream,
                                       LavishRdoGraph** out) {
  if (out == nullptr) return -3;
  *out = nullptr;
  size_t bytes = 0;
  int rc = lavish::rdo_reconstruct_impl(size_mask, (const LavishRdoBlock* const*)records,
                                        (const int32_t* const*)dqcoeff, width, height, pred,
                                        recon, stride, bit_depth, sb_tx_size, nullptr, nullptr,
                                        &bytes);
  if (rc) return rc;
  LavishRdoGraph* g = new LavishRdoGraph();
  LAVISH_CHECK(hipMalloc(&g->scratch, bytes > 0 ? bytes : 16));
  hipStream_t cs;
  LAVISH_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  // the warm-up below reads src / pred and writes every output buffer: order
  // it after the caller's pending work on them (e.g. a fill of the
  // reconstruction plane still queued on the caller's stream)
  hipEvent_t after;
  LAVISH_CHECK(hipEventCreateWithFlags(&after, hipEventDisableTiming));
  LAVISH_CHECK(hipEventRecord(after, (hipStream_t)stream));
  LAVISH_CHECK(hipStreamWaitEvent(cs, after, 0));
  LAVISH_CHECK(hipEventDestroy(after));
  // one uncaptured run first: the library's lazily created state (internal
  // streams, device scan tables: synchronous uploads) must exist before the
  // capture, which may only record stream work
  rc = lavish::rdo_frame(src, pred, stride, width, height, size_mask, type_masks, bit_depth, qp,
                         rdmult, records, qcoeff, dqcoeff, cs);
  if (rc == 0)
    rc = lavish::rdo_reconstruct_impl(size_mask, (const LavishRdoBlock* const*)records,
                                      (const int32_t* const*)dqcoeff, width, height, pred, recon,
                                      stride, bit_depth, sb_tx_size, cs, (char*)g->scratch,
                                      &bytes);
  LAVISH_CHECK(hipStreamSynchronize(cs));
  if (rc != 0) {
    LAVISH_CHECK(hipStreamDestroy(cs));
    lavish_rdo_graph_destroy(g);
    return rc;
  }
  LAVISH_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
  rc = lavish::rdo_frame(src, pred, stride, width, height, size_mask, type_masks, bit_depth, qp,
                         rdmult, records, qcoeff, dqcoeff, cs);
  if (rc == 0)
    rc = lavish::rdo_reconstruct_impl(size_mask, (const LavishRdoBlock* const*)records,
                                      (const int32_t* const*)dqcoeff, width, height, pred, recon,
                                      stride, bit_depth, sb_tx_size, cs, (char*)g->scratch,
                                      &bytes);
  hipGraph_t graph = nullptr;
  LAVISH_CHECK(hipStreamEndCapture(cs, &graph));
  LAVISH_CHECK(hipStreamDestroy(cs));
  g->graph = graph;
  if (rc == 0 && graph != nullptr)
    LAVISH_CHECK(hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0));
  if (rc != 0 || g->exec == nullptr) {
    lavish_rdo_graph_destroy(g);
    return rc ? rc : -8;
  }
  *out = g;
  return 0;
}

extern "C" int lavish_rdo_graph_launch(LavishRdoGraph* g, void* stream) {
  if (g == nullptr || g->exec == nullptr) return -3;
  LAVISH_CHECK(hipGraphLaunch(g->exec, (hipStream_t)stream));
  return 0;
}

extern "C" void lavish_rdo_graph_destroy(LavishRdoGraph* g) {
  if (g == nullptr) return;
  if (g->exec) LAVISH_CHECK(hipGraphExecDestroy(g->exec));
  if (g->graph) LAVISH_CHECK(hipGraphDestroy(g->graph));
  if (g->scratch) LAVISH_CHECK(hipFree(g->scratch));
  delete g;
}
