// txq_dev.h -- the C2 device code (batched forward transform + quantization
// of every TX type, txq.hip) shared by txq.hip's kernels and the fused C2 + C3
// launch (mcomp.hip, lavish_txq_frame_search).
#pragma once

#include "lane_red.h"
#include "lavish_internal.h"
#include "quant_dev.h"

namespace lavish {

struct TxqArgs {
  const int16_t* res;
  int stride;
  int bw;       // blocks per row
  int nblocks;  // total blocks
  int ntypes;
  int types[16];
  // type chunks along the grid: the types of a chunk share one vertical
  // (column) 1-D kind, so a workgroup runs the column pass once per chunk;
  // chunk g holds type slots chunk_ti[chunk_off[g] .. chunk_off[g+1])
  int tgroups;
  int chunk_off[17];
  int chunk_ti[16];
  int quant_kind;
  int highbd;
  QP qp;
  const int16_t* iscan_default;  // default-scan inverse table (n entries)
  int32_t* qcoeff;
  int32_t* dqcoeff;
  uint16_t* eob;
  int32_t* coeff;
};

template <int W, int H>
struct Tile {
  static constexpr int MN = W < H ? W : H;
  static constexpr int P = 64 / MN;     // blocks per wave tile
  static constexpr int CPT = W / MN;    // column transforms per lane
  static constexpr int RPT = H / MN;    // row transforms per lane
  static constexpr int N = W * H;       // coefficients per block (sizes <= 32)
  static constexpr int T1S = W + 1;     // padded LDS row stride
  static constexpr int T1 = P * H * T1S;
  static constexpr int T2 = P * N;
};

template <int W, int H, bool FAST, int QK, bool HBD>
__device__ __forceinline__ void txq_types(const TxqArgs& a,
                                          const int32_t (&res)[Tile<W, H>::CPT][H],
                                          int32_t* t1, int32_t* t2, const int16_t* isc, int lane,
                                          int blk0, int nvalid, int c0, int c1) {
  using C = TxCfg<W, H>;
  using T = Tile<W, H>;
  constexpr int N = T::N, T1S = T::T1S;
  constexpr int LS = C::log_scale;
  // ---- columns, once for the chunk's vertical kind (av1_fwd_txfm2d.c:88-106) ----
  {
    // wave-uniform by construction; readfirstlane keeps the transform-kind
    // branches scalar (otherwise hipcc if-converts all three kernels)
    const int t = __builtin_amdgcn_readfirstlane(a.types[a.chunk_ti[c0]]);
    const int vt = (kVtxPacked >> (2 * t)) & 3;
    const int kc = vt == 3 ? 2 : (vt == 0 ? 0 : 1);
    const bool ud = vt == 2;
#pragma unroll
    for (int k = 0; k < T::CPT; ++k) {
      const int j = k * 64 + lane;
      const int b = j / W, c = j % W;
      int32_t in[H], out[H];
#pragma unroll
      for (int r = 0; r < H; ++r) {
        const int32_t x = ud ? res[k][H - 1 - r] : res[k][r];
        if constexpr (FAST) in[r] = x * (1 << C::s0);  // |x| <= 1023: no saturation
        else in[r] = round_shift_1<-C::s0>(x);
      }
      fwd_1d<H, C::cos_bit_col, FAST>(kc, in, out);
#pragma unroll
      for (int r = 0; r < H; ++r) t1[(b * H + r) * T1S + c] = round_shift_1<-C::s1>(out[r]);
    }
    wave_sync();
  }

  // lowbd quantize_fp on the FAST range (the C2 bench path), uniform per
  // (dc, ac): the rounding, quant, the pass threshold ceil(dequant /
  // 2^(1 + LS)) - 1 (see the coefficient loop)
  int qf_rnd[2], qf_thr1[2], qf_qt[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    qf_rnd[i] = (a.qp.round[i] + ((1 << LS) >> 1)) >> LS;
    qf_qt[i] = a.qp.quant[i];
    qf_thr1[i] = ((a.qp.dequant[i] + (1 << (1 + LS)) - 1) >> (1 + LS)) - 1;
  }

  for (int ci = c0; ci < c1; ++ci) {
    const int ti = __builtin_amdgcn_readfirstlane(a.chunk_ti[ci]);
    const int t = __builtin_amdgcn_readfirstlane(a.types[ti]);
    const int ht = (kHtxPacked >> (2 * t)) & 3;
    const int kr = ht == 3 ? 2 : (ht == 0 ? 0 : 1);
    const bool lr = ht == 2;  // FLIPADST rows: the column results read right to left
    const int skind = t < 10 ? 0 : ((t & 1) ? 1 : 2);

    // ---- rows + quantization (av1_fwd_txfm2d.c:110-126, av1_quantize.c) ----
#pragma unroll
    for (int k = 0; k < T::RPT; ++k) {
      const int j = k * 64 + lane;
      const int b = j / H, r = j % H;
      int32_t in[W], out[W];
      const int32_t* row = t1 + (b * H + r) * T1S;
      if (lr) {
#pragma unroll
        for (int c = 0; c < W; ++c) in[c] = row[W - 1 - c];
      } else {
#pragma unroll
        for (int c = 0; c < W; ++c) in[c] = row[c];
      }
      fwd_1d<W, C::cos_bit_row, FAST>(kr, in, out);
      const size_t obase = ((size_t)ti * a.nblocks + blk0 + b) * N;
      // eob = 1 + last scan position holding a nonzero qcoeff; the inverse
      // scan of this type's scan kind is row skind of the LDS table
      const int16_t* iscan = isc + skind * N;
      int last = 0;
      if constexpr (QK == LAVISH_QUANT_FP && FAST && !HBD) {
        // av1_quantize_fp_c (av1_quantize.c:174-194, lowbd) restated in the
        // VALU's 2-cycle classes (tools/microbench/valu_rates.hip: add / sub
        // / xor / and / ashr ~2 cycles; multiplies, min / max, cndmask,
        // shifts left ~4): a = |v|; pass <=> a << (1 + LS) >= dequant <=>
        // a > thr1, a mask; q = (min(a + rnd, 32767) * quant) >> (16 - LS)
        // (24-bit multiply: both < 2^15); eob = max over nonzero q of
        // iscan + 1, nonzero = (q + 2^23 - 1) >> 23 (q < 2^23).  The same
        // integers as quant_one.
        const bool dcl = r == 0;
        const int rnd0 = dcl ? qf_rnd[0] : qf_rnd[1];
        const int qt0 = dcl ? qf_qt[0] : qf_qt[1];
        const int thr0 = dcl ? qf_thr1[0] : qf_thr1[1];
#pragma unroll
        for (int c = 0; c < W; ++c) {
          int32_t v = round_shift_1<-C::s2>(out[c]);
          if constexpr (C::rect2) v = rshift64((int64_t)v * 5793, 12);
          const int rc = c * H + r;
          if (a.coeff != nullptr) {
            if (b < nvalid) a.coeff[obase + rc] = v;
          }
          const int32_t sgn = v >> 31;
          const int32_t av = (v ^ sgn) - sgn;
          const int32_t pass = ((c ? qf_thr1[1] : thr0) - av) >> 31;
          const int32_t t = min(av + (c ? qf_rnd[1] : rnd0), 32767);
          const int32_t qa = (mul_i24(t, c ? qf_qt[1] : qt0) >> (16 - LS)) & pass;
          const int32_t q = (qa ^ sgn) - sgn;
          t2[b * N + rc] = q;
          const int32_t nz = (qa + 0x7FFFFF) >> 23;
          last = max(last, ((int)iscan[rc] + 1) & -nz);
        }
      } else {
#pragma unroll
      for (int c = 0; c < W; ++c) {
        int32_t v = round_shift_1<-C::s2>(out[c]);
        if constexpr (C::rect2) v = rshift64((int64_t)v * 5793, 12);
        const int rc = c * H + r;
        int32_t q = 0;
        if constexpr (QK == LAVISH_QUANT_NONE) {
          if (b < nvalid) a.coeff[obase + rc] = v;
        } else {
          if (a.coeff != nullptr) {
            if (b < nvalid) a.coeff[obase + rc] = v;
          }
          q = quant_one<LS, QK, HBD, FAST>(v, c != 0 || r != 0, a.qp);
        }
        t2[b * N + rc] = q;
        const int pos1 = iscan[rc] + 1;
        last = q != 0 ? max(last, pos1) : last;
      }
      }
      last = lane_max<H>(last);
      if (r == 0 && b < nvalid && a.eob != nullptr)
        a.eob[(size_t)ti * a.nblocks + blk0 + b] = (uint16_t)last;
    }
    wave_sync();

    // ---- coalesced copy-out of qcoeff / dqcoeff (1 KiB per instruction) ----
    if (a.qcoeff != nullptr) {
      const int total = nvalid * N;
      const size_t gbase = ((size_t)ti * a.nblocks + blk0) * N;
      // streaming (nontemporal) stores: the outputs are written once and
      // far exceed the 256 MiB Infinity Cache
      for (int i = lane * 4; i < total; i += 64 * 4) {
        const v4i q4 = *reinterpret_cast<const v4i*>(&t2[i]);
        __builtin_nontemporal_store(q4, reinterpret_cast<v4i*>(&a.qcoeff[gbase + i]));
        if (a.dqcoeff != nullptr) {
          const int rc0 = i % N;  // N % 4 == 0: all four share the block
          v4i d4;
          d4.x = dequant_one<LS, FAST>(q4.x, rc0 != 0, a.qp);  // only x can be DC
          d4.y = dequant_one<LS, FAST>(q4.y, 1, a.qp);
          d4.z = dequant_one<LS, FAST>(q4.z, 1, a.qp);
          d4.w = dequant_one<LS, FAST>(q4.w, 1, a.qp);
          __builtin_nontemporal_store(d4, reinterpret_cast<v4i*>(&a.dqcoeff[gbase + i]));
        }
      }
    }
    wave_sync();  // t2 is rewritten by the next type's row pass
  }
}

// LDS of one workgroup of size W x H: t1 (column results, padded rows), t2
// (coefficients, 16-byte aligned), the three inverse scans
template <int W, int H>
struct TxqLds {
  using T = Tile<W, H>;
  static constexpr int kT2Off = (4 * T::T1 * 4 + 15) & ~15;          // bytes
  static constexpr int kIscOff = kT2Off + 4 * T::T2 * 4;
  static constexpr int kBytes = kIscOff + 3 * T::N * 2;
};

// One 256-thread workgroup = 4 independent wave tiles (no workgroup
// barriers after the shared iscan load).  Grid: (tile quad, type group); the
// type groups of one tile quad get workgroup ids congruent mod 8, i.e. the
// same XCD, so repeated residual reads hit that XCD's L2.  `id` is the
// workgroup's index within this size's grid (a multiple of 8 from the
// launch's start, so id & 7 is still the XCD).
template <int W, int H>
__device__ __forceinline__ void txq_plane_body(const TxqArgs& a, int id, char* lds) {
  using T = Tile<W, H>;
  using LL = TxqLds<W, H>;
  constexpr int H_ = H;
  int32_t* t1s = reinterpret_cast<int32_t*>(lds);
  int32_t* t2s = reinterpret_cast<int32_t*>(lds + LL::kT2Off);
  int16_t* isc = reinterpret_cast<int16_t*>(lds + LL::kIscOff);  // default, mcol, mrow

  const int inner = id & 7, rest = id >> 3;
  const int tg = rest % a.tgroups, quad = (rest / a.tgroups) * 8 + inner;
  const int ntiles = (a.nblocks + T::P - 1) / T::P;
  if (quad * 4 >= ntiles) return;
  const int c0 = a.chunk_off[tg], c1 = a.chunk_off[tg + 1];

  const int tid = threadIdx.x;
  for (int i = tid; i < T::N; i += 256) {
    isc[i] = a.iscan_default[i];
    isc[T::N + i] = (int16_t)i;                                   // mcol: identity
    isc[2 * T::N + i] = (int16_t)((i % H) * W + i / H);           // mrow: r*W + c
  }
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63;
  const int tile = quad * 4 + wave;
  if (tile >= ntiles) return;
  const int blk0 = tile * T::P;
  const int nvalid = min(T::P, a.nblocks - blk0);
  int32_t* t1 = t1s + wave * T::T1;
  int32_t* t2 = t2s + wave * T::T2;

  // residual columns -> registers (read once for all TX types of the group)
  int32_t res[T::CPT][H_];
  int32_t amax = 0;
#pragma unroll
  for (int k = 0; k < T::CPT; ++k) {
    const int j = k * 64 + lane;
    const int b = j / W, c = j % W;
    const int blk = blk0 + b;
    if (b < nvalid) {
      const int by = blk / a.bw, bx = blk - by * a.bw;
      const int16_t* src = a.res + (size_t)by * H * a.stride + bx * W + c;
#pragma unroll
      for (int r = 0; r < H; ++r) {
        res[k][r] = src[(size_t)r * a.stride];
        amax = max(amax, abs(res[k][r]));
      }
    } else {
#pragma unroll
      for (int r = 0; r < H; ++r) res[k][r] = 0;
    }
  }
  // wave-uniform choice of the certified-exact fast arithmetic
  const bool fast = __builtin_amdgcn_ballot_w64(amax > kFastResidualMax) == 0;
#define LAVISH_TXQ_RUN(F, Q, HB) \
  txq_types<W, H, F, Q, HB>(a, res, t1, t2, isc, lane, blk0, nvalid, c0, c1)
  const int qk = a.quant_kind;
  if (qk == LAVISH_QUANT_NONE) {
    if (fast) LAVISH_TXQ_RUN(true, LAVISH_QUANT_NONE, false);
    else LAVISH_TXQ_RUN(false, LAVISH_QUANT_NONE, false);
  } else if (qk == LAVISH_QUANT_FP) {
    if (a.highbd) {
      if (fast) LAVISH_TXQ_RUN(true, LAVISH_QUANT_FP, true);
      else LAVISH_TXQ_RUN(false, LAVISH_QUANT_FP, true);
    } else {
      if (fast) LAVISH_TXQ_RUN(true, LAVISH_QUANT_FP, false);
      else LAVISH_TXQ_RUN(false, LAVISH_QUANT_FP, false);
    }
  } else {
    if (a.highbd) {
      if (fast) LAVISH_TXQ_RUN(true, LAVISH_QUANT_B, true);
      else LAVISH_TXQ_RUN(false, LAVISH_QUANT_B, true);
    } else {
      if (fast) LAVISH_TXQ_RUN(true, LAVISH_QUANT_B, false);
      else LAVISH_TXQ_RUN(false, LAVISH_QUANT_B, false);
    }
  }
#undef LAVISH_TXQ_RUN
}

// ---------------------------------------------------------------------------
// One launch for many TX sizes (lavish_txq_frame): the sizes' grids back to
// back in one grid, heaviest first; workgroup g runs size k with
// wg0[k] <= g < wg0[k + 1].  No cross-stream fork / join and no per-kernel
// tail between sizes.  Class 0: the sizes up to 16 points (<= 115 VGPRs,
// <= 37 KB LDS: 4 waves / SIMD); class 1: the 32-point sizes.
// The per-size arguments are separate kernel parameters at a fixed slot per
// size (txq_slot): one aggregate parameter holding all of them is copied to
// scratch memory once any field is indexed dynamically (measured: 10x
// slower); a TxqArgs parameter of its own is read in place, as in
// txq_plane_kernel.
constexpr int kMultiMax = 9;
struct TxqDispatch {
  int code[kMultiMax];       // dispatch entry k: tx_size
  int wg0[kMultiMax + 1];    // dispatch entry k: first workgroup (multiples of 8)
  int n;
};
struct TxqMulti {
  TxqArgs a[kMultiMax];      // by slot (txq_slot(tx_size))
  TxqDispatch d;
};
__host__ __device__ constexpr int txq_slot(int s) {
  return s == 0 ? 0 : s == 1 ? 1 : s == 2 ? 2 : s == 5 ? 3 : s == 6 ? 4 : s == 7 ? 5
       : s == 8 ? 6 : s == 13 ? 7 : s == 14 ? 8
       : s == 3 ? 0 : s == 9 ? 1 : s == 10 ? 2 : s == 15 ? 3 : s == 16 ? 4 : -1;
}
static_assert(sizeof(TxqMulti) <= 4096, "kernel argument size");

constexpr int lds_bytes(int s) {
  return s == 0 ? TxqLds<4, 4>::kBytes : s == 1 ? TxqLds<8, 8>::kBytes
       : s == 2 ? TxqLds<16, 16>::kBytes : s == 3 ? TxqLds<32, 32>::kBytes
       : s == 5 ? TxqLds<4, 8>::kBytes : s == 6 ? TxqLds<8, 4>::kBytes
       : s == 7 ? TxqLds<8, 16>::kBytes : s == 8 ? TxqLds<16, 8>::kBytes
       : s == 9 ? TxqLds<16, 32>::kBytes : s == 10 ? TxqLds<32, 16>::kBytes
       : s == 13 ? TxqLds<4, 16>::kBytes : s == 14 ? TxqLds<16, 4>::kBytes
       : s == 15 ? TxqLds<8, 32>::kBytes : s == 16 ? TxqLds<32, 8>::kBytes : 0;
}
__host__ __device__ constexpr bool txq_class(int s) {  // 1: a 32-point size
  return s == 3 || s == 9 || s == 10 || s == 15 || s == 16;
}
constexpr int class_lds(int cls) {
  int m = 16;
  for (int s = 0; s < 17; ++s)
    if ((s < 4 || s > 4) && s != 11 && s != 12 && lds_bytes(s) > 0 && (txq_class(s) ? 1 : 0) == cls)
      m = lds_bytes(s) > m ? lds_bytes(s) : m;
  return m;
}

// workgroup g of a class's launch (the sizes' grids back to back)
template <int CLS>
__device__ __forceinline__ void txq_multi_body(const TxqDispatch& d, const TxqArgs& a0,
                                               const TxqArgs& a1, const TxqArgs& a2,
                                               const TxqArgs& a3, const TxqArgs& a4,
                                               const TxqArgs& a5, const TxqArgs& a6,
                                               const TxqArgs& a7, const TxqArgs& a8, int g,
                                               char* lds) {
  int code = d.code[0], id = g;
#pragma unroll
  for (int k = 1; k < kMultiMax; ++k) {  // constant indices only
    if (k < d.n && g >= d.wg0[k]) {
      code = d.code[k];
      id = g - d.wg0[k];
    }
  }
  if constexpr (CLS == 0) {
    switch (code) {
      case 0: txq_plane_body<4, 4>(a0, id, lds); break;
      case 1: txq_plane_body<8, 8>(a1, id, lds); break;
      case 2: txq_plane_body<16, 16>(a2, id, lds); break;
      case 5: txq_plane_body<4, 8>(a3, id, lds); break;
      case 6: txq_plane_body<8, 4>(a4, id, lds); break;
      case 7: txq_plane_body<8, 16>(a5, id, lds); break;
      case 8: txq_plane_body<16, 8>(a6, id, lds); break;
      case 13: txq_plane_body<4, 16>(a7, id, lds); break;
      case 14: txq_plane_body<16, 4>(a8, id, lds); break;
      default: break;
    }
  } else {
    switch (code) {
      case 3: txq_plane_body<32, 32>(a0, id, lds); break;
      case 9: txq_plane_body<16, 32>(a1, id, lds); break;
      case 10: txq_plane_body<32, 16>(a2, id, lds); break;
      case 15: txq_plane_body<8, 32>(a3, id, lds); break;
      case 16: txq_plane_body<32, 8>(a4, id, lds); break;
      default: break;
    }
  }
}

// the host side of lavish_txq_frame for one class (txq.hip): the dispatch
// table and per-size arguments of the class's sizes <= 32 points, and the
// class's grid (0: none of its sizes requested)
int txq_frame_plan(const int16_t* residual, int stride, int width, int height, uint32_t size_mask,
                   const uint32_t* type_masks, int bd, int quant_kind, const LavishQuantParams* qp,
                   int32_t* const* qcoeff, int32_t* const* dqcoeff, uint16_t* const* eob, int cls,
                   TxqMulti& m, int& grid);

// lavish_txq_frame (txq.hip)
int txq_frame(const int16_t* residual, int stride, int width, int height, uint32_t size_mask,
              const uint32_t* type_masks, int bd, int quant_kind, const LavishQuantParams* qp,
              int32_t* const* qcoeff, int32_t* const* dqcoeff, uint16_t* const* eob,
              hipStream_t caller);

}  // namespace lavish
