// txq.hip -- batched forward transform + quantization for gfx950.
//
// The reference evaluates, per TX block and per candidate TX type, av1_xform
// (av1/encoder/encodemb.c:295 -> hybrid_fwd_txfm.c:233-313 ->
// av1_fwd_txfm2d.c:56-127) followed by av1_quant (encodemb.c:308 ->
// av1_quantize.c:36-122 / aom_dsp/quantize.c:108-169), one block at a time
// on one CPU thread.  Here one 256-thread workgroup owns P = 256/min(W,H)
// blocks of one TX size and walks every requested TX type over them:
//
//   residual (HBM, read once) -> registers (one column per thread)
//   per type: column 1-D transform (registers) -> LDS t1 (padded rows)
//             row 1-D transform + fp/b quantizer + eob reduction
//                                               -> LDS t2 (coefficient order)
//             coalesced 16-byte copy-out of qcoeff, dqcoeff (recomputed from
//             qcoeff: dq = sign * ((|q| * dequant) >> log_scale))
//
// The transforms are fully unrolled straight-line integer code (txfm_dev.h);
// no MFMA: AV1 butterflies with per-stage 64-bit rounding are not a matrix
// product.  HBM traffic is the residual once plus 8 bytes per output
// coefficient per type, so the kernel is bounded by the output write stream.
#include <atomic>

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



// runtime-kind wrapper for the generic per-block quantizer kernel
template <int LS>
__device__ __forceinline__ int32_t quant_rt(int32_t c, bool ac, int kind, int highbd,
                                            const QP& qp) {
  if (kind == LAVISH_QUANT_FP)
    return highbd ? quant_one<LS, LAVISH_QUANT_FP, true>(c, ac, qp)
                  : quant_one<LS, LAVISH_QUANT_FP, false>(c, ac, qp);
  return highbd ? quant_one<LS, LAVISH_QUANT_B, true>(c, ac, qp)
                : quant_one<LS, LAVISH_QUANT_B, false>(c, ac, qp);
}

constexpr int kFrameStreams = 3;


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
          q = quant_one<LS, QK, HBD>(v, c != 0 || r != 0, a.qp);
        }
        t2[b * N + rc] = q;
        const int pos1 = iscan[rc] + 1;
        last = q != 0 ? max(last, pos1) : last;
      }
#pragma unroll
      for (int m = 1; m < H; m <<= 1) last = max(last, __shfl_xor(last, m));
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
          d4.x = dequant_one<LS>(q4.x, rc0 != 0, a.qp);  // only x can be DC
          d4.y = dequant_one<LS>(q4.y, 1, a.qp);
          d4.z = dequant_one<LS>(q4.z, 1, a.qp);
          d4.w = dequant_one<LS>(q4.w, 1, a.qp);
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

template <int W, int H>
__global__ __launch_bounds__(256, 2) void txq_plane_kernel(TxqArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[TxqLds<W, H>::kBytes];
  txq_plane_body<W, H>(a, blockIdx.x, lds);
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

template <int CLS>
__global__ __launch_bounds__(256, 2) void txq_multi_kernel(TxqDispatch d, TxqArgs a0, TxqArgs a1,
                                                           TxqArgs a2, TxqArgs a3, TxqArgs a4,
                                                           TxqArgs a5, TxqArgs a6, TxqArgs a7,
                                                           TxqArgs a8) {
  __shared__ __attribute__((aligned(16))) char lds[class_lds(CLS)];
  const int g = blockIdx.x;
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

// generic quantizer: one workgroup per block, any scan order.
template <int LS>
__global__ __launch_bounds__(256) void quant_kernel(const int32_t* coeff, int n,
                                                     const int16_t* scan, int kind,
                                                     int highbd, QP qp,
                                                     int32_t* qcoeff, int32_t* dqcoeff,
                                                     uint16_t* eob) {
  __shared__ int red[4];
  const size_t base = (size_t)blockIdx.x * n;
  const int tid = threadIdx.x;
  int last = 0;
  for (int i = tid; i < n; i += 256) {
    const int rc = scan[i];
    const int32_t q = quant_rt<LS>(coeff[base + rc], rc != 0, kind, highbd, qp);
    qcoeff[base + rc] = q;
    dqcoeff[base + rc] = dequant_one<LS>(q, rc != 0, qp);
    if (q != 0) last = max(last, i + 1);
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) last = max(last, __shfl_xor(last, m));
  if ((tid & 63) == 0) red[tid >> 6] = last;
  __syncthreads();
  if (tid == 0) eob[blockIdx.x] = (uint16_t)max(max(red[0], red[1]), max(red[2], red[3]));
}

// ----------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------
// Type chunks: one per vertical 1-D kind present (DCT, ADST, FLIPADST,
// IDTX; the 16 types are all 4 x 4 (vertical, horizontal) pairs, so a block
// needs 4 column passes, not 16), split further -- largest first -- until the
// grid has enough workgroups to give every CU several (>= ~8 per CU over 256
// CUs).  Each extra chunk re-reads the residual tile (2 bytes/pixel against
// 8 bytes/coefficient/type written) and repeats one column pass.
static void build_chunks(TxqArgs& a, int nbg) {
  int cnt = 0, sz[16] = {}, ti[16][16];
  for (int vk = 0; vk < 4; ++vk) {
    int n = 0;
    for (int i = 0; i < a.ntypes; ++i)
      if (((kVtxPacked >> (2 * a.types[i])) & 3) == (uint32_t)vk) ti[cnt][n++] = i;
    if (n) sz[cnt++] = n;
  }
  while (nbg * cnt < 2048 && cnt < 16) {
    int big = 0;
    for (int g = 1; g < cnt; ++g)
      if (sz[g] > sz[big]) big = g;
    if (sz[big] < 2) break;
    const int keep = (sz[big] + 1) / 2;
    for (int i = keep; i < sz[big]; ++i) ti[cnt][i - keep] = ti[big][i];
    sz[cnt++] = sz[big] - keep;
    sz[big] = keep;
  }
  int o = 0;
  for (int g = 0; g < cnt; ++g) {
    a.chunk_off[g] = o;
    for (int i = 0; i < sz[g]; ++i) a.chunk_ti[o++] = ti[g][i];
  }
  a.chunk_off[cnt] = o;
  a.tgroups = cnt;
}

// the grid of one size (0: nothing to do); fills the type chunks of `a`
template <int W, int H>
static int plan_plane(TxqArgs& a) {
  constexpr int P = Tile<W, H>::P * 4;  // blocks per workgroup (4 wave tiles)
  const int nbg = (a.nblocks + P - 1) / P;
  if (nbg == 0) return 0;
  build_chunks(a, nbg);
  return ((nbg + 7) / 8) * 8 * a.tgroups;
}

template <int W, int H>
static void launch_plane(TxqArgs a, hipStream_t s) {
  const int grid = plan_plane<W, H>(a);
  if (grid == 0) return;
  hipLaunchKernelGGL((txq_plane_kernel<W, H>), dim3(grid), dim3(256), 0, s, a);
  LAVISH_CHECK(hipGetLastError());
}

static int plan_size(int tx_size, TxqArgs& a) {
  switch (tx_size) {
    case 0: return plan_plane<4, 4>(a);
    case 1: return plan_plane<8, 8>(a);
    case 2: return plan_plane<16, 16>(a);
    case 3: return plan_plane<32, 32>(a);
    case 5: return plan_plane<4, 8>(a);
    case 6: return plan_plane<8, 4>(a);
    case 7: return plan_plane<8, 16>(a);
    case 8: return plan_plane<16, 8>(a);
    case 9: return plan_plane<16, 32>(a);
    case 10: return plan_plane<32, 16>(a);
    case 13: return plan_plane<4, 16>(a);
    case 14: return plan_plane<16, 4>(a);
    case 15: return plan_plane<8, 32>(a);
    case 16: return plan_plane<32, 8>(a);
    default: return -1;
  }
}

static QP to_qp(const LavishQuantParams* p) {
  QP q{};
  if (p) {
    for (int i = 0; i < 2; ++i) {
      q.zbin[i] = p->zbin[i];
      q.round[i] = p->round[i];
      q.quant[i] = p->quant[i];
      q.quant_shift[i] = p->quant_shift[i];
      q.dequant[i] = p->dequant[i];
    }
  }
  return q;
}

int txq_args(const int16_t* residual, int stride, int width, int height, int tx_size,
             uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
             int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff, TxqArgs& a);

int txq_plane(const int16_t* residual, int stride, int width, int height, int tx_size,
              uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
              int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff,
              hipStream_t s) {
  if (tx_size < 0 || tx_size >= 19) return -1;
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  if (quant_kind < 0 || quant_kind > 2) return -3;
  if (quant_kind != LAVISH_QUANT_NONE && qp == nullptr) return -3;
  if (width <= 0 || height <= 0 || stride < width) return -4;
  if (W > 32 || H > 32)  // 64-point sizes: rdo.hip, mode 0
    return txq_plane_64(residual, stride, width, height, tx_size, type_mask, bd, quant_kind, qp,
                        qcoeff, dqcoeff, eob, coeff, s);
  TxqArgs a{};
  const int rc = txq_args(residual, stride, width, height, tx_size, type_mask, bd, quant_kind,
                          qp, qcoeff, dqcoeff, eob, coeff, a);
  if (rc) return rc;
  switch (tx_size) {
    case 0: launch_plane<4, 4>(a, s); break;
    case 1: launch_plane<8, 8>(a, s); break;
    case 2: launch_plane<16, 16>(a, s); break;
    case 3: launch_plane<32, 32>(a, s); break;
    case 5: launch_plane<4, 8>(a, s); break;
    case 6: launch_plane<8, 4>(a, s); break;
    case 7: launch_plane<8, 16>(a, s); break;
    case 8: launch_plane<16, 8>(a, s); break;
    case 9: launch_plane<16, 32>(a, s); break;
    case 10: launch_plane<32, 16>(a, s); break;
    case 13: launch_plane<4, 16>(a, s); break;
    case 14: launch_plane<16, 4>(a, s); break;
    case 15: launch_plane<8, 32>(a, s); break;
    case 16: launch_plane<32, 8>(a, s); break;
    default: return -2;
  }
  return 0;
}

// TxqArgs of one (size <= 32 points, plane) job; 0 or the API's error code
int txq_args(const int16_t* residual, int stride, int width, int height, int tx_size,
             uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
             int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff, TxqArgs& a) {
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  a = TxqArgs{};
  a.res = residual;
  a.stride = stride;
  a.bw = width / W;
  a.nblocks = (width / W) * (height / H);
  for (int t = 0; t < 16; ++t) {
    if (!((type_mask >> t) & 1)) continue;
    if (!tx_type_valid(tx_size, t)) return -5;
    a.types[a.ntypes++] = t;
  }
  if (a.ntypes == 0) return -5;
  a.quant_kind = quant_kind;
  a.highbd = bd > 8;
  a.qp = to_qp(qp);
  a.iscan_default = dev_iscan(tx_size, 0);
  a.qcoeff = qcoeff;
  a.dqcoeff = dqcoeff;
  a.eob = eob;
  a.coeff = coeff;
  return 0;
}

int quantize_batch(const int32_t* coeff, int n, int nblocks, const int16_t* scan,
                   int log_scale, int bd, int quant_kind, const LavishQuantParams* qp,
                   int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, hipStream_t s) {
  if (n <= 0 || nblocks <= 0 || qp == nullptr) return -1;
  if (quant_kind != LAVISH_QUANT_FP && quant_kind != LAVISH_QUANT_B) return -3;
  const QP q = to_qp(qp);
  const int hb = bd > 8;
  switch (log_scale) {
    case 0:
      hipLaunchKernelGGL(quant_kernel<0>, dim3(nblocks), dim3(256), 0, s, coeff, n, scan,
                         quant_kind, hb, q, qcoeff, dqcoeff, eob);
      break;
    case 1:
      hipLaunchKernelGGL(quant_kernel<1>, dim3(nblocks), dim3(256), 0, s, coeff, n, scan,
                         quant_kind, hb, q, qcoeff, dqcoeff, eob);
      break;
    case 2:
      hipLaunchKernelGGL(quant_kernel<2>, dim3(nblocks), dim3(256), 0, s, coeff, n, scan,
                         quant_kind, hb, q, qcoeff, dqcoeff, eob);
      break;
    default:
      return -2;
  }
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

// Frame batch: every requested TX size over the same residual plane.  The
// per-size kernels are independent, so they are spread over the caller's
// stream plus two internal streams (forked from / joined back to the caller
// with events): register-heavy 16/32-point kernels and light 4/8-point
// kernels then share the CUs, which a single in-order stream cannot do.  The
// caller's stream takes every third kernel (the largest first) so it never
// waits on a fork; a cross-stream event wait costs tens of microseconds.
struct FrameStreams {
  int device = -1;
  hipStream_t s[kFrameStreams] = {};  // s[0] = the caller's stream (set per call)
  hipEvent_t fork = nullptr, join[kFrameStreams] = {};
};
static thread_local FrameStreams t_fs;

static FrameStreams& frame_streams() {
  int dev = 0;
  LAVISH_CHECK(hipGetDevice(&dev));
  if (t_fs.device != dev) {
    for (int i = 1; i < kFrameStreams; ++i) {
      LAVISH_CHECK(hipStreamCreateWithFlags(&t_fs.s[i], hipStreamNonBlocking));
      LAVISH_CHECK(hipEventCreateWithFlags(&t_fs.join[i], hipEventDisableTiming));
    }
    LAVISH_CHECK(hipEventCreateWithFlags(&t_fs.fork, hipEventDisableTiming));
    t_fs.device = dev;
  }
  return t_fs;
}

// streams the per-size work of lavish_rdo_frame / lavish_rdo_reconstruct is
// dealt over: kFrameStreams (the caller + internal streams), or 1 (every
// size on the caller's stream: isolated per-kernel timings under a
// profiler), set by lavish_set_fan_width
static std::atomic<int> g_fan_width{kFrameStreams};
int fan_width() { return g_fan_width.load(std::memory_order_relaxed); }
int set_fan_width(int w) {
  if (w < 1 || w > kFrameStreams) return -1;
  g_fan_width.store(w, std::memory_order_relaxed);
  return 0;
}

// fork: the internal streams wait for everything queued on `caller`; slot 0
// is the caller itself
hipStream_t* fan_out(hipStream_t caller) {
  FrameStreams& fs = frame_streams();
  fs.s[0] = caller;
  LAVISH_CHECK(hipEventRecord(fs.fork, caller));
  for (int i = 1; i < kFrameStreams; ++i) LAVISH_CHECK(hipStreamWaitEvent(fs.s[i], fs.fork, 0));
  return fs.s;
}

// join: `caller` waits for everything queued on the internal streams
void fan_in(hipStream_t caller) {
  FrameStreams& fs = frame_streams();
  for (int i = 1; i < kFrameStreams; ++i) {
    LAVISH_CHECK(hipEventRecord(fs.join[i], fs.s[i]));
    LAVISH_CHECK(hipStreamWaitEvent(caller, fs.join[i], 0));
  }
}

int txq_frame(const int16_t* residual, int stride, int width, int height, uint32_t size_mask,
              const uint32_t* type_masks, int bd, int quant_kind, const LavishQuantParams* qp,
              int32_t* const* qcoeff, int32_t* const* dqcoeff, uint16_t* const* eob,
              hipStream_t caller) {
  // order: most output bytes first, dealt round-robin over the streams
  int order[19], n = 0;
  for (int s = 0; s < 19; ++s)
    if ((size_mask >> s) & 1) order[n++] = s;
  auto work = [&](int s) {
    return (long)__builtin_popcount(type_masks[s]) * max_eob(s) * (width / tx_w(s)) *
           (height / tx_h(s));
  };
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && work(order[j]) > work(order[j - 1]); --j) {
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  int rc = 0;
  // one launch per class, on the caller's stream: the 32-point class (few,
  // register-heavy workgroups) first, then the <= 16-point class.  (Measured
  // and dropped: the round-2 per-size kernels over the caller + 2 internal
  // streams, ~50 us of fork / join per frame; the 32-point class on an
  // internal stream beside the other, C2 0.565 -> 0.577 ms,
  // profiles/r04_v5_c2_streams_ab.txt.)
  for (int cls = 1; cls >= 0; --cls) {
    const hipStream_t cs = caller;
    TxqMulti m{};
    int g = 0;
    for (int i = 0; i < n; ++i) {
      const int s = order[i];
      if ((txq_class(s) ? 1 : 0) != cls) continue;
      if (tx_w(s) > 32 || tx_h(s) > 32) {  // 64-point sizes: their own path
        rc = txq_plane(residual, stride, width, height, s, type_masks[s], bd, quant_kind, qp,
                       qcoeff[s], dqcoeff[s], eob[s], nullptr, cs);
        if (rc) break;
        continue;
      }
      if (m.d.n == kMultiMax) {
        rc = -2;
        break;
      }
      TxqArgs& a = m.a[txq_slot(s)];
      rc = txq_args(residual, stride, width, height, s, type_masks[s], bd, quant_kind, qp,
                    qcoeff[s], dqcoeff[s], eob[s], nullptr, a);
      if (rc) break;
      const int grid = plan_size(s, a);
      if (grid <= 0) continue;
      m.d.code[m.d.n] = s;
      m.d.wg0[m.d.n] = g;
      g += grid;
      ++m.d.n;
    }
    if (rc) break;
    if (m.d.n == 0) continue;
    m.d.wg0[m.d.n] = g;
    // (Measured and dropped: an LDS pad so fewer C2 workgroups fit a CU
    // beside a concurrent leg -- C2 alone 0.51 -> 0.55 / 1.31 ms at 3 / 2
    // workgroups per CU, profiles/r04_v11_ab_notes.txt.)
    if (cls == 0)
      hipLaunchKernelGGL(txq_multi_kernel<0>, dim3(g), dim3(256), 0, cs, m.d, m.a[0], m.a[1],
                         m.a[2], m.a[3], m.a[4], m.a[5], m.a[6], m.a[7], m.a[8]);
    else
      hipLaunchKernelGGL(txq_multi_kernel<1>, dim3(g), dim3(256), 0, cs, m.d, m.a[0], m.a[1],
                         m.a[2], m.a[3], m.a[4], m.a[5], m.a[6], m.a[7], m.a[8]);
    LAVISH_CHECK(hipGetLastError());
  }
  return rc;
}

}  // namespace lavish

extern "C" int lavish_set_fan_width(int streams) { return lavish::set_fan_width(streams); }

extern "C" int lavish_txq_frame(const int16_t* residual, int stride, int width, int height,
                                uint32_t size_mask, const uint32_t* type_masks, int bit_depth,
                                int quant_kind, const LavishQuantParams* qp,
                                int32_t* const* qcoeff, int32_t* const* dqcoeff,
                                uint16_t* const* eob, void* stream) {
  return lavish::txq_frame(residual, stride, width, height, size_mask, type_masks, bit_depth,
                           quant_kind, qp, qcoeff, dqcoeff, eob, (hipStream_t)stream);
}

extern "C" int lavish_txq_plane(const int16_t* residual, int stride, int width, int height,
                                int tx_size, uint32_t type_mask, int bit_depth,
                                int quant_kind, const LavishQuantParams* qp,
                                int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob,
                                int32_t* coeff, void* stream) {
  return lavish::txq_plane(residual, stride, width, height, tx_size, type_mask, bit_depth,
                           quant_kind, qp, qcoeff, dqcoeff, eob, coeff,
                           (hipStream_t)stream);
}

extern "C" int lavish_quantize_batch(const int32_t* coeff, int n, int nblocks,
                                     const int16_t* scan, const int16_t* iscan,
                                     int log_scale, int bit_depth, int quant_kind,
                                     const LavishQuantParams* qp, int32_t* qcoeff,
                                     int32_t* dqcoeff, uint16_t* eob, void* stream) {
  (void)iscan;  // the reference quantizers walk `scan` only
  return lavish::quantize_batch(coeff, n, nblocks, scan, log_scale, bit_depth, quant_kind,
                                qp, qcoeff, dqcoeff, eob, (hipStream_t)stream);
}
