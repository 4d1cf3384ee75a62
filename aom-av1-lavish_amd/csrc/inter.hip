// inter.hip -- batched single-reference inter prediction for gfx950
// ("its prediction output feeds C4").
//
// Reference (one block per call, one CPU thread):
//   av1_enc_build_one_inter_predictor (av1/encoder/reconinter_enc.c:47-51)
//   -> enc_calc_subpel_params / init_subpel_params (av1/common/reconinter.h:
//      131-165): q10 position of the block + mv, clamped to the frame's
//      border window, split into an integer pixel and a 1/16 phase
//   -> av1_get_interp_filter_params_with_block_size (filter.h:253-259):
//      4-tap kernels for block dimensions <= 4
//   -> convolve_2d_facade_single (convolve.c:614-634, highbd :1106-1128):
//      copy / av1_convolve_x_sr / _y_sr / _2d_sr with the single-prediction
//      rounding of get_conv_params_no_round (convolve.h:63-95).
//
// Here a job is one (block, mv, filter pair); a thread owns CW adjacent
// output columns x R rows of one job.  It reads each source row segment it
// needs (CW + 7 pixels) with dword-aligned loads + v_alignbyte, runs the
// horizontal pass in registers, keeps the R + 7 intermediate rows of its
// columns in VGPRs and finishes the vertical pass there -- no LDS, no
// barrier; adjacent threads read adjacent bytes, so a wave's loads coalesce
// and the (w + 7) x (h + 7) source window of a block is fetched from HBM
// about once (the overlap hits L2: consecutive jobs share an XCD).  12-tap
// kernels (MULTITAP_SHARP2, temporal filtering only) take a direct,
// per-pixel path.
#include "interp_kernels.h"
#include "lavish_internal.h"

namespace lavish {
namespace {

struct IJob {
  int64_t ref_off, dst_off;
  int32_t pix_row, pix_col;
  int16_t mv_row, mv_col;
  uint8_t filter_x, filter_y, pad[2];
};
static_assert(sizeof(IJob) == sizeof(LavishInterPredJob) && sizeof(IJob) == 32, "job layout");

// filter.h:111-243 (interp_kernels.h)
__constant__ int16_t kK8[6][16][8] = LAVISH_K8_INIT;

// MULTITAP_SHARP2
__constant__ int16_t kK12[16][12] = LAVISH_K12_INIT;

struct IpArgs {
  const void* ref;
  int64_t rs;
  int fw, fh, ssx, ssy, w, h;
  const IJob* jobs;
  const LavishSubpelResult* mvs;  // optional mv override
  int njobs;
  void* dst;
  int64_t ds;
  int bd, r0, r1;
  // RTCD shims: the caller's own kernels and path (kCustom layout); the
  // job's ref_off is then the block's integer position
  const int16_t* custom;
};
enum { kCPath = 0, kCTx = 1, kCTy = 2, kCFx = 4, kCFy = 16, kCustomLen = 28 };

typedef const __attribute__((address_space(1))) uint32_t* gptr;
typedef uint32_t u4a __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ int rpot(int v, int n) { return (v + ((1 << n) >> 1)) >> n; }
__device__ __forceinline__ int clip_bd(int v, int mx) { return v < 0 ? 0 : v > mx ? mx : v; }

// NP consecutive pixels starting at p (any alignment), from dword-aligned
// loads; reads up to 4 bytes either side of the span (inside the border)
template <int NP>
__device__ __forceinline__ void load_px(const uint8_t* p, int (&o)[NP]) {
  const uintptr_t a = (uintptr_t)p;
  const gptr q = (gptr)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  constexpr int NE = (NP + 3) / 4;
  uint32_t d[NE + 1];
#pragma unroll
  for (int i = 0; i <= NE; ++i) d[i] = q[i];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const uint32_t e = __builtin_amdgcn_alignbyte(d[(j >> 2) + 1], d[j >> 2], sh);
    o[j] = (int)((e >> (8 * (j & 3))) & 0xFFu);
  }
}
template <int NP>
__device__ __forceinline__ void load_px(const uint16_t* p, int (&o)[NP]) {
  const uintptr_t a = (uintptr_t)p;
  const gptr q = (gptr)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 2);
  constexpr int NE = (NP + 1) / 2;
  uint32_t d[NE + 1];
#pragma unroll
  for (int i = 0; i <= NE; ++i) d[i] = q[i];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const uint32_t e = __builtin_amdgcn_alignbyte(d[(j >> 1) + 1], d[j >> 1], sh);
    o[j] = (int)((e >> (16 * (j & 1))) & 0xFFFFu);
  }
}

template <int CW>
__device__ __forceinline__ void store_px(uint8_t* p, const int (&v)[CW]) {
  const uintptr_t a = (uintptr_t)p;
  if constexpr (CW == 4) {
    if ((a & 3) == 0) {
      *(uint32_t*)p = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) |
                      ((uint32_t)v[3] << 24);
      return;
    }
  } else {
    if ((a & 1) == 0) {
      *(uint16_t*)p = (uint16_t)(v[0] | (v[1] << 8));
      return;
    }
  }
#pragma unroll
  for (int c = 0; c < CW; ++c) p[c] = (uint8_t)v[c];
}
template <int CW>
__device__ __forceinline__ void store_px(uint16_t* p, const int (&v)[CW]) {
  const uintptr_t a = (uintptr_t)p;
  if ((a & 3) == 0) {
#pragma unroll
    for (int c = 0; c < CW; c += 2)
      *(uint32_t*)(p + c) = (uint32_t)v[c] | ((uint32_t)v[c + 1] << 16);
    return;
  }
#pragma unroll
  for (int c = 0; c < CW; ++c) p[c] = (uint16_t)v[c];
}

template <typename T>
__device__ __forceinline__ int px(const T* p, int64_t i) {
  return (int)p[i];
}

// direct per-pixel evaluation for any tap count (12-tap kernels)
template <typename T, int CW, int R>
__device__ void generic_block(const T* src, int64_t rs, T* dst, int64_t ds, int path,
                              const int16_t* fx, int tx, const int16_t* fy, int ty, int bd,
                              int r0, int r1) {
  const int mx = (1 << bd) - 1;
  const int foh = tx / 2 - 1, fov = ty / 2 - 1;
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < CW; ++c) {
      int v;
      if (path == 0) {
        v = px(src, r * rs + c);
      } else if (path == 1) {
        int s = 0;
        for (int k = 0; k < tx; ++k) s += fx[k] * px(src, r * rs + c - foh + k);
        v = clip_bd(rpot(rpot(s, r0), 7 - r0), mx);
      } else if (path == 2) {
        int s = 0;
        for (int k = 0; k < ty; ++k) s += fy[k] * px(src, (r - fov + k) * rs + c);
        v = clip_bd(rpot(s, 7), mx);
      } else {
        const int ob = bd + 14 - r0;
        int s = 1 << ob;
        for (int k = 0; k < ty; ++k) {
          int hs = 1 << (bd + 6);
          for (int m = 0; m < tx; ++m) hs += fx[m] * px(src, (r - fov + k) * rs + c - foh + m);
          s += fy[k] * (int)(int16_t)rpot(hs, r0);
        }
        const int res = rpot(s, r1) - ((1 << (ob - r1)) + (1 << (ob - r1 - 1)));
        v = clip_bd(rpot(res, 14 - r0 - r1), mx);
      }
      dst[r * ds + c] = (T)v;
    }
}

// 4 negated taps as packed signed bytes (every 8-tap kernel's negation fits
// i8: the taps lie in [-24, 128])
__device__ __forceinline__ int pack_neg4(const int16_t* f) {
  return (int)((uint32_t)(uint8_t)(-f[0]) | ((uint32_t)(uint8_t)(-f[1]) << 8) |
               ((uint32_t)(uint8_t)(-f[2]) << 16) | ((uint32_t)(uint8_t)(-f[3]) << 24));
}

// u8 prediction with the default rounding (round_0 3, round_1 11, bd 8)
// through the 2-D form for every phase: with the phase-0 kernel (128 at the
// centre) the 2-D rounding reduces exactly to the x-only / y-only / copy
// results (im = 16 p + 2^11 or rpot(s, 3) + 2^11; the vertical offsets
// cancel), so one branch-free path serves all four facade cases.
// Horizontal taps run as v_dot4_i32_i8 on (p - 128) bytes against the
// negated kernel: sum f p = 128 * 128 - dot(-f, p - 128).
template <int R>
__device__ __forceinline__ void u8_2d(const uint8_t* src, int64_t rs, uint8_t* dst, int64_t ds,
                                      const int16_t* fx, const int16_t* fy) {
  const int nlo = pack_neg4(fx), nhi = pack_neg4(fx + 4);
  int ky[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) ky[k] = fy[k];
  constexpr int kC1 = 16384 + (1 << 14) + 4;  // 128 * 128 + 2^(bd + 6) + rounding of >> 3
  int im[R + 7][4];
#pragma unroll
  for (int i = 0; i < R + 7; ++i) {
    const uintptr_t ad = (uintptr_t)(src + (i - 3) * rs - 3);
    const gptr q = (gptr)(ad & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(ad & 3);
    // one 16-byte load per row (4-byte aligned: the hardware's unaligned
    // mode serves it; a quarter of the vector-memory instructions)
    const u4a v = *(const __attribute__((address_space(1))) u4a*)q;
    const uint32_t d0 = v.x, d1 = v.y, d2 = v.z, d3 = v.w;
    const uint32_t e0 = __builtin_amdgcn_alignbyte(d1, d0, sh) ^ 0x80808080u;
    const uint32_t e1 = __builtin_amdgcn_alignbyte(d2, d1, sh) ^ 0x80808080u;
    const uint32_t e2 = __builtin_amdgcn_alignbyte(d3, d2, sh) ^ 0x80808080u;
    const int w[8] = {(int)e0,
                      (int)__builtin_amdgcn_alignbyte(e1, e0, 1),
                      (int)__builtin_amdgcn_alignbyte(e1, e0, 2),
                      (int)__builtin_amdgcn_alignbyte(e1, e0, 3),
                      (int)e1,
                      (int)__builtin_amdgcn_alignbyte(e2, e1, 1),
                      (int)__builtin_amdgcn_alignbyte(e2, e1, 2),
                      (int)__builtin_amdgcn_alignbyte(e2, e1, 3)};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int t = __builtin_amdgcn_sdot4(nhi, w[c + 4], __builtin_amdgcn_sdot4(nlo, w[c], 0, false),
                                           false);
      im[i][c] = (kC1 - t) >> 3;
    }
  }
  // vertical: rpot(s, 11) - offsets folded into the accumulator's start;
  // the im rows (int16 for u8 input) pair up as (2i, 2i+1) / (2i+1, 2i+2)
  // for v_dot2_i32_i16 against the tap pairs
  constexpr int kOb = 8 + 14 - 3;
  constexpr int kVoff = (1 << (kOb - 11)) + (1 << (kOb - 12));
  constexpr int kVinit = (1 << kOb) + (1 << 10) - (kVoff << 11);
  typedef short s2 __attribute__((ext_vector_type(2)));
  s2 kp[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) kp[m] = s2{(short)ky[2 * m], (short)ky[2 * m + 1]};
  constexpr int NP = (R + 7) / 2 + 1;  // (2i, 2i+1) pairs covering rows 0 .. R + 6
  uint32_t pe[NP][4];
#pragma unroll
  for (int i = 0; i < NP; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t lo = 2 * i < R + 7 ? (uint32_t)im[2 * i][c] : 0u;
      const uint32_t hi = 2 * i + 1 < R + 7 ? (uint32_t)im[2 * i + 1][c] : 0u;
      pe[i][c] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
    }
  // output rows as packed bytes, stored after the loop (one alignment test)
  uint32_t ow[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint32_t w = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      int s = kVinit;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int i = (r >> 1) + m;
        // odd rows pair (2i+1, 2i+2): the upper half of pair i + lower of i+1
        const uint32_t pr =
            (r & 1) ? __builtin_amdgcn_alignbyte(pe[i + 1][c], pe[i][c], 2) : pe[i][c];
        s = __builtin_amdgcn_sdot2(kp[m], __builtin_bit_cast(s2, pr), s, false);
      }
      w |= (uint32_t)clip_bd(s >> 11, 255) << (8 * c);
    }
    ow[r] = w;
  }
  if ((((uintptr_t)dst | (uintptr_t)ds) & 3) == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) *(uint32_t*)(dst + r * ds) = ow[r];
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[r * ds + c] = (uint8_t)(ow[r] >> (8 * c));
  }
}

template <typename T, int CW, int R, bool FAST>
__global__ __launch_bounds__(256) void inter_kernel(IpArgs a) {
  const int ncg = a.w / CW;
  const int tpj = ncg * (a.h / R);
  // XCD-aware: consecutive jobs (neighbouring blocks, overlapping source
  // windows) land on the same XCD's L2
  const int nwg = gridDim.x;  // multiple of 8
  const int wg = (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  const uint32_t gid = (uint32_t)wg * 256u + threadIdx.x;  // < 2^31 (host check)
  const uint32_t j = gid / (uint32_t)tpj;
  if (j >= (uint32_t)a.njobs) return;
  const int sub = (int)(gid - j * (uint32_t)tpj);
  const int rsi = sub / ncg, cg = sub - rsi * ncg;
  const IJob jb = a.jobs[j];
  const T* src;
  int path, tx, ty;
  const int16_t *fx, *fy;
  if (a.custom) {
    src = (const T*)a.ref + jb.ref_off;
    path = a.custom[kCPath];
    tx = a.custom[kCTx];
    ty = a.custom[kCTy];
    fx = a.custom + kCFx;
    fy = a.custom + kCFy;
  } else {
    int mvr = jb.mv_row, mvc = jb.mv_col;
    if (a.mvs) {
      mvr = a.mvs[j].best_row;
      mvc = a.mvs[j].best_col;
    }
    // init_subpel_params (unscaled): q4 -> q10 (+ SCALE_EXTRA_OFF), clamp
    int pos_y = ((jb.pix_row << 4) + mvr * (1 << (1 - a.ssy))) * 64 + 32;
    int pos_x = ((jb.pix_col << 4) + mvc * (1 << (1 - a.ssx))) * 64 + 32;
    const int top = -(((288 >> a.ssy) - 4) << 10), left = -(((288 >> a.ssx) - 4) << 10);
    pos_y = min(max(pos_y, top), (a.fh + 4) << 10);
    pos_x = min(max(pos_x, left), (a.fw + 4) << 10);
    const int sx = (pos_x & 1023) >> 6, sy = (pos_y & 1023) >> 6;
    src = (const T*)a.ref + jb.ref_off + (int64_t)(pos_y >> 10) * a.rs + (pos_x >> 10);
    path = (sx ? 1 : 0) + (sy ? 2 : 0);
    // av1_get_interp_filter_params_with_block_size
    const int f_x = jb.filter_x, f_y = jb.filter_y;
    const int kx = a.w <= 4 ? (f_x == 1 ? 5 : f_x == 3 ? 3 : 4) : f_x;
    const int ky = a.h <= 4 ? (f_y == 1 ? 5 : f_y == 3 ? 3 : 4) : f_y;
    // a direction at phase 0 is not filtered: the 8-tap identity row stands
    // in for it (the FAST path runs every job through the 2-D form)
    const bool x12 = f_x == 4 && sx, y12 = f_y == 4 && sy;
    tx = x12 ? 12 : 8;
    ty = y12 ? 12 : 8;
    fx = x12 ? kK12[sx] : kK8[kx > 5 ? 0 : kx][sx];
    fy = y12 ? kK12[sy] : kK8[ky > 5 ? 0 : ky][sy];
  }
  src += (int64_t)(rsi * R) * a.rs + cg * CW;
  T* dst = (T*)a.dst + jb.dst_off + (int64_t)(rsi * R) * a.ds + cg * CW;
  const int mx = (1 << a.bd) - 1;
  const bool wide = ((path & 1) && tx != 8) || ((path & 2) && ty != 8);
  if (wide) {
    generic_block<T, CW, R>(src, a.rs, dst, a.ds, path, fx, tx, fy, ty, a.bd, a.r0, a.r1);
    return;
  }
  if constexpr (FAST) {
    u8_2d<R>((const uint8_t*)src, a.rs, (uint8_t*)dst, a.ds, fx, fy);
    return;
  } else {
    int kx[8], ky[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      kx[k] = fx[k];
      ky[k] = fy[k];
    }
    if (path == 0) {  // aom_convolve_copy
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int p[CW];
        load_px<CW>(src + r * a.rs, p);
        store_px<CW>(dst + r * a.ds, p);
      }
    } else if (path == 1) {  // av1_convolve_x_sr
      const int r0 = a.r0, bits = 7 - a.r0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int p[CW + 7], o[CW];
        load_px<CW + 7>(src + r * a.rs - 3, p);
#pragma unroll
        for (int c = 0; c < CW; ++c) {
          int s = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) s += kx[k] * p[c + k];
          o[c] = clip_bd(rpot(rpot(s, r0), bits), mx);
        }
        store_px<CW>(dst + r * a.ds, o);
      }
    } else if (path == 2) {  // av1_convolve_y_sr
      int col[R + 7][CW];
#pragma unroll
      for (int i = 0; i < R + 7; ++i) load_px<CW>(src + (i - 3) * a.rs, col[i]);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int o[CW];
#pragma unroll
        for (int c = 0; c < CW; ++c) {
          int s = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) s += ky[k] * col[r + k][c];
          o[c] = clip_bd(rpot(s, 7), mx);
        }
        store_px<CW>(dst + r * a.ds, o);
      }
    } else {  // av1_convolve_2d_sr
      const int r0 = a.r0, r1 = a.r1, bits = 14 - r0 - r1;
      const int hoff = 1 << (a.bd + 6);
      const int ob = a.bd + 14 - r0;
      const int voff = (1 << (ob - r1)) + (1 << (ob - r1 - 1));
      int im[R + 7][CW];
#pragma unroll
      for (int i = 0; i < R + 7; ++i) {
        int p[CW + 7];
        load_px<CW + 7>(src + (i - 3) * a.rs - 3, p);
#pragma unroll
        for (int c = 0; c < CW; ++c) {
          int s = hoff;
#pragma unroll
          for (int k = 0; k < 8; ++k) s += kx[k] * p[c + k];
          im[i][c] = (int)(int16_t)rpot(s, r0);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int o[CW];
#pragma unroll
        for (int c = 0; c < CW; ++c) {
          int s = 1 << ob;
#pragma unroll
          for (int k = 0; k < 8; ++k) s += ky[k] * im[r + k][c];
          o[c] = clip_bd(rpot(rpot(s, r1) - voff, bits), mx);
        }
        store_px<CW>(dst + r * a.ds, o);
      }
    }
  }
}

template <typename T, int CW>
void launch_cw(const IpArgs& a, hipStream_t s) {
  constexpr bool kFastOk = sizeof(T) == 1 && CW == 4;
  const bool fast = kFastOk && !a.custom;
  // rows per thread: 16 amortises the 7 extra horizontal rows better than 8
  // (which would keep more waves resident)
  const int R = a.h < 8 ? a.h : (fast && a.h >= 16 ? 16 : 8);
  const int64_t threads = (int64_t)a.njobs * (a.w / CW) * (a.h / R);
  if (threads >= (1LL << 31) - 256 * 8) {
    set_error("lavish_build_inter_pred_batch: job list too large for one launch",
              hipErrorInvalidValue, __FILE__, __LINE__);
    return;
  }
  const int nwg = (int)(((threads + 255) / 256 + 7) & ~7LL);
  if (fast) {
    if (R == 16)
      hipLaunchKernelGGL((inter_kernel<T, CW, 16, kFastOk>), dim3(nwg), dim3(256), 0, s, a);
    else if (R == 8)
      hipLaunchKernelGGL((inter_kernel<T, CW, 8, kFastOk>), dim3(nwg), dim3(256), 0, s, a);
    else if (R == 4)
      hipLaunchKernelGGL((inter_kernel<T, CW, 4, kFastOk>), dim3(nwg), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((inter_kernel<T, CW, 2, kFastOk>), dim3(nwg), dim3(256), 0, s, a);
  } else if (R == 8) {
    hipLaunchKernelGGL((inter_kernel<T, CW, 8, false>), dim3(nwg), dim3(256), 0, s, a);
  } else if (R == 4) {
    hipLaunchKernelGGL((inter_kernel<T, CW, 4, false>), dim3(nwg), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((inter_kernel<T, CW, 2, false>), dim3(nwg), dim3(256), 0, s, a);
  }
  LAVISH_CHECK(hipGetLastError());
}

template <typename T>
void launch_t(const IpArgs& a, hipStream_t s) {
  if (a.w == 2)
    launch_cw<T, 2>(a, s);
  else
    launch_cw<T, 4>(a, s);
}

bool pow2_size(int v) { return v >= 2 && v <= 128 && (v & (v - 1)) == 0; }

// get_conv_params_no_round(0, plane, NULL, 0, 0, bd)
void conv_rounds(int bd, int& r0, int& r1) {
  r0 = 3;
  r1 = 14 - 3;
  const int ibr = bd + 7 - r0 + 2;
  if (ibr > 16) {
    r0 += ibr - 16;
    r1 -= ibr - 16;
  }
}

}  // namespace

int inter_pred_batch(const void* ref, int ref_stride, int ref_width, int ref_height, int ss_x,
                     int ss_y, int w, int h, const LavishInterPredJob* jobs, int njobs,
                     const LavishSubpelResult* mvs, void* dst, int dst_stride, int bd, int highbd,
                     const int16_t* custom, int r0, int r1, hipStream_t s) {
  if (!pow2_size(w) || !pow2_size(h)) return -3;
  if (ss_x < 0 || ss_x > 1 || ss_y < 0 || ss_y > 1) return -1;
  if (highbd ? (bd != 8 && bd != 10 && bd != 12) : bd != 8) return -1;
  if (ref_width < 0 || ref_height < 0) return -4;
  if (njobs < 0) return -4;
  if (njobs == 0) return 0;
  IpArgs a;
  a.ref = ref;
  a.rs = ref_stride;
  a.fw = ref_width;
  a.fh = ref_height;
  a.ssx = ss_x;
  a.ssy = ss_y;
  a.w = w;
  a.h = h;
  a.jobs = (const IJob*)jobs;
  a.mvs = mvs;
  a.njobs = njobs;
  a.dst = dst;
  a.ds = dst_stride;
  a.bd = bd;
  if (custom) {
    a.r0 = r0;
    a.r1 = r1;
  } else {
    conv_rounds(bd, a.r0, a.r1);
  }
  a.custom = custom;
  if (highbd)
    launch_t<uint16_t>(a, s);
  else
    launch_t<uint8_t>(a, s);
  return 0;
}

}  // namespace lavish

using namespace lavish;

extern "C" int lavish_build_inter_pred_batch(const void* ref, int ref_stride, int ref_width,
                                             int ref_height, int ss_x, int ss_y, int w, int h,
                                             const LavishInterPredJob* jobs, int njobs,
                                             void* dst, int dst_stride, int bit_depth, int highbd,
                                             void* stream) {
  return inter_pred_batch(ref, ref_stride, ref_width, ref_height, ss_x, ss_y, w, h, jobs, njobs,
                          nullptr, dst, dst_stride, bit_depth, highbd, nullptr, 0, 0,
                          (hipStream_t)stream);
}

extern "C" int lavish_build_inter_pred_after_subpel(const void* ref, int ref_stride,
                                                    int ref_width, int ref_height, int ss_x,
                                                    int ss_y, int w, int h,
                                                    const LavishInterPredJob* jobs,
                                                    const LavishSubpelResult* mvs, int njobs,
                                                    void* dst, int dst_stride, int bit_depth,
                                                    int highbd, void* stream) {
  if (!mvs) return -4;
  return inter_pred_batch(ref, ref_stride, ref_width, ref_height, ss_x, ss_y, w, h, jobs, njobs,
                          mvs, dst, dst_stride, bit_depth, highbd, nullptr, 0, 0,
                          (hipStream_t)stream);
}

// Host copy of the same kernels: av1_get_interp_filter_params_with_block_size
// (av1/common/filter.h:253-259) as data -- the kernel rows a caller puts in
// LavishInterpFilterParams::filter_ptr for (interp_filter, block dimension).
static const int16_t kK8Host[6][16][8] = LAVISH_K8_INIT;
static const int16_t kK12Host[16][12] = LAVISH_K12_INIT;

extern "C" int lavish_interp_kernels(int interp_filter, int size, int16_t* out) {
  if (interp_filter < 0 || interp_filter > 4 || size <= 0 || out == nullptr) return -1;
  if (interp_filter == 4) {  // MULTITAP_SHARP2: 12 taps at every size
    for (int p = 0; p < 16; ++p)
      for (int k = 0; k < 12; ++k) out[p * 12 + k] = kK12Host[p][k];
    return 12;
  }
  // av1_interp_4tap for sizes <= 4: REGULAR / SMOOTH / SHARP(-> REGULAR 4) / BILINEAR
  static const int k4[4] = {4, 5, 4, 3};
  const int kind = size <= 4 ? k4[interp_filter] : interp_filter;
  for (int p = 0; p < 16; ++p)
    for (int k = 0; k < 8; ++k) out[p * 8 + k] = kK8Host[kind][p][k];
  return 8;
}

