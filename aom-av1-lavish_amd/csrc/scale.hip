// scale.hip -- the scaled convolution on gfx950 (the
// inter predictor of a reference of another resolution).
//
// Reference: av1_convolve_2d_scale_c / av1_highbd_convolve_2d_scale_c
// (av1/common/convolve.c:488-574, 992-1078), reached through
// convolve_2d_scale_wrapper (:576-588) when the reference is scaled.  Output
// pixel (x, y) sits at position subpel_x_qn + x * x_step_qn (1/1024 pel,
// SCALE_SUBPEL_BITS) horizontally and subpel_y_qn + y * y_step_qn
// vertically; the kernel phase of a position is its top 4 sub-pel bits.  The
// horizontal pass filters im_h = ((h - 1) * y_step_qn + subpel_y_qn >> 10) +
// taps rows of w outputs into an int16 intermediate (rounded by round_0);
// the vertical pass walks it at the vertical positions, rounds by round_1
// into the CONV_BUF value and finishes as the reference does: the single
// prediction (offset removed, rounded, clipped), or the compound first pass
// (the CONV_BUF stored) / average (plain or distance-weighted with the
// buffer, then offset, round, clip).
//
// Blocks per 256-thread workgroup: NB = 256 / (w h) for blocks below 256
// pixels (16 for 4x4, capped), one otherwise; each block's slice of the
// workgroup (256 / NB threads) runs the horizontal pass into the block's LDS
// intermediate, a barrier, then the vertical pass.  The kernel is
// instantiated per tap count pair (TX, TY) in {(8, 8), (12, 12), (4, 4),
// (4, 8), (8, 4), (2, 2)} (0, 0: any count at run time): the tap loops
// unroll, a horizontal output's TX source pixels come in one byte-addressed
// vector load (8 u8 = one dwordx2, 8 u16 = one dwordx4; the runtime-bound
// loop issued one dependent load per tap), and the 16 kernel rows of the
// caller's filters sit in LDS (32-byte rows: one ds_read_b128 per 8 taps).
// Steps up to 2048 (the 2:1 downscale limit of av1_is_valid_scale) bound the
// intermediate at 2 h + taps rows.
#include "lavish_internal.h"

namespace lavish {
namespace {

constexpr int kFBits = 7;      // FILTER_BITS
constexpr int kScaleBits = 10; // SCALE_SUBPEL_BITS
constexpr int kScaleExtra = 6; // SCALE_EXTRA_BITS
constexpr int kMaxTaps = 12;
constexpr int kMaxStep = 2048;

struct ScaleArgs {
  const void* src;
  void* dst;
  uint16_t* conv;
  const LavishScaleJob* jobs;
  int src_stride, dst_stride, conv_stride, w, h, lw, njobs, bd;
  int tx, ty;
  int nb, im_cap;  // blocks per workgroup, int16 slots of one block's intermediate
  int16_t fx[16][kMaxTaps], fy[16][kMaxTaps];
  int r0, r1, offset_bits, round_offset, round_bits, is_compound, do_average, dist_wtd, fwd, bck;
};

constexpr int kFRow = 16;  // LDS kernel row stride (int16): 32 bytes

// the T source pixels p[0 .. T - 1] of one tap window, one vector load where
// T is fixed (byte-addressed: the queues run in unaligned-access mode)
template <typename Pix, int T>
__device__ __forceinline__ void load_taps(const Pix* p, int (&v)[T]) {
  if constexpr (sizeof(Pix) == 1 && T == 8) {
    const u32x2u d = *(const u32x2u*)p;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (d[k >> 2] >> (8 * (k & 3))) & 0xFF;
  } else if constexpr (sizeof(Pix) == 1 && T == 12) {
    const u32x2u d = *(const u32x2u*)p;
    const uint32_t e = *(const u32u*)(p + 8);
#pragma unroll
    for (int k = 0; k < 12; ++k) v[k] = ((k < 8 ? d[k >> 2] : e) >> (8 * (k & 3))) & 0xFF;
  } else if constexpr (sizeof(Pix) == 1 && T == 4) {
    const uint32_t d = *(const u32u*)p;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (d >> (8 * k)) & 0xFF;
  } else if constexpr (sizeof(Pix) == 2 && T == 8) {
    const u32x4u d = *(const u32x4u*)p;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (d[k >> 1] >> (16 * (k & 1))) & 0xFFFF;
  } else if constexpr (sizeof(Pix) == 2 && T == 12) {
    const u32x4u d = *(const u32x4u*)p;
    const u32x2u e = *(const u32x2u*)(p + 8);
#pragma unroll
    for (int k = 0; k < 12; ++k)
      v[k] = ((k < 8 ? d[k >> 1] : e[(k - 8) >> 1]) >> (16 * (k & 1))) & 0xFFFF;
  } else if constexpr (sizeof(Pix) == 2 && T == 4) {
    const u32x2u d = *(const u32x2u*)p;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (d[k >> 1] >> (16 * (k & 1))) & 0xFFFF;
  } else {
#pragma unroll
    for (int k = 0; k < T; ++k) v[k] = p[k];
  }
}

template <typename Pix, int T>
__device__ __forceinline__ int32_t taps_dot(const Pix* p, const int16_t* f, int32_t s) {
  int v[T];
  load_taps<Pix, T>(p, v);
#pragma unroll
  for (int k = 0; k < T; ++k) s += f[k] * v[k];
  return s;
}

template <typename Pix, int TX, int TY>
__global__ __launch_bounds__(256) void scale_kernel(ScaleArgs a) {
  extern __shared__ __attribute__((aligned(16))) int16_t lds[];
  int16_t* fxs = lds;                 // [16][kFRow]
  int16_t* fys = lds + 16 * kFRow;    // [16][kFRow]
  const int t = threadIdx.x;
  for (int e = t; e < 2 * 16 * kFRow; e += 256) {
    const int tab = e / (16 * kFRow), r = (e / kFRow) & 15, k = e % kFRow;
    lds[e] = k < kMaxTaps ? (tab ? a.fy[r][k] : a.fx[r][k]) : 0;
  }
  const int nb = a.nb, tpb = 256 / nb;
  const int slot = t / tpb, tb = t - slot * tpb;
  const int job = blockIdx.x * nb + slot;
  int16_t* im = lds + 2 * 16 * kFRow + slot * a.im_cap;
  const int w = a.w, h = a.h, lw = a.lw;
  const int tx = TX ? TX : a.tx, ty = TY ? TY : a.ty;
  LavishScaleJob jb{};
  if (job < a.njobs) jb = a.jobs[job];
  const int xs = jb.x_step_qn, ys = jb.y_step_qn, spx = jb.subpel_x_qn, spy = jb.subpel_y_qn;
  // (outside the supported steps the block is left alone: its intermediate
  // would not fit the launch's LDS; a slot past the batch does nothing)
  const bool valid = job < a.njobs && xs >= 1 && xs <= kMaxStep && ys >= 1 && ys <= kMaxStep &&
                     spx >= 0 && spy >= 0 && spx <= (1 << kScaleBits) - 1 &&
                     spy <= (1 << kScaleBits) - 1;
  __syncthreads();  // the kernel rows
  const Pix* src = (const Pix*)a.src + jb.src_off;
  const int im_h = (((h - 1) * ys + spy) >> kScaleBits) + ty;
  const int fo_y = ty / 2 - 1, fo_x = tx / 2 - 1;
  // horizontal filter (convolve.c:509-527): im_h rows from fo_y above the block
  if (valid) {
    for (int e = tb; e < im_h * w; e += tpb) {
      const int y = e >> lw, x = e & (w - 1);
      const int x_qn = spx + x * xs;
      const Pix* p = src + (int64_t)(y - fo_y) * a.src_stride + (x_qn >> kScaleBits) - fo_x;
      const int16_t* f = fxs + ((x_qn & ((1 << kScaleBits) - 1)) >> kScaleExtra) * kFRow;
      int32_t s = 1 << (a.bd + kFBits - 1);
      if constexpr (TX != 0) {
        s = taps_dot<Pix, TX>(p, f, s);
      } else {
        for (int k = 0; k < tx; ++k) s += f[k] * (int)p[k];
      }
      im[e] = (int16_t)((s + ((1 << a.r0) >> 1)) >> a.r0);
    }
  }
  __syncthreads();
  if (!valid) return;
  // vertical filter and the finish (:530-573)
  Pix* dst = (Pix*)a.dst + jb.dst_off;
  uint16_t* conv = a.conv + jb.conv_off;
  const int pmax = (1 << a.bd) - 1;
  for (int e = tb; e < h * w; e += tpb) {
    const int y = e >> lw, x = e & (w - 1);
    const int y_qn = spy + y * ys;
    const int16_t* f = fys + ((y_qn & ((1 << kScaleBits) - 1)) >> kScaleExtra) * kFRow;
    const int16_t* col = im + ((y_qn >> kScaleBits) << lw) + x;
    int32_t s = 1 << a.offset_bits;
    if constexpr (TY != 0) {
#pragma unroll
      for (int k = 0; k < TY; ++k) s += f[k] * (int)col[k << lw];
    } else {
      for (int k = 0; k < ty; ++k) s += f[k] * (int)col[k << lw];
    }
    const int32_t res = (uint16_t)((s + ((1 << a.r1) >> 1)) >> a.r1);  // CONV_BUF_TYPE
    int32_t tmp;
    if (a.is_compound) {
      uint16_t* c = conv + (int64_t)y * a.conv_stride + x;
      if (!a.do_average) {
        *c = (uint16_t)res;
        continue;
      }
      tmp = *c;
      tmp = a.dist_wtd ? (tmp * a.fwd + res * a.bck) >> 4 : (tmp + res) >> 1;
      tmp -= a.round_offset;
    } else {
      tmp = res - a.round_offset;
    }
    const int v = (tmp + ((1 << a.round_bits) >> 1)) >> a.round_bits;
    dst[(int64_t)y * a.dst_stride + x] = (Pix)min(max(v, 0), pmax);
  }
}

template <typename Pix>
void scale_launch(const ScaleArgs& a, int grid, size_t lds, hipStream_t s) {
#define LAVISH_SCALE_K(X, Y)                                                                   \
  if (a.tx == X && a.ty == Y) {                                                                \
    hipLaunchKernelGGL((scale_kernel<Pix, X, Y>), dim3(grid), dim3(256), lds, s, a);           \
    return;                                                                                    \
  }
  LAVISH_SCALE_K(8, 8)
  LAVISH_SCALE_K(12, 12)
  LAVISH_SCALE_K(4, 4)
  LAVISH_SCALE_K(4, 8)
  LAVISH_SCALE_K(8, 4)
  LAVISH_SCALE_K(2, 2)
#undef LAVISH_SCALE_K
  hipLaunchKernelGGL((scale_kernel<Pix, 0, 0>), dim3(grid), dim3(256), lds, s, a);
}

}  // namespace

int scale_batch(const void* src, int src_stride, void* dst, int dst_stride, uint16_t* conv,
                int conv_stride, int w, int h, const LavishScaleJob* jobs, int njobs,
                const LavishInterpFilterParams* fpx, const LavishInterpFilterParams* fpy,
                const LavishConvolveParams* cp, int bd, int highbd, hipStream_t s) {
  if (njobs <= 0) return 0;
  if (!src || !jobs || !cp || !fpx || !fpy) return -1;
  if ((cp->is_compound && !conv) || ((!cp->is_compound || cp->do_average) && !dst)) return -1;
  if (w < 2 || h < 1 || w > 128 || h > 128 || (w & (w - 1))) return -2;
  if (highbd ? (bd != 8 && bd != 10 && bd != 12) : bd != 8) return -3;
  if (fpx->taps < 2 || fpx->taps > kMaxTaps || fpy->taps < 2 || fpy->taps > kMaxTaps ||
      (fpx->taps & 1) || (fpy->taps & 1) || !fpx->filter_ptr || !fpy->filter_ptr)
    return -4;
  const int round_bits = 2 * kFBits - cp->round_0 - cp->round_1;
  if (cp->round_0 < 0 || cp->round_1 < 0 || round_bits < 0 || cp->round_0 > kFBits ||
      cp->round_1 > 2 * kFBits)
    return -5;
  ScaleArgs a{};
  a.src = src;
  a.dst = dst;
  a.conv = conv;
  a.jobs = jobs;
  a.src_stride = src_stride;
  a.dst_stride = dst_stride;
  a.conv_stride = conv_stride;
  a.w = w;
  a.h = h;
  a.lw = 31 - __builtin_clz(w);
  a.njobs = njobs;
  a.bd = bd;
  a.tx = fpx->taps;
  a.ty = fpy->taps;
  for (int p = 0; p < 16; ++p)  // av1_get_interp_filter_subpel_kernel rows
    for (int k = 0; k < kMaxTaps; ++k) {
      a.fx[p][k] = k < a.tx ? fpx->filter_ptr[a.tx * p + k] : 0;
      a.fy[p][k] = k < a.ty ? fpy->filter_ptr[a.ty * p + k] : 0;
    }
  a.r0 = cp->round_0;
  a.r1 = cp->round_1;
  a.offset_bits = bd + 2 * kFBits - cp->round_0;
  a.round_offset =
      (1 << (a.offset_bits - cp->round_1)) + (1 << (a.offset_bits - cp->round_1 - 1));
  a.round_bits = round_bits;
  a.is_compound = cp->is_compound;
  a.do_average = cp->do_average;
  a.dist_wtd = cp->use_dist_wtd_comp_avg;
  a.fwd = cp->fwd_offset;
  a.bck = cp->bck_offset;
  // the largest intermediate a supported step can make, per block slot
  // (rounded to 8 int16: each slot 16-byte aligned)
  const int im_rows = (((h - 1) * kMaxStep + (1 << kScaleBits) - 1) >> kScaleBits) + a.ty;
  a.im_cap = (im_rows * w + 7) & ~7;
  a.nb = w * h >= 256 ? 1 : min(16, 256 / (w * h));
  const int grid = (njobs + a.nb - 1) / a.nb;
  const size_t lds = (size_t)(2 * 16 * kFRow + a.nb * a.im_cap) * sizeof(int16_t);
  if (highbd)
    scale_launch<uint16_t>(a, grid, lds, s);
  else
    scale_launch<uint8_t>(a, grid, lds, s);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

}  // namespace lavish

using namespace lavish;

extern "C" int lavish_convolve_2d_scale_batch(
    const void* src, int src_stride, void* dst, int dst_stride, uint16_t* conv_dst,
    int conv_stride, int w, int h, const LavishScaleJob* jobs, int njobs,
    const LavishInterpFilterParams* filter_params_x,
    const LavishInterpFilterParams* filter_params_y, const LavishConvolveParams* conv_params,
    int bit_depth, int highbd, void* stream) {
  return scale_batch(src, src_stride, dst, dst_stride, conv_dst, conv_stride, w, h, jobs, njobs,
                     filter_params_x, filter_params_y, conv_params, bit_depth, highbd,
                     (hipStream_t)stream);
}

// ---- per-call RTCD shims (av1/common/av1_rtcd_defs.pl:580-588) ----
// Host buffers: the block's source window (the scaled extent plus the taps'
// margins), the prediction block and the CONV_BUF block are staged; one job.
namespace {
template <typename Pix>
void scale_shim(const Pix* src, int ss, Pix* dst, int ds, int w, int h,
                const LavishInterpFilterParams* fpx, const LavishInterpFilterParams* fpy,
                int spx, int xs, int spy, int ys, LavishConvolveParams* cp, int bd) {
  if (w <= 0 || h <= 0 || !fpx || !fpy || !cp) return;
  // a step or phase the kernel does not take: refuse before staging, so the
  // caller's buffers stay untouched (the kernel would skip the block and the
  // copy-back would hand over unwritten scratch)
  if (xs < 1 || xs > kMaxStep || ys < 1 || ys > kMaxStep || spx < 0 || spy < 0 ||
      spx > (1 << kScaleBits) - 1 || spy > (1 << kScaleBits) - 1) {
    shim_reject("av1_convolve_2d_scale_hip", -6);
    return;
  }
  const int fo_x = fpx->taps / 2 - 1, fo_y = fpy->taps / 2 - 1;
  const int wx = (((w - 1) * xs + spx) >> kScaleBits) + fpx->taps;
  const int wy = (((h - 1) * ys + spy) >> kScaleBits) + fpy->taps;
  const hipStream_t s = shim_stream();
  const size_t sb = ((size_t)wx * wy * sizeof(Pix) + 255) & ~(size_t)255;
  const size_t db = ((size_t)w * h * sizeof(Pix) + 255) & ~(size_t)255;
  const size_t cb = ((size_t)w * h * 2 + 255) & ~(size_t)255;
  char* base = (char*)shim_scratch(sb + db + cb + 256);
  Pix* dsrc = (Pix*)base;
  Pix* ddst = (Pix*)(base + sb);
  uint16_t* dconv = (uint16_t*)(base + sb + db);
  LavishScaleJob* djob = (LavishScaleJob*)(base + sb + db + cb);
  LAVISH_CHECK(hipMemcpy2DAsync(dsrc, (size_t)wx * sizeof(Pix), src - (int64_t)fo_y * ss - fo_x,
                                (size_t)ss * sizeof(Pix), (size_t)wx * sizeof(Pix), wy,
                                hipMemcpyHostToDevice, s));
  if (cp->is_compound && cp->do_average)
    LAVISH_CHECK(hipMemcpy2DAsync(dconv, (size_t)w * 2, cp->dst, (size_t)cp->dst_stride * 2,
                                  (size_t)w * 2, h, hipMemcpyHostToDevice, s));
  LavishScaleJob jb{};
  jb.src_off = (int64_t)fo_y * wx + fo_x;
  jb.subpel_x_qn = spx;
  jb.x_step_qn = xs;
  jb.subpel_y_qn = spy;
  jb.y_step_qn = ys;
  LAVISH_CHECK(hipMemcpyAsync(djob, &jb, sizeof(jb), hipMemcpyHostToDevice, s));
  const int rc = scale_batch(dsrc, wx, ddst, w, dconv, w, w, h, djob, 1, fpx, fpy, cp, bd,
                             sizeof(Pix) == 2, s);
  if (rc != 0) {
    shim_reject("av1_convolve_2d_scale_hip", rc);
    return;
  }
  if (cp->is_compound && !cp->do_average)
    LAVISH_CHECK(hipMemcpy2DAsync(cp->dst, (size_t)cp->dst_stride * 2, dconv, (size_t)w * 2,
                                  (size_t)w * 2, h, hipMemcpyDeviceToHost, s));
  else
    LAVISH_CHECK(hipMemcpy2DAsync(dst, (size_t)ds * sizeof(Pix), ddst, (size_t)w * sizeof(Pix),
                                  (size_t)w * sizeof(Pix), h, hipMemcpyDeviceToHost, s));
  LAVISH_CHECK(hipStreamSynchronize(s));
}
}  // namespace

extern "C" {
void av1_convolve_2d_scale_hip(const uint8_t* src, int src_stride, uint8_t* dst, int dst_stride,
                               int w, int h, const LavishInterpFilterParams* filter_params_x,
                               const LavishInterpFilterParams* filter_params_y,
                               const int subpel_x_qn, const int x_step_qn, const int subpel_y_qn,
                               const int y_step_qn, LavishConvolveParams* conv_params) {
  scale_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, filter_params_x, filter_params_y,
                      subpel_x_qn, x_step_qn, subpel_y_qn, y_step_qn, conv_params, 8);
}
void av1_highbd_convolve_2d_scale_hip(const uint16_t* src, int src_stride, uint16_t* dst,
                                      int dst_stride, int w, int h,
                                      const LavishInterpFilterParams* filter_params_x,
                                      const LavishInterpFilterParams* filter_params_y,
                                      const int subpel_x_qn, const int x_step_qn,
                                      const int subpel_y_qn, const int y_step_qn,
                                      LavishConvolveParams* conv_params, int bd) {
  scale_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, filter_params_x, filter_params_y,
                       subpel_x_qn, x_step_qn, subpel_y_qn, y_step_qn, conv_params, bd);
}
}
