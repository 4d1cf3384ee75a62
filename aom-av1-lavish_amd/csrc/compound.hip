// compound.hip -- the compound (CONV_BUF) convolutions on gfx950 (SURVEY.md
// 8(f) rank 2: the second half of inter prediction for compound modes).
//
// Reference: av1_dist_wtd_convolve_2d_copy_c / _x_c / _y_c / _2d_c and the
// highbd forms (av1/common/convolve.c:291-489,790-988); the path per block
// is convolve_2d_facade_compound's (:590-612): copy when both sub-pel
// offsets are 0, x or y when one is, 2-D otherwise.  Every form makes the
// offset CONV_BUF value; the first pass (do_average 0) stores it, the second
// (do_average 1) averages it with the buffer -- plain or distance-weighted
// (fwd / bck offsets, DIST_PRECISION_BITS) -- removes the offset, rounds and
// clips into the prediction.
//
// One workgroup per block (blocks of <= 256 pixels share one 2 or 4 ways,
// each with its slice of the dynamic LDS): for the 2-D path its threads
// first filter the (h + taps - 1) x w intermediate rows into LDS (int16, as
// the reference stores them), then every thread takes output pixels (rows
// coalesced across threads) and applies the vertical taps / the single 1-D
// pass / the copy and the write-out.  The kernel rows of the caller's filters
// (InterpFilterParams, up to 12 taps x 16 phases) travel as kernel
// arguments.
#include <algorithm>

#include "lavish_internal.h"


namespace lavish {
namespace {

constexpr int kFBits = 7;   // FILTER_BITS
constexpr int kMaxTaps = 12;
constexpr int kMaxW = 128, kMaxH = 128;

struct CompArgs {
  const void* src;
  void* dst;
  uint16_t* conv;
  const LavishCompoundJob* jobs;
  int src_stride, dst_stride, conv_stride, w, h, njobs, bd;
  int tx, ty;                           // tap counts
  int lw, bpw, any2d;                   // log2(w), blocks per workgroup, 2-D path possible
  int16_t fx[16][kMaxTaps], fy[16][kMaxTaps];
  int r0, r1, offset_bits, round_offset, round_bits, do_average, dist_wtd, fwd, bck;
};

// a.bpw blocks per 256-thread workgroup (small blocks share one), each with
// 256 / bpw threads and its own slice of the dynamic LDS intermediate
// T8: both filters have 8 taps (every block wider and taller than 4): the tap
// loops unroll, so a pixel's 8 loads are in flight together
template <typename Pix, bool T8>
__global__ __launch_bounds__(256) void compound_kernel(CompArgs a) {
  extern __shared__ int16_t im_all[];
  const int nwg = gridDim.x;  // multiple of 8: consecutive blocks share an XCD's L2
  const int wg = (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  const int tpb = 256 / a.bpw;  // threads per block
  const int sub = threadIdx.x / tpb, t = threadIdx.x - sub * tpb;
  const int j = wg * a.bpw + sub;
  const bool live = j < a.njobs;
  const LavishCompoundJob& jb = a.jobs[live ? j : a.njobs - 1];
  const int sx = jb.subpel_x_qn & 15, sy = jb.subpel_y_qn & 15;
  const int path = (sx != 0) + 2 * (sy != 0);
  const Pix* src = (const Pix*)a.src + jb.src_off;
  Pix* dst = (Pix*)a.dst + jb.dst_off;
  uint16_t* conv = a.conv + jb.conv_off;
  const int w = a.w, lw = a.lw;
  const int ntx = T8 ? 8 : a.tx, nty = T8 ? 8 : a.ty;
  constexpr int kUnroll = T8 ? 8 : 1;  // full unroll of the T8 tap loops only
  const int fo_x = ntx / 2 - 1, fo_y = nty / 2 - 1;
  const int16_t* fxp = a.fx[sx];
  const int16_t* fyp = a.fy[sy];
  // T8: the block's two tap rows live in registers for all its pixels
  int16_t fx[T8 ? 8 : 1], fy[T8 ? 8 : 1];
  if (T8) {
#pragma unroll
    for (int k = 0; k < (T8 ? 8 : 1); ++k) {
      fx[k] = fxp[k];
      fy[k] = fyp[k];
    }
  }
#define FX(k) (T8 ? fx[(k) & (T8 ? 7 : 0)] : fxp[k])
#define FY(k) (T8 ? fy[(k) & (T8 ? 7 : 0)] : fyp[k])
  int16_t* im = im_all + sub * (a.h + a.ty - 1) * w;
  if (a.any2d) {  // horizontal pass of the 2-D form into LDS (w is a power of two)
    if (path == 3) {
      const int ih = a.h + nty - 1;
      for (int e = t; e < ih * w; e += tpb) {
        const int y = e >> lw, x = e & (w - 1);
        const Pix* row = src + (int64_t)(y - fo_y) * a.src_stride + x - fo_x;
        int32_t s = 1 << (a.bd + kFBits - 1);
#pragma unroll kUnroll
        for (int k = 0; k < ntx; ++k) s += FX(k) * (int)row[k];
        im[e] = (int16_t)((s + ((1 << a.r0) >> 1)) >> a.r0);
      }
    }
    __syncthreads();
  }
  if (!live) return;
  const int pmax = (1 << a.bd) - 1;
  for (int e = t; e < a.h * w; e += tpb) {
    const int y = e >> lw, x = e & (w - 1);
    int32_t res;
    if (path == 0) {
      res = (uint16_t)(((int)src[(int64_t)y * a.src_stride + x] << a.round_bits) +
                       a.round_offset);
    } else if (path == 1) {
      const Pix* row = src + (int64_t)y * a.src_stride + x - fo_x;
      int32_t s = 0;
#pragma unroll kUnroll
      for (int k = 0; k < ntx; ++k) s += FX(k) * (int)row[k];
      res = (1 << (kFBits - a.r1)) * ((s + ((1 << a.r0) >> 1)) >> a.r0) + a.round_offset;
    } else if (path == 2) {
      const Pix* col = src + (int64_t)(y - fo_y) * a.src_stride + x;
      int32_t s = 0;
#pragma unroll kUnroll
      for (int k = 0; k < nty; ++k) s += FY(k) * (int)col[(int64_t)k * a.src_stride];
      s *= 1 << (kFBits - a.r0);
      res = ((s + ((1 << a.r1) >> 1)) >> a.r1) + a.round_offset;
    } else {
      int32_t s = 1 << a.offset_bits;
#pragma unroll kUnroll
      for (int k = 0; k < nty; ++k) s += FY(k) * (int)im[((y + k) << lw) + x];
      res = (uint16_t)((s + ((1 << a.r1) >> 1)) >> a.r1);
    }
    uint16_t* c = conv + (int64_t)y * a.conv_stride + x;
    if (!a.do_average) {
      *c = (uint16_t)res;
      continue;
    }
    int32_t tt = *c;
    tt = a.dist_wtd ? (tt * a.fwd + res * a.bck) >> 4 : (tt + res) >> 1;
    tt -= a.round_offset;
    const int v = (tt + ((1 << a.round_bits) >> 1)) >> a.round_bits;
    dst[(int64_t)y * a.dst_stride + x] = (Pix)min(max(v, 0), pmax);
  }
#undef FX
#undef FY
}

}  // namespace

int compound_batch(const void* src, int src_stride, void* dst, int dst_stride, uint16_t* conv,
                   int conv_stride, int w, int h, const LavishCompoundJob* jobs, int njobs,
                   const LavishInterpFilterParams* fpx, const LavishInterpFilterParams* fpy,
                   const LavishConvolveParams* cp, int bd, int highbd, hipStream_t s) {
  if (njobs <= 0) return 0;
  if (!src || !conv || !jobs || !cp || !fpx || !fpy || (cp->do_average && !dst)) return -1;
  if (w < 2 || h < 1 || w > kMaxW || h > kMaxH || (w & (w - 1))) return -2;
  if (highbd ? (bd != 8 && bd != 10 && bd != 12) : bd != 8) return -3;
  if (fpx->taps < 2 || fpx->taps > kMaxTaps || fpy->taps < 2 || fpy->taps > kMaxTaps ||
      (fpx->taps & 1) || (fpy->taps & 1) || !fpx->filter_ptr || !fpy->filter_ptr)
    return -4;
  const int round_bits = 2 * kFBits - cp->round_0 - cp->round_1;
  if (cp->round_0 < 0 || cp->round_1 < 0 || round_bits < 0 || cp->round_1 > kFBits ||
      cp->round_0 > kFBits)
    return -5;
  CompArgs a{};
  a.src = src;
  a.dst = dst;
  a.conv = conv;
  a.jobs = jobs;
  a.src_stride = src_stride;
  a.dst_stride = dst_stride;
  a.conv_stride = conv_stride;
  a.w = w;
  a.h = h;
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
  a.round_offset = (1 << (a.offset_bits - cp->round_1)) + (1 << (a.offset_bits - cp->round_1 - 1));
  a.round_bits = round_bits;
  a.do_average = cp->do_average;
  a.dist_wtd = cp->use_dist_wtd_comp_avg;
  a.fwd = cp->fwd_offset;
  a.bck = cp->bck_offset;
  a.lw = 31 - __builtin_clz(w);
  // blocks of <= 256 pixels share a workgroup 4 ways, <= 1024 2 ways
  a.bpw = w * h <= 256 ? 4 : (w * h <= 1024 ? 2 : 1);
  a.any2d = 1;  // the per-block path is decided on the device
  const size_t lds = (size_t)a.bpw * (h + a.ty - 1) * w * sizeof(int16_t);
  int nwg = (njobs + a.bpw - 1) / a.bpw;
  nwg = (nwg + 7) & ~7;
  const bool t8 = a.tx == 8 && a.ty == 8;
  if (highbd) {
    if (t8) hipLaunchKernelGGL((compound_kernel<uint16_t, true>), dim3(nwg), dim3(256), lds, s, a);
    else hipLaunchKernelGGL((compound_kernel<uint16_t, false>), dim3(nwg), dim3(256), lds, s, a);
  } else {
    if (t8) hipLaunchKernelGGL((compound_kernel<uint8_t, true>), dim3(nwg), dim3(256), lds, s, a);
    else hipLaunchKernelGGL((compound_kernel<uint8_t, false>), dim3(nwg), dim3(256), lds, s, a);
  }
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

}  // namespace lavish

using namespace lavish;

extern "C" int lavish_dist_wtd_convolve_batch(
    const void* src, int src_stride, void* dst, int dst_stride, uint16_t* conv_dst,
    int conv_stride, int w, int h, const LavishCompoundJob* jobs, int njobs,
    const LavishInterpFilterParams* filter_params_x,
    const LavishInterpFilterParams* filter_params_y, const LavishConvolveParams* conv_params,
    int bit_depth, int highbd, void* stream) {
  return compound_batch(src, src_stride, dst, dst_stride, conv_dst, conv_stride, w, h, jobs, njobs,
                        filter_params_x, filter_params_y, conv_params, bit_depth, highbd,
                        (hipStream_t)stream);
}

// ---- per-call RTCD shims (av1/common/av1_rtcd_defs.pl:568-579) ----
// Host buffers: the block's source window (taps margins), the prediction
// block and the CONV_BUF block are staged; one job.
namespace {
const int16_t kZeroTaps[2 * 16] = {};
const LavishInterpFilterParams kNoFilter = {kZeroTaps, 2, 0};

template <typename Pix>
void compound_shim(const Pix* src, int ss, Pix* dst, int ds, int w, int h,
                   const LavishInterpFilterParams* fpx, const LavishInterpFilterParams* fpy,
                   int sx, int sy, LavishConvolveParams* cp, int bd) {
  if (w <= 0 || h <= 0) return;
  const LavishInterpFilterParams* px = fpx ? fpx : &kNoFilter;
  const LavishInterpFilterParams* py = fpy ? fpy : &kNoFilter;
  const int path = (sx & 15 ? 1 : 0) + (sy & 15 ? 2 : 0);
  const int mx = (path & 1) ? px->taps / 2 - 1 : 0, my = (path & 2) ? py->taps / 2 - 1 : 0;
  const int wx = w + ((path & 1) ? px->taps - 1 : 0), wy = h + ((path & 2) ? py->taps - 1 : 0);
  const hipStream_t s = shim_stream();
  const size_t sb = ((size_t)wx * wy * sizeof(Pix) + 255) & ~(size_t)255;
  const size_t db = ((size_t)w * h * sizeof(Pix) + 255) & ~(size_t)255;
  const size_t cb = ((size_t)w * h * 2 + 255) & ~(size_t)255;
  char* base = (char*)shim_scratch(sb + db + cb + 256);
  Pix* dsrc = (Pix*)base;
  Pix* ddst = (Pix*)(base + sb);
  uint16_t* dconv = (uint16_t*)(base + sb + db);
  LavishCompoundJob* djob = (LavishCompoundJob*)(base + sb + db + cb);
  LAVISH_CHECK(hipMemcpy2DAsync(dsrc, (size_t)wx * sizeof(Pix), src - (int64_t)my * ss - mx,
                                (size_t)ss * sizeof(Pix), (size_t)wx * sizeof(Pix), wy,
                                hipMemcpyHostToDevice, s));
  LAVISH_CHECK(hipMemcpy2DAsync(dconv, (size_t)w * 2, cp->dst, (size_t)cp->dst_stride * 2,
                                (size_t)w * 2, h, hipMemcpyHostToDevice, s));
  LavishCompoundJob jb{};
  jb.src_off = (int64_t)my * wx + mx;
  jb.subpel_x_qn = path & 1 ? sx : 0;
  jb.subpel_y_qn = path & 2 ? sy : 0;
  LAVISH_CHECK(hipMemcpyAsync(djob, &jb, sizeof(jb), hipMemcpyHostToDevice, s));
  const int rc = compound_batch(dsrc, wx, ddst, w, dconv, w, w, h, djob, 1, px, py, cp, bd,
                                sizeof(Pix) == 2, s);
  if (rc != 0) {
    shim_reject("av1_dist_wtd_convolve_hip", rc);
    return;
  }
  if (cp->do_average)
    LAVISH_CHECK(hipMemcpy2DAsync(dst, (size_t)ds * sizeof(Pix), ddst, (size_t)w * sizeof(Pix),
                                  (size_t)w * sizeof(Pix), h, hipMemcpyDeviceToHost, s));
  else
    LAVISH_CHECK(hipMemcpy2DAsync(cp->dst, (size_t)cp->dst_stride * 2, dconv, (size_t)w * 2,
                                  (size_t)w * 2, h, hipMemcpyDeviceToHost, s));
  LAVISH_CHECK(hipStreamSynchronize(s));
}
}  // namespace

extern "C" {
void av1_dist_wtd_convolve_2d_hip(const uint8_t* src, int src_stride, uint8_t* dst,
                                  int dst_stride, int w, int h,
                                  const LavishInterpFilterParams* fpx,
                                  const LavishInterpFilterParams* fpy, const int subpel_x_qn,
                                  const int subpel_y_qn, LavishConvolveParams* cp) {
  compound_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, fpx, fpy, subpel_x_qn,
                         subpel_y_qn, cp, 8);
}
void av1_dist_wtd_convolve_2d_copy_hip(const uint8_t* src, int src_stride, uint8_t* dst,
                                       int dst_stride, int w, int h, LavishConvolveParams* cp) {
  compound_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, nullptr, nullptr, 0, 0, cp, 8);
}
void av1_dist_wtd_convolve_x_hip(const uint8_t* src, int src_stride, uint8_t* dst, int dst_stride,
                                 int w, int h, const LavishInterpFilterParams* fpx,
                                 const int subpel_x_qn, LavishConvolveParams* cp) {
  compound_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, fpx, nullptr, subpel_x_qn, 0,
                         cp, 8);
}
void av1_dist_wtd_convolve_y_hip(const uint8_t* src, int src_stride, uint8_t* dst, int dst_stride,
                                 int w, int h, const LavishInterpFilterParams* fpy,
                                 const int subpel_y_qn, LavishConvolveParams* cp) {
  compound_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, nullptr, fpy, 0, subpel_y_qn,
                         cp, 8);
}
void av1_highbd_dist_wtd_convolve_2d_hip(const uint16_t* src, int src_stride, uint16_t* dst,
                                         int dst_stride, int w, int h,
                                         const LavishInterpFilterParams* fpx,
                                         const LavishInterpFilterParams* fpy,
                                         const int subpel_x_qn, const int subpel_y_qn,
                                         LavishConvolveParams* cp, int bd) {
  compound_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, fpx, fpy, subpel_x_qn,
                          subpel_y_qn, cp, bd);
}
void av1_highbd_dist_wtd_convolve_x_hip(const uint16_t* src, int src_stride, uint16_t* dst,
                                        int dst_stride, int w, int h,
                                        const LavishInterpFilterParams* fpx,
                                        const int subpel_x_qn, LavishConvolveParams* cp, int bd) {
  compound_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, fpx, nullptr, subpel_x_qn, 0,
                          cp, bd);
}
void av1_highbd_dist_wtd_convolve_y_hip(const uint16_t* src, int src_stride, uint16_t* dst,
                                        int dst_stride, int w, int h,
                                        const LavishInterpFilterParams* fpy,
                                        const int subpel_y_qn, LavishConvolveParams* cp, int bd) {
  compound_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, nullptr, fpy, 0, subpel_y_qn,
                          cp, bd);
}
void av1_highbd_dist_wtd_convolve_2d_copy_hip(const uint16_t* src, int src_stride, uint16_t* dst,
                                              int dst_stride, int w, int h,
                                              LavishConvolveParams* cp, int bd) {
  compound_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, nullptr, nullptr, 0, 0, cp, bd);
}
}
