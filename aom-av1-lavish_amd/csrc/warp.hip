// warp.hip -- the affine warp predictor on gfx950.
//
// Reference: av1_warp_affine_c (av1/common/warped_motion.c:538-666) and
// av1_highbd_warp_affine_c (:264-388), with av1_get_shear_params (:218-247)
// for the caller's alpha / beta / gamma / delta.  Per 8x8 output unit the
// unit centre is projected through the matrix (luma coordinates when the
// plane is subsampled); 15 rows x 8 columns are filtered horizontally with a
// per-pixel phase (sx4 + alpha c + beta (r - 3)) over edge-clamped samples,
// then every output takes 8 vertical taps (phase sy4 + gamma c + delta r)
// and is written as a single prediction, a compound first pass (the
// CONV_BUF_TYPE value) or a compound (distance-weighted) average.
//
// Here one wave owns one job (a prediction block of p_width x p_height) and
// walks its 8x8 units: lanes 0..59 each filter two of the 120 horizontal
// outputs (an in-frame row segment is one byte-addressed 8 / 16-byte load,
// rows that touch the frame edge take the clamped per-sample path), with
// v_dot2_i32_i16 over packed sample / tap pairs (the table's rows are
// already int16 pairs); the 15 x 8 intermediate (int16 by the reference's
// bit-width design) goes through LDS column-major, and lane (r, c) of the
// unit does the vertical taps (4 dot2 over row pairs) and the write-out.
// The filter table (193 x 8 taps) is staged in LDS once per 4 jobs.
#include <algorithm>

#include "lavish_internal.h"
#include "warp_tables.h"

namespace lavish {
namespace {

constexpr int kWmBits = 16;    // WARPEDMODEL_PREC_BITS (mv.h:96)
constexpr int kWdBits = 10;    // WARPEDDIFF_PREC_BITS
constexpr int kWpShifts = 64;  // WARPEDPIXEL_PREC_SHIFTS
constexpr int kWrBits = 6;     // WARP_PARAM_REDUCE_BITS
constexpr int kFBits = 7;      // FILTER_BITS

struct WarpArgs {
  const void* ref;
  void* pred;
  uint16_t* dst;
  const LavishWarpJob* jobs;
  int width, height, stride, p_stride, dst_stride, njobs, ss_x, ss_y, bd;
  int rh, rv, off_h, off_v, round_bits, off_sub;  // derived rounding (per call)
  int is_compound, do_average, dist_wtd, fwd, bck;
};

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b), c,
                                false);
}

// the 8 samples ref[row + x .. row + x + 7] as 4 packed int16 pairs; x may be
// < 0 or run past the right edge (clamped per sample)
template <typename Pix>
__device__ __forceinline__ void load8(const Pix* row, int x, int width, uint32_t (&p)[4]) {
  if (x >= 0 && x + 7 < width) {
    if constexpr (sizeof(Pix) == 1) {
      const u32x2u w = *(const __attribute__((address_space(1))) u32x2u*)(row + x);
      // v_perm_b32: bytes (b0, 0, b1, 0) ... (0x0c selects a zero byte)
      p[0] = __builtin_amdgcn_perm(0u, w.x, 0x0c010c00u);
      p[1] = __builtin_amdgcn_perm(0u, w.x, 0x0c030c02u);
      p[2] = __builtin_amdgcn_perm(0u, w.y, 0x0c010c00u);
      p[3] = __builtin_amdgcn_perm(0u, w.y, 0x0c030c02u);
    } else {
      const u32x4u w = *(const __attribute__((address_space(1))) u32x4u*)(row + x);
      p[0] = w.x;
      p[1] = w.y;
      p[2] = w.z;
      p[3] = w.w;
    }
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      p[m] = (uint32_t)row[min(max(x + 2 * m, 0), width - 1)] |
             ((uint32_t)row[min(max(x + 2 * m + 1, 0), width - 1)] << 16);
  }
}

// the 8 taps of filter row `offs` as 4 packed int16 pairs (LDS copy)
__device__ __forceinline__ void taps(const int16_t* filt, int offs, uint32_t (&t)[4]) {
  typedef __attribute__((address_space(3))) const u32x4* lp4;
  const u32x4 w = *(lp4)(filt + 8 * offs);
  t[0] = w.x;
  t[1] = w.y;
  t[2] = w.z;
  t[3] = w.w;
}

constexpr int kJobsPerWg = 4;  // one wave per job; the table is staged once per 4 jobs

template <typename Pix>
__global__ __launch_bounds__(64 * kJobsPerWg) void warp_kernel(WarpArgs a) {
  __shared__ __attribute__((aligned(16))) int16_t filt[193 * 8];
  // per wave: the 15 x 8 horizontal outputs, column-major (16 per column) so
  // vertical tap pairs come from aligned 32-bit LDS reads; they fit int16
  // (< 2^(bd + 8 - round_0) <= 2^15, warped_motion.c:516-522)
  __shared__ __attribute__((aligned(16))) int16_t tmp_s[kJobsPerWg][8 * 16];
  for (int i = threadIdx.x; i < 193 * 8 / 2; i += 64 * kJobsPerWg)
    ((uint32_t*)filt)[i] = ((const uint32_t*)&kWarpedFilter[0][0])[i];
  __syncthreads();
  const int nwg = gridDim.x;  // multiple of 8: consecutive jobs share an XCD's L2
  const int wg = (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = wg * kJobsPerWg + wave;
  if (j >= a.njobs) return;
  int16_t* tmp = tmp_s[wave];
  const LavishWarpJob& jb = a.jobs[j];
  const int64_t m0 = jb.mat[0], m1 = jb.mat[1], m2 = jb.mat[2], m3 = jb.mat[3], m4 = jb.mat[4],
                m5 = jb.mat[5];
  const int alpha = jb.alpha, beta = jb.beta, gamma = jb.gamma, delta = jb.delta;
  const int p_col = jb.p_col, p_row = jb.p_row, pw = jb.p_width, ph = jb.p_height;
  const Pix* ref = (const Pix*)a.ref + jb.ref_off;
  Pix* pred = (Pix*)a.pred + jb.pred_off;
  uint16_t* dst = a.dst ? a.dst + jb.dst_off : nullptr;
  const int pmax = (1 << a.bd) - 1;
  // the job's 8x8 units in raster order
  const int ucols = (pw + 7) >> 3, units = ucols * ((ph + 7) >> 3);
  for (int u = 0; u < units; ++u) {
    const int i = p_row + 8 * (u / ucols), jc = p_col + 8 * (u % ucols);
    const int64_t cx = (int64_t)((jc + 4) << a.ss_x), cy = (int64_t)((i + 4) << a.ss_y);
    const int64_t x4 = (m2 * cx + m3 * cy + m0) >> a.ss_x;
    const int64_t y4 = (m4 * cx + m5 * cy + m1) >> a.ss_y;
    const int ix4 = (int)(x4 >> kWmBits), iy4 = (int)(y4 >> kWmBits);
    const int sx4 = ((int)(x4 & ((1 << kWmBits) - 1)) - 4 * alpha - 4 * beta) &
                    ~((1 << kWrBits) - 1);
    const int sy4 = ((int)(y4 & ((1 << kWmBits) - 1)) - 4 * gamma - 4 * delta) &
                    ~((1 << kWrBits) - 1);
    // horizontal: outputs o = lane and lane + 64 of the 15 x 8, v_dot2_i32_i16
    // over packed sample / tap pairs
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int o = lane + 64 * hh;
      if (o < 120) {
        const int r = o >> 3, c = o & 7;
        const Pix* row = ref + (int64_t)min(max(iy4 + r - 7, 0), a.height - 1) * a.stride;
        const int sx = sx4 + beta * (r - 3) + alpha * c;
        uint32_t t[4], p[4];
        taps(filt, ((sx + (1 << (kWdBits - 1))) >> kWdBits) + kWpShifts, t);
        load8<Pix>(row, ix4 + c - 7, a.width, p);
        int32_t s = 1 << a.off_h;
#pragma unroll
        for (int m = 0; m < 4; ++m) s = dot2(p[m], t[m], s);
        tmp[c * 16 + r] = (int16_t)((s + ((1 << a.rh) >> 1)) >> a.rh);
      }
    }
    wave_sync();
    // vertical: lane = (r, c) of the unit, cropped to the block
    const int r = lane >> 3, c = lane & 7;
    if (r < p_row + ph - i && c < p_col + pw - jc) {
      const int sy = sy4 + delta * r + gamma * c;
      uint32_t t[4];
      taps(filt, ((sy + (1 << (kWdBits - 1))) >> kWdBits) + kWpShifts, t);
      // rows r .. r + 7 of column c: 5 aligned dwords from the even row at or
      // below r, shifted by a half-word when r is odd
      const __attribute__((address_space(3))) uint32_t* col =
          (const __attribute__((address_space(3))) uint32_t*)(tmp + c * 16 + (r & ~1));
      uint32_t d[5];
#pragma unroll
      for (int m = 0; m < 5; ++m) d[m] = col[m];
      const uint32_t sh = (uint32_t)(r & 1) * 16;
      int32_t s = 1 << a.off_v;
#pragma unroll
      for (int m = 0; m < 4; ++m) s = dot2(__builtin_amdgcn_alignbit(d[m + 1], d[m], sh), t[m], s);
      s = (s + ((1 << a.rv) >> 1)) >> a.rv;
      const int py = i - p_row + r, px = jc - p_col + c;
      bool write = true;
      int out = 0;
      if (a.is_compound) {
        uint16_t* d = dst + (int64_t)py * a.dst_stride + px;
        if (!a.do_average) {
          *d = (uint16_t)s;
          write = false;
        } else {
          int32_t tt = *d;
          tt = a.dist_wtd ? (tt * a.fwd + s * a.bck) >> 4 : (tt + s) >> 1;  // DIST_PRECISION_BITS
          tt -= a.off_sub;
          out = (tt + ((1 << a.round_bits) >> 1)) >> a.round_bits;
        }
      } else {
        out = s - (1 << (a.bd - 1)) - (1 << a.bd);
      }
      if (write) pred[(int64_t)py * a.p_stride + px] = (Pix)min(max(out, 0), pmax);
    }
    wave_sync();  // tmp is rewritten by the next unit
  }
}

}  // namespace

// the rounding constants of av1_warp_affine_c / av1_highbd_warp_affine_c
static void derive(WarpArgs& a, const LavishConvolveParams& cp, int bd, int highbd) {
  const int extra = bd + kFBits - cp.round_0 - 14;
  a.rh = highbd ? cp.round_0 + (extra > 0 ? extra : 0) : cp.round_0;
  a.rv = cp.is_compound ? cp.round_1 : 2 * kFBits - a.rh;
  a.off_h = bd + kFBits - 1;
  a.off_v = bd + 2 * kFBits - a.rh;
  a.round_bits = 2 * kFBits - cp.round_0 - cp.round_1;
  const int off_bits = bd + 2 * kFBits - cp.round_0;
  a.off_sub = (1 << (off_bits - cp.round_1)) + (1 << (off_bits - cp.round_1 - 1));
  a.is_compound = cp.is_compound;
  a.do_average = cp.do_average;
  a.dist_wtd = cp.use_dist_wtd_comp_avg;
  a.fwd = cp.fwd_offset;
  a.bck = cp.bck_offset;
}

int warp_batch(const void* ref, int width, int height, int stride, void* pred, int p_stride,
               uint16_t* conv_dst, int dst_stride, const LavishWarpJob* jobs, int njobs,
               int ss_x, int ss_y, int bd, int highbd, const LavishConvolveParams* cp,
               hipStream_t s) {
  if (njobs <= 0) return 0;
  if (ref == nullptr || pred == nullptr || jobs == nullptr || cp == nullptr) return -1;
  if (width <= 0 || height <= 0 || stride <= 0) return -2;
  if (ss_x < 0 || ss_x > 1 || ss_y < 0 || ss_y > 1) return -3;
  if (highbd ? (bd != 8 && bd != 10 && bd != 12) : bd != 8) return -4;
  if (cp->is_compound && conv_dst == nullptr) return -5;
  if (cp->do_average && !cp->is_compound) return -5;
  if (cp->round_0 < 0 || cp->round_0 > 8 || cp->round_1 < 0 || cp->round_1 > 14) return -6;
  WarpArgs a{};
  a.ref = ref;
  a.pred = pred;
  a.dst = conv_dst;
  a.jobs = jobs;
  a.width = width;
  a.height = height;
  a.stride = stride;
  a.p_stride = p_stride;
  a.dst_stride = dst_stride;
  a.njobs = njobs;
  a.ss_x = ss_x;
  a.ss_y = ss_y;
  a.bd = bd;
  derive(a, *cp, bd, highbd);
  int nwg = (njobs + kJobsPerWg - 1) / kJobsPerWg;
  nwg = (nwg + 7) & ~7;
  if (highbd)
    hipLaunchKernelGGL(warp_kernel<uint16_t>, dim3(nwg), dim3(64 * kJobsPerWg), 0, s, a);
  else
    hipLaunchKernelGGL(warp_kernel<uint8_t>, dim3(nwg), dim3(64 * kJobsPerWg), 0, s, a);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

}  // namespace lavish

using namespace lavish;

extern "C" int lavish_warp_affine_batch(const void* ref, int width, int height, int stride,
                                        void* pred, int p_stride, uint16_t* conv_dst,
                                        int dst_stride, const LavishWarpJob* jobs, int njobs,
                                        int subsampling_x, int subsampling_y, int bit_depth,
                                        int highbd, const LavishConvolveParams* conv_params,
                                        void* stream) {
  return warp_batch(ref, width, height, stride, pred, p_stride, conv_dst, dst_stride, jobs, njobs,
                    subsampling_x, subsampling_y, bit_depth, highbd, conv_params,
                    (hipStream_t)stream);
}

// av1_get_shear_params (warped_motion.c:218-247) on the host: the caller's
// per-model setup, pure integer arithmetic (resolve_divisor_32 over div_lut)
extern "C" int lavish_get_shear_params(const int32_t* mat, int16_t* out) {
  auto rps64 = [](int64_t v, int n) -> int64_t {  // ROUND_POWER_OF_TWO_SIGNED_64
    const int64_t h = ((int64_t)1 << n) >> 1;
    return v < 0 ? -((-v + h) >> n) : (v + h) >> n;
  };
  auto rps = [](int v, int n) -> int {
    const int h = (1 << n) >> 1;
    return v < 0 ? -((-v + h) >> n) : (v + h) >> n;
  };
  auto cl16 = [](int64_t v) -> int { return (int)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); };
  if (mat[2] <= 0) return 0;
  int alpha = cl16(mat[2] - (1 << kWmBits));
  int beta = cl16(mat[3]);
  const uint32_t D = (uint32_t)(mat[2] < 0 ? -mat[2] : mat[2]);
  int shift = 31 - __builtin_clz(D);
  const int32_t e = (int32_t)(D - (1u << shift));
  const int32_t f = shift > 8 ? (e + ((1 << (shift - 8)) >> 1)) >> (shift - 8) : e << (8 - shift);
  shift += 14;  // DIV_LUT_PREC_BITS
  const int y = kDivLut[f];
  int gamma = cl16((int)rps64(((int64_t)mat[4] * (1 << kWmBits)) * y, shift));
  int delta = cl16(mat[5] - (int)rps64(((int64_t)mat[3] * mat[4]) * y, shift) - (1 << kWmBits));
  alpha = rps(alpha, kWrBits) * (1 << kWrBits);
  beta = rps(beta, kWrBits) * (1 << kWrBits);
  gamma = rps(gamma, kWrBits) * (1 << kWrBits);
  delta = rps(delta, kWrBits) * (1 << kWrBits);
  out[0] = (int16_t)alpha;
  out[1] = (int16_t)beta;
  out[2] = (int16_t)gamma;
  out[3] = (int16_t)delta;
  return !(4 * abs(alpha) + 7 * abs(beta) >= (1 << kWmBits) ||
           4 * abs(gamma) + 4 * abs(delta) >= (1 << kWmBits));
}

// ---- per-call RTCD shims (av1/common/av1_rtcd_defs.pl:544,548) ----
// Host buffers: the reference window the block's units can read (the unit
// centres projected here with the kernel's arithmetic, +-7 samples, clamped
// to the plane), the prediction block and, for compound, the CONV_BUF block
// are staged; the kernel addresses the window through plane coordinates.
template <typename Pix>
static void warp_shim(const int32_t* mat, const Pix* ref, int width, int height, int stride,
                      Pix* pred, int p_col, int p_row, int p_width, int p_height, int p_stride,
                      int ss_x, int ss_y, int bd, LavishConvolveParams* cp, int16_t alpha,
                      int16_t beta, int16_t gamma, int16_t delta) {
  if (p_width <= 0 || p_height <= 0) return;
  int x0 = width, x1 = -1, y0 = height, y1 = -1;
  for (int i = p_row; i < p_row + p_height; i += 8)
    for (int j = p_col; j < p_col + p_width; j += 8) {
      const int64_t cx = (int64_t)((j + 4) << ss_x), cy = (int64_t)((i + 4) << ss_y);
      const int ix4 = (int)((((int64_t)mat[2] * cx + (int64_t)mat[3] * cy + mat[0]) >> ss_x) >> kWmBits);
      const int iy4 = (int)((((int64_t)mat[4] * cx + (int64_t)mat[5] * cy + mat[1]) >> ss_y) >> kWmBits);
      x0 = std::min(x0, std::max(ix4 - 7, 0));
      x1 = std::max(x1, std::min(ix4 + 7, width - 1));
      y0 = std::min(y0, std::max(iy4 - 7, 0));
      y1 = std::max(y1, std::min(iy4 + 7, height - 1));
    }
  // a unit entirely off one side still reads the clamped edge column / row
  x0 = std::min(x0, width - 1); x1 = std::max(x1, 0);
  y0 = std::min(y0, height - 1); y1 = std::max(y1, 0);
  const int ww = x1 - x0 + 1, wh = y1 - y0 + 1;
  const hipStream_t s = shim_stream();
  const size_t rb = ((size_t)ww * wh * sizeof(Pix) + 255) & ~(size_t)255;
  const size_t pb = ((size_t)p_width * p_height * sizeof(Pix) + 255) & ~(size_t)255;
  const size_t db = ((size_t)p_width * p_height * sizeof(uint16_t) + 255) & ~(size_t)255;
  char* base = (char*)shim_scratch(rb + pb + db + 256);
  Pix* dref = (Pix*)base;
  Pix* dpred = (Pix*)(base + rb);
  uint16_t* ddst = (uint16_t*)(base + rb + pb);
  LavishWarpJob* djob = (LavishWarpJob*)(base + rb + pb + db);
  LAVISH_CHECK(hipMemcpy2DAsync(dref, (size_t)ww * sizeof(Pix), ref + (int64_t)y0 * stride + x0,
                                (size_t)stride * sizeof(Pix), (size_t)ww * sizeof(Pix), wh,
                                hipMemcpyHostToDevice, s));
  LAVISH_CHECK(hipMemcpy2DAsync(dpred, (size_t)p_width * sizeof(Pix), pred,
                                (size_t)p_stride * sizeof(Pix), (size_t)p_width * sizeof(Pix),
                                p_height, hipMemcpyHostToDevice, s));
  if (cp->is_compound)
    LAVISH_CHECK(hipMemcpy2DAsync(ddst, (size_t)p_width * 2, cp->dst, (size_t)cp->dst_stride * 2,
                                  (size_t)p_width * 2, p_height, hipMemcpyHostToDevice, s));
  LavishWarpJob jb{};
  for (int k = 0; k < 6; ++k) jb.mat[k] = mat[k];
  jb.alpha = alpha;
  jb.beta = beta;
  jb.gamma = gamma;
  jb.delta = delta;
  jb.p_col = p_col;
  jb.p_row = p_row;
  jb.p_width = p_width;
  jb.p_height = p_height;
  jb.ref_off = -((int64_t)y0 * ww + x0);  // plane coordinates into the staged window
  LAVISH_CHECK(hipMemcpyAsync(djob, &jb, sizeof(jb), hipMemcpyHostToDevice, s));
  const int rc = warp_batch(dref, width, height, ww, dpred, p_width, ddst, p_width, djob, 1, ss_x,
                            ss_y, bd, sizeof(Pix) == 2, cp, s);
  if (rc != 0) {
    shim_reject("av1_warp_affine_hip", rc);
    return;
  }
  LAVISH_CHECK(hipMemcpy2DAsync(pred, (size_t)p_stride * sizeof(Pix), dpred,
                                (size_t)p_width * sizeof(Pix), (size_t)p_width * sizeof(Pix),
                                p_height, hipMemcpyDeviceToHost, s));
  if (cp->is_compound)
    LAVISH_CHECK(hipMemcpy2DAsync(cp->dst, (size_t)cp->dst_stride * 2, ddst, (size_t)p_width * 2,
                                  (size_t)p_width * 2, p_height, hipMemcpyDeviceToHost, s));
  LAVISH_CHECK(hipStreamSynchronize(s));
}

extern "C" void av1_warp_affine_hip(const int32_t* mat, const uint8_t* ref, int width, int height,
                                    int stride, uint8_t* pred, int p_col, int p_row, int p_width,
                                    int p_height, int p_stride, int subsampling_x,
                                    int subsampling_y, LavishConvolveParams* conv_params,
                                    int16_t alpha, int16_t beta, int16_t gamma, int16_t delta) {
  warp_shim<uint8_t>(mat, ref, width, height, stride, pred, p_col, p_row, p_width, p_height,
                     p_stride, subsampling_x, subsampling_y, 8, conv_params, alpha, beta, gamma,
                     delta);
}

extern "C" void av1_highbd_warp_affine_hip(const int32_t* mat, const uint16_t* ref, int width,
                                           int height, int stride, uint16_t* pred, int p_col,
                                           int p_row, int p_width, int p_height, int p_stride,
                                           int subsampling_x, int subsampling_y, int bd,
                                           LavishConvolveParams* conv_params, int16_t alpha,
                                           int16_t beta, int16_t gamma, int16_t delta) {
  warp_shim<uint16_t>(mat, ref, width, height, stride, pred, p_col, p_row, p_width, p_height,
                      p_stride, subsampling_x, subsampling_y, bd, conv_params, alpha, beta, gamma,
                      delta);
}
