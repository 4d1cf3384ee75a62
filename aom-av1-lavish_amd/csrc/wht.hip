// wht.hip -- lossless 4x4 Walsh-Hadamard transforms (SURVEY.md 8(a) row a5 /
// a17) and av1_quick_txfm, for gfx950.
//
//   av1_fwht4x4_c                 av1/encoder/hybrid_fwd_txfm.c:24-76
//   av1_highbd_iwht4x4_16_add_c   av1/common/av1_inv_txfm2d.c:20-79
//   av1_highbd_iwht4x4_1_add_c    av1/common/av1_inv_txfm2d.c:81-107
//   av1_highbd_iwht4x4_add        av1/common/idct.c:34-40 (eob > 1 -> 16)
//   av1_quick_txfm                av1/encoder/hybrid_fwd_txfm.c:315-336
//
// A 4x4 WHT is 16 coefficients and ~60 integer ops: one lane per block, the
// block's 16 values in registers; jobs are independent, so a wave covers 64
// blocks.  The lossless path is rare (segments with qindex 0); what matters is
// that an RTCD-bound encoder never aborts on it.
#include "lavish_internal.h"

namespace lavish {
namespace {

// one butterfly stage of the forward WHT (int64 tran_high_t arithmetic)
__device__ __forceinline__ void fwht_stage(int64_t& a1, int64_t& b1, int64_t& c1, int64_t& d1) {
  a1 += b1;
  d1 = d1 - c1;
  const int64_t e1 = (a1 - d1) >> 1;
  b1 = e1 - b1;
  c1 = e1 - c1;
  a1 -= c1;
  d1 += b1;
}

// in[r * stride + c] -> out[16] (the reference's layout: first pass writes
// row i of out from column i of in, second pass runs down the columns)
__device__ __forceinline__ void fwht4x4(const int16_t* in, int stride, int32_t* out) {
  int32_t t[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t a1 = in[0 * stride + i], b1 = in[1 * stride + i];
    int64_t c1 = in[2 * stride + i], d1 = in[3 * stride + i];
    fwht_stage(a1, b1, c1, d1);
    t[4 * i + 0] = (int32_t)a1;
    t[4 * i + 1] = (int32_t)c1;
    t[4 * i + 2] = (int32_t)d1;
    t[4 * i + 3] = (int32_t)b1;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t a1 = t[0 + i], b1 = t[4 + i], c1 = t[8 + i], d1 = t[12 + i];
    fwht_stage(a1, b1, c1, d1);
    out[0 + i] = (int32_t)(a1 * 4);  // UNIT_QUANT_FACTOR
    out[4 + i] = (int32_t)(c1 * 4);
    out[8 + i] = (int32_t)(d1 * 4);
    out[12 + i] = (int32_t)(b1 * 4);
  }
}

// tran_low_t (int32) arithmetic of the inverse, wrapping like the C
__device__ __forceinline__ int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
__device__ __forceinline__ int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

__device__ __forceinline__ void iwht_stage(int32_t& a1, int32_t& b1, int32_t& c1, int32_t& d1) {
  a1 = wadd(a1, c1);
  d1 = wsub(d1, b1);
  const int32_t e1 = wsub(a1, d1) >> 1;
  b1 = wsub(e1, b1);
  c1 = wsub(e1, c1);
  a1 = wsub(a1, b1);
  d1 = wadd(d1, c1);
}

template <typename Pix>
__device__ __forceinline__ void clip_add(Pix* p, int32_t v, int maxv) {
  const int x = (int)*p + v;
  *p = (Pix)(x < 0 ? 0 : (x > maxv ? maxv : x));
}

template <typename Pix>
__device__ __forceinline__ void iwht4x4_add(const int32_t* in, Pix* dst, int stride, int eob,
                                            int maxv) {
  if (eob > 1) {  // av1_highbd_iwht4x4_16_add_c
    int32_t o[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int32_t a1 = in[0 + i] >> 2, c1 = in[4 + i] >> 2;  // UNIT_QUANT_SHIFT
      int32_t d1 = in[8 + i] >> 2, b1 = in[12 + i] >> 2;
      iwht_stage(a1, b1, c1, d1);
      o[0 + i] = a1;
      o[4 + i] = b1;
      o[8 + i] = c1;
      o[12 + i] = d1;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int32_t a1 = o[4 * i + 0], c1 = o[4 * i + 1], d1 = o[4 * i + 2], b1 = o[4 * i + 3];
      iwht_stage(a1, b1, c1, d1);
      clip_add(dst + 0 * stride + i, a1, maxv);
      clip_add(dst + 1 * stride + i, b1, maxv);
      clip_add(dst + 2 * stride + i, c1, maxv);
      clip_add(dst + 3 * stride + i, d1, maxv);
    }
  } else {  // av1_highbd_iwht4x4_1_add_c
    int32_t a1 = in[0] >> 2;
    int32_t e1 = a1 >> 1;
    a1 = wsub(a1, e1);
    const int32_t t[4] = {a1, e1, e1, e1};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int32_t e = t[i] >> 1;
      const int32_t a = wsub(t[i], e);
      clip_add(dst + 0 * stride + i, a, maxv);
      clip_add(dst + 1 * stride + i, e, maxv);
      clip_add(dst + 2 * stride + i, e, maxv);
      clip_add(dst + 3 * stride + i, e, maxv);
    }
  }
}

__global__ __launch_bounds__(64) void fwht_kernel(const int16_t* src, int stride,
                                                  const LavishPixJob* jobs, int njobs,
                                                  int32_t* coeff) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= njobs) return;
  const LavishPixJob jb = jobs[j];
  int32_t o[16];
  fwht4x4(src + jb.src_off, stride, o);
#pragma unroll
  for (int i = 0; i < 16; ++i) coeff[jb.aux_off + i] = o[i];
}

template <typename Pix>
__global__ __launch_bounds__(64) void iwht_kernel(const int32_t* dq, const LavishInvJob* jobs,
                                                  int njobs, Pix* dst, int stride, int maxv) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= njobs) return;
  const LavishInvJob jb = jobs[j];
  if (jb.eob == 0) return;  // av1_inverse_transform_block returns early on eob 0
  int32_t c[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) c[i] = dq[jb.coeff_off + i];
  iwht4x4_add(c, dst + jb.dst_off, stride, jb.eob, maxv);
}

}  // namespace
}  // namespace lavish

using namespace lavish;

extern "C" {

int lavish_fwht4x4_batch(const int16_t* src_diff, int stride, const LavishPixJob* jobs, int njobs,
                         int32_t* coeff, void* stream) {
  if (njobs <= 0) return 0;
  hipLaunchKernelGGL(fwht_kernel, dim3((njobs + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     src_diff, stride, jobs, njobs, coeff);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

int lavish_iwht4x4_add_batch(const int32_t* dqcoeff, const LavishInvJob* jobs, int njobs,
                             void* dst, int dst_stride, int bit_depth, int highbd, void* stream) {
  if (njobs <= 0) return 0;
  if (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) return -3;
  if (!highbd && bit_depth != 8) return -3;
  const int maxv = (1 << bit_depth) - 1;
  hipStream_t s = (hipStream_t)stream;
  if (highbd)
    hipLaunchKernelGGL(iwht_kernel<uint16_t>, dim3((njobs + 63) / 64), dim3(64), 0, s, dqcoeff,
                       jobs, njobs, (uint16_t*)dst, dst_stride, maxv);
  else
    hipLaunchKernelGGL(iwht_kernel<uint8_t>, dim3((njobs + 63) / 64), dim3(64), 0, s, dqcoeff,
                       jobs, njobs, (uint8_t*)dst, dst_stride, maxv);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

// ---- per-call shims (host buffers) ----
void av1_fwht4x4_hip(const int16_t* input, int32_t* output, int stride) {
  hipStream_t s = shim_stream();
  char* base = (char*)shim_scratch(4096);
  int16_t* din = (int16_t*)base;
  LavishPixJob* dj = (LavishPixJob*)(base + 256);
  int32_t* dout = (int32_t*)(base + 512);
  LavishPixJob jb{};
  LAVISH_CHECK(hipMemcpy2DAsync(din, 4 * sizeof(int16_t), input, (size_t)stride * sizeof(int16_t),
                                4 * sizeof(int16_t), 4, hipMemcpyHostToDevice, s));
  LAVISH_CHECK(hipMemcpyAsync(dj, &jb, sizeof(jb), hipMemcpyHostToDevice, s));
  lavish_fwht4x4_batch(din, 4, dj, 1, dout, s);
  LAVISH_CHECK(hipMemcpyAsync(output, dout, 16 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  LAVISH_CHECK(hipStreamSynchronize(s));
}

static void iwht_shim(const int32_t* input, uint16_t* dest, int stride, int eob, int bd) {
  hipStream_t s = shim_stream();
  char* base = (char*)shim_scratch(4096);
  int32_t* din = (int32_t*)base;
  LavishInvJob* dj = (LavishInvJob*)(base + 256);
  uint16_t* dd = (uint16_t*)(base + 512);
  LavishInvJob jb{};
  jb.eob = eob;
  LAVISH_CHECK(hipMemcpyAsync(din, input, 16 * sizeof(int32_t), hipMemcpyHostToDevice, s));
  LAVISH_CHECK(hipMemcpyAsync(dj, &jb, sizeof(jb), hipMemcpyHostToDevice, s));
  LAVISH_CHECK(hipMemcpy2DAsync(dd, 4 * sizeof(uint16_t), dest, (size_t)stride * sizeof(uint16_t),
                                4 * sizeof(uint16_t), 4, hipMemcpyHostToDevice, s));
  const int rc = lavish_iwht4x4_add_batch(din, dj, 1, dd, 4, bd, 1, s);
  if (rc) shim_reject("lavish_iwht4x4_add_batch", rc);
  LAVISH_CHECK(hipMemcpy2DAsync(dest, (size_t)stride * sizeof(uint16_t), dd, 4 * sizeof(uint16_t),
                                4 * sizeof(uint16_t), 4, hipMemcpyDeviceToHost, s));
  LAVISH_CHECK(hipStreamSynchronize(s));
}

// av1/common/av1_rtcd_defs.pl:217-219 (tagged u16 destinations)
void av1_highbd_iwht4x4_16_add_hip(const int32_t* input, uint8_t* dest, int dest_stride, int bd) {
  iwht_shim(input, (uint16_t*)((uintptr_t)dest << 1), dest_stride, 16, bd);
}
void av1_highbd_iwht4x4_1_add_hip(const int32_t* input, uint8_t* dest, int dest_stride, int bd) {
  iwht_shim(input, (uint16_t*)((uintptr_t)dest << 1), dest_stride, 1, bd);
}

}  // extern "C"

namespace lavish {
void iwht_host(const int32_t* input, uint16_t* dest, int stride, int eob, int bd) {
  iwht_shim(input, dest, stride, eob, bd);
}
}  // namespace lavish
