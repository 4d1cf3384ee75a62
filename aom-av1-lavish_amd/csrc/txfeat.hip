// txfeat.hip -- TX-type pruning features for gfx950.
//
// prune_tx_2D (av1/encoder/tx_search.c:1487-1537) scores the 16 TX types of
// a block with two small neural nets whose inputs are
//   get_energy_distribution_finer (tx_search.c:1411-1473): the block's
//     energy on a (w/2 for w > 8) x (h/2 for h > 8) grid, projected on the
//     columns / rows and normalised (float), and
//   av1_get_horver_correlation_full (av1/encoder/rdopt.c:514-609, an RTCD
//     function): the horizontal / vertical lag-1 correlation of the residual
//     (float).
// One 256-thread workgroup per block: the integer sums are exact (int64 /
// u32 accumulations, reduced through LDS), the float tails run in the
// reference's operation order with IEEE single precision -- correctly
// rounded division and sqrt (hipcc's default), no contraction -- so the
// results match the C reference bit for bit (the reference's own test allows
// 1e-6, test/horver_correlation_test.cc:70-73).
#include "lavish_internal.h"

#pragma clang fp contract(off)

namespace lavish {
namespace {

constexpr int kTfThreads = 256;

// 12 exact sums of av1_get_horver_correlation_full
struct HvSums {
  int64_t v[12];  // x, x2, xy, xz, firstrow, finalrow, firstcol, finalcol, and their x2
};

__device__ __forceinline__ int64_t wg_sum64(int64_t v, int64_t* red) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// horver correlation of the w x h block at d (stride): every thread returns
// the same (hcorr, vcorr)
__device__ void horver(const int16_t* d, int stride, int w, int h, float& hcorr, float& vcorr,
                       int64_t* red) {
  int64_t s[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int p = threadIdx.x; p < w * h; p += kTfThreads) {
    const int i = p / w, j = p - i * w;
    const int x = d[(int64_t)i * stride + j];
    const int x2 = x * x;
    s[0] += x;
    s[1] += x2;
    if (j >= 1) s[2] += x * d[(int64_t)i * stride + j - 1];
    if (i >= 1) s[3] += x * d[(int64_t)(i - 1) * stride + j];
    if (i == 0) { s[4] += x; s[8] += x2; }
    if (i == h - 1) { s[5] += x; s[9] += x2; }
    if (j == 0) { s[6] += x; s[10] += x2; }
    if (j == w - 1) { s[7] += x; s[11] += x2; }
  }
#pragma unroll
  for (int k = 0; k < 12; ++k) s[k] = wg_sum64(s[k], red);
  const int64_t x_sum = s[0], x2_sum = s[1], xy_sum = s[2], xz_sum = s[3];
  const int64_t xhor_sum = x_sum - s[7], xver_sum = x_sum - s[5];
  const int64_t y_sum = x_sum - s[6], z_sum = x_sum - s[4];
  const int64_t x2hor_sum = x2_sum - s[11], x2ver_sum = x2_sum - s[9];
  const int64_t y2_sum = x2_sum - s[10], z2_sum = x2_sum - s[8];
  const float num_hor = (float)(h * (w - 1));
  const float num_ver = (float)((h - 1) * w);
  // C: int64 - (int64 / float): both int64 operands convert to float
  const float xhor_var_n = (float)x2hor_sum - (float)(xhor_sum * xhor_sum) / num_hor;
  const float xver_var_n = (float)x2ver_sum - (float)(xver_sum * xver_sum) / num_ver;
  const float y_var_n = (float)y2_sum - (float)(y_sum * y_sum) / num_hor;
  const float z_var_n = (float)z2_sum - (float)(z_sum * z_sum) / num_ver;
  const float xy_var_n = (float)xy_sum - (float)(xhor_sum * y_sum) / num_hor;
  const float xz_var_n = (float)xz_sum - (float)(xver_sum * z_sum) / num_ver;
  if (xhor_var_n > 0 && y_var_n > 0) {
    hcorr = xy_var_n / sqrtf(xhor_var_n * y_var_n);
    hcorr = hcorr < 0 ? 0 : hcorr;
  } else {
    hcorr = 1.0f;
  }
  if (xver_var_n > 0 && z_var_n > 0) {
    vcorr = xz_var_n / sqrtf(xver_var_n * z_var_n);
    vcorr = vcorr < 0 ? 0 : vcorr;
  } else {
    vcorr = 1.0f;
  }
}

// av1_get_horver_correlation_full over jobs of w x h blocks
__global__ __launch_bounds__(kTfThreads) void horver_kernel(const int16_t* __restrict__ res,
                                                            int stride, int bw, int nbx, int w,
                                                            int h, float* hcorr, float* vcorr) {
  __shared__ int64_t red[4];
  const int blk = blockIdx.x;
  const int by = blk / nbx, bx = blk - by * nbx;
  float hc, vc;
  horver(res + (int64_t)by * h * stride + (int64_t)bx * bw, stride, w, h, hc, vc, red);
  if (threadIdx.x == 0) {
    hcorr[blk] = hc;
    vcorr[blk] = vc;
  }
}

// prune_tx_2D's two feature vectors (tx_search.c:1516-1529) per block:
// [0, esq_w - 1) energy projection, [esq_w - 1] correlation; rest zero
__global__ __launch_bounds__(kTfThreads) void prune_features_kernel(
    const int16_t* __restrict__ res, int stride, int nbx, int bw, int bh, float* hfeat,
    float* vfeat) {
  __shared__ int64_t red[4];
  __shared__ uint32_t esq[256];
  const int blk = blockIdx.x;
  const int by = blk / nbx, bx = blk - by * nbx;
  const int16_t* d = res + (int64_t)by * bh * stride + (int64_t)bx * bw;
  const int ws = bw <= 8 ? 0 : 1, hs = bh <= 8 ? 0 : 1;
  const int ew = bw >> ws, eh = bh >> hs, esz = ew * eh;
  // downscaled energies (get_energy_distribution_finer's esq)
  uint64_t tot = 0;
  for (int e = threadIdx.x; e < esz; e += kTfThreads) {
    const int ei = e / ew, ej = e - ei * ew;
    uint32_t acc = 0;
    for (int yy = 0; yy <= hs; ++yy)
      for (int xx = 0; xx <= ws; ++xx) {
        const int v = d[(int64_t)((ei << hs) + yy) * stride + (ej << ws) + xx];
        acc += (uint32_t)(v * v);
      }
    esq[e] = acc;
    tot += acc;
  }
  const uint64_t total = (uint64_t)wg_sum64((int64_t)tot, red);  // also orders esq[]
  float* hf = hfeat + (int64_t)blk * 16;
  float* vf = vfeat + (int64_t)blk * 16;
  const int t = threadIdx.x;
  if (total == 0) {
    if (t < ew - 1) hf[t] = 1.0f / ew;
    if (t >= 16 && t - 16 < eh - 1) vf[t - 16] = 1.0f / eh;
  } else {
    const float e_recip = 1.0f / (float)total;
    if (t < ew - 1) {  // hordist[t]: rows in order
      float a = 0.0f;
      for (int i = 0; i < eh; ++i) a += (float)esq[i * ew + t];
      hf[t] = a * e_recip;
    }
    if (t >= 16 && t - 16 < eh - 1) {  // verdist[i]: columns in order
      const int i = t - 16;
      float a = 0.0f;
      for (int j = 0; j < ew; ++j) a += (float)esq[i * ew + j];
      vf[i] = a * e_recip;
    }
  }
  if (t >= 32 && t < 48 && t - 32 >= ew) hf[t - 32] = 0.0f;
  if (t >= 48 && t < 64 && t - 48 >= eh) vf[t - 48] = 0.0f;
  float hc, vc;
  horver(d, stride, bw, bh, hc, vc, red);
  if (t == 0) {
    hf[ew - 1] = hc;
    vf[eh - 1] = vc;
  }
}

}  // namespace

int horver_batch(const int16_t* residual, int stride, int width, int height, int bw, int bh,
                 float* hcorr, float* vcorr, hipStream_t s) {
  if (bw < 2 || bh < 2 || bw > 128 || bh > 128) return -1;
  if (width < 0 || height < 0 || stride < width) return -4;
  const int nbx = width / bw, nb = nbx * (height / bh);
  if (nb == 0) return 0;
  hipLaunchKernelGGL(horver_kernel, dim3(nb), dim3(kTfThreads), 0, s, residual, stride, bw, nbx,
                     bw, bh, hcorr, vcorr);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

}  // namespace lavish

using namespace lavish;

extern "C" int lavish_horver_correlation_batch(const int16_t* residual, int stride, int width,
                                               int height, int bw, int bh, float* hcorr,
                                               float* vcorr, void* stream) {
  return horver_batch(residual, stride, width, height, bw, bh, hcorr, vcorr,
                      (hipStream_t)stream);
}

extern "C" int lavish_tx_prune_features_batch(const int16_t* residual, int stride, int width,
                                              int height, int tx_size, float* hfeatures,
                                              float* vfeatures, void* stream) {
  if (tx_size < 0 || tx_size >= 19) return -1;
  const int bw = tx_w(tx_size), bh = tx_h(tx_size);
  if (bw > 32 || bh > 32) return -2;  // prune_tx_2D: at most 16 features per direction
  if (width < 0 || height < 0 || stride < width) return -4;
  const int nbx = width / bw, nb = nbx * (height / bh);
  if (nb == 0) return 0;
  hipLaunchKernelGGL(prune_features_kernel, dim3(nb), dim3(kTfThreads), 0, (hipStream_t)stream,
                     residual, stride, nbx, bw, bh, hfeatures, vfeatures);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}
