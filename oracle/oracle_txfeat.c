/* oracle_txfeat.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the TX-type pruning features
 * that prune_tx_2D (av1/encoder/tx_search.c:1487-1537) feeds to its two
 * neural nets:
 *   av1_get_horver_correlation_full_c   av1/encoder/rdopt.c:514-609
 *   get_energy_distribution_finer       av1/encoder/tx_search.c:1411-1473
 * Single-precision arithmetic in the reference's operation order (x86-64
 * SSE: no excess precision, no contraction).
 */
#include <math.h>
#include <string.h>

#include "oracle.h"

void orc_horver_correlation_full(const int16_t *diff, int stride, int width, int height,
                                 float *hcorr, float *vcorr) {
  int64_t x_sum = 0, x2_sum = 0, xy_sum = 0, xz_sum = 0;
  int64_t x_firstrow = 0, x_finalrow = 0, x_firstcol = 0, x_finalcol = 0;
  int64_t x2_firstrow = 0, x2_finalrow = 0, x2_firstcol = 0, x2_finalcol = 0;
  /* first row: horizontal pairs */
  x_sum += diff[0];
  x2_sum += diff[0] * diff[0];
  x_firstrow += diff[0];
  x2_firstrow += diff[0] * diff[0];
  for (int j = 1; j < width; ++j) {
    const int16_t x = diff[j], y = diff[j - 1];
    x_sum += x;
    x_firstrow += x;
    x2_sum += x * x;
    x2_firstrow += x * x;
    xy_sum += x * y;
  }
  /* first column: vertical pairs */
  x_firstcol += diff[0];
  x2_firstcol += diff[0] * diff[0];
  for (int i = 1; i < height; ++i) {
    const int16_t x = diff[i * stride], z = diff[(i - 1) * stride];
    x_sum += x;
    x_firstcol += x;
    x2_sum += x * x;
    x2_firstcol += x * x;
    xz_sum += x * z;
  }
  /* the rest */
  for (int i = 1; i < height; ++i)
    for (int j = 1; j < width; ++j) {
      const int16_t x = diff[i * stride + j], y = diff[i * stride + j - 1];
      const int16_t z = diff[(i - 1) * stride + j];
      x_sum += x;
      x2_sum += x * x;
      xy_sum += x * y;
      xz_sum += x * z;
    }
  for (int j = 0; j < width; ++j) {
    const int v = diff[(height - 1) * stride + j];
    x_finalrow += v;
    x2_finalrow += v * v;
  }
  for (int i = 0; i < height; ++i) {
    const int v = diff[i * stride + width - 1];
    x_finalcol += v;
    x2_finalcol += v * v;
  }
  const int64_t xhor_sum = x_sum - x_finalcol, xver_sum = x_sum - x_finalrow;
  const int64_t y_sum = x_sum - x_firstcol, z_sum = x_sum - x_firstrow;
  const int64_t x2hor_sum = x2_sum - x2_finalcol, x2ver_sum = x2_sum - x2_finalrow;
  const int64_t y2_sum = x2_sum - x2_firstcol, z2_sum = x2_sum - x2_firstrow;
  const float num_hor = (float)(height * (width - 1));
  const float num_ver = (float)((height - 1) * width);
  const float xhor_var_n = x2hor_sum - (xhor_sum * xhor_sum) / num_hor;
  const float xver_var_n = x2ver_sum - (xver_sum * xver_sum) / num_ver;
  const float y_var_n = y2_sum - (y_sum * y_sum) / num_hor;
  const float z_var_n = z2_sum - (z_sum * z_sum) / num_ver;
  const float xy_var_n = xy_sum - (xhor_sum * y_sum) / num_hor;
  const float xz_var_n = xz_sum - (xver_sum * z_sum) / num_ver;
  if (xhor_var_n > 0 && y_var_n > 0) {
    *hcorr = xy_var_n / sqrtf(xhor_var_n * y_var_n);
    *hcorr = *hcorr < 0 ? 0 : *hcorr;
  } else {
    *hcorr = 1.0;
  }
  if (xver_var_n > 0 && z_var_n > 0) {
    *vcorr = xz_var_n / sqrtf(xver_var_n * z_var_n);
    *vcorr = *vcorr < 0 ? 0 : *vcorr;
  } else {
    *vcorr = 1.0;
  }
}

void orc_energy_distribution_finer(const int16_t *diff, int stride, int bw, int bh,
                                   float *hordist, float *verdist) {
  unsigned int esq[256];
  const int w_shift = bw <= 8 ? 0 : 1, h_shift = bh <= 8 ? 0 : 1;
  const int esq_w = bw >> w_shift, esq_h = bh >> h_shift, esq_sz = esq_w * esq_h;
  memset(esq, 0, esq_sz * sizeof(esq[0]));
  for (int i = 0; i < bh; i++) {
    unsigned int *row = esq + (i >> h_shift) * esq_w;
    const int16_t *d = diff + i * stride;
    if (w_shift)
      for (int j = 0; j < bw; j += 2) row[j >> 1] += (d[j] * d[j] + d[j + 1] * d[j + 1]);
    else
      for (int j = 0; j < bw; j++) row[j] += d[j] * d[j];
  }
  uint64_t total = 0;
  for (int i = 0; i < esq_sz; i++) total += esq[i];
  if (total == 0) {
    const float hor_val = 1.0f / esq_w, ver_val = 1.0f / esq_h;
    for (int j = 0; j < esq_w - 1; j++) hordist[j] = hor_val;
    for (int i = 0; i < esq_h - 1; i++) verdist[i] = ver_val;
    return;
  }
  const float e_recip = 1.0f / (float)total;
  memset(hordist, 0, (esq_w - 1) * sizeof(hordist[0]));
  memset(verdist, 0, (esq_h - 1) * sizeof(verdist[0]));
  int i, j;
  for (i = 0; i < esq_h - 1; i++) {
    const unsigned int *row = esq + i * esq_w;
    for (j = 0; j < esq_w - 1; j++) {
      hordist[j] += (float)row[j];
      verdist[i] += (float)row[j];
    }
    verdist[i] += (float)row[j];
  }
  const unsigned int *row = esq + i * esq_w;
  for (j = 0; j < esq_w - 1; j++) hordist[j] += (float)row[j];
  for (j = 0; j < esq_w - 1; j++) hordist[j] *= e_recip;
  for (i = 0; i < esq_h - 1; i++) verdist[i] *= e_recip;
}

/* prune_tx_2D's NN inputs for every full bw x bh block of a residual plane
 * (raster order): hfeatures[blk][16] = hordist[0 .. esq_w-2], hcorr at
 * esq_w-1; vfeatures likewise (tx_search.c:1516-1529); unused entries 0. */
long orc_tx_prune_features(const int16_t *residual, int stride, int width, int height, int bw,
                           int bh, float *hfeatures, float *vfeatures) {
  const int nbx = width / bw, nby = height / bh;
  const int hn = bw <= 8 ? bw : bw / 2, vn = bh <= 8 ? bh : bh / 2;
  for (int by = 0; by < nby; ++by)
    for (int bx = 0; bx < nbx; ++bx) {
      const long blk = (long)by * nbx + bx;
      const int16_t *d = residual + (size_t)by * bh * stride + (size_t)bx * bw;
      float *hf = hfeatures + blk * 16, *vf = vfeatures + blk * 16;
      memset(hf, 0, 16 * sizeof(float));
      memset(vf, 0, 16 * sizeof(float));
      orc_energy_distribution_finer(d, stride, bw, bh, hf, vf);
      orc_horver_correlation_full(d, stride, bw, bh, &hf[hn - 1], &vf[vn - 1]);
    }
  return (long)nbx * nby;
}
