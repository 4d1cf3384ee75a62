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

/* ---------------------------------------------------------------------------
 * prune_tx_2D (av1/encoder/tx_search.c:1487-1641) on top of the features:
 *   av1_nn_predict_c              av1/encoder/ml.c:31-70 (+ prec reduce :19-26)
 *   av1_nn_fast_softmax_16_c      ml.c:159-171, approx_exp aom_dsp/mathutils.h:130-144
 *   get_adaptive_thresholds       tx_search.c:1394-1409 (the table comes from
 *                                 the caller: prune_2D_adaptive_thresholds)
 *   av1_sort_fi32_8 / _16         av1/encoder/sorting_network.h
 * -------------------------------------------------------------------------*/
void orc_nn_predict(const float *input_nodes, const OrcNNConfig *c, int reduce_prec,
                    float *output) {
  float buf[2][128];
  int nin = c->num_inputs, bi = 0;
  for (int layer = 0; layer < c->num_hidden_layers; ++layer) {
    const float *w = c->weights[layer], *b = c->bias[layer];
    float *out = buf[bi];
    const int nout = c->num_hidden_nodes[layer];
    for (int node = 0; node < nout; ++node) {
      float val = b[node];
      for (int i = 0; i < nin; ++i) val += w[node * nin + i] * input_nodes[i];
      out[node] = val > 0.0f ? val : 0.0f;
    }
    nin = nout;
    input_nodes = out;
    bi = 1 - bi;
  }
  const float *w = c->weights[c->num_hidden_layers], *b = c->bias[c->num_hidden_layers];
  for (int node = 0; node < c->num_outputs; ++node) {
    float val = b[node];
    for (int i = 0; i < nin; ++i) val += w[node * nin + i] * input_nodes[i];
    output[node] = val;
  }
  if (reduce_prec) {
    const float inv_prec = (float)(1.0 / 512);
    for (int i = 0; i < c->num_outputs; ++i)
      output[i] = ((int)(output[i] * 512 + 0.5)) * inv_prec;
  }
}

static float orc_approx_exp(float y) {
  union {
    float f;
    int32_t i;
  } u;
  u.i = ((int32_t)(y * ((1 << 23) / 0.69314718056f))) + ((127 << 23) - 60801);
  return u.f;
}

static void orc_fast_softmax_16(float *v) {
  float mx = v[0];
  for (int i = 1; i < 16; ++i) mx = mx > v[i] ? mx : v[i];
  float sum = 0.0f;
  for (int i = 0; i < 16; ++i) {
    const float t = v[i] - mx;
    v[i] = orc_approx_exp(t > -10.0f ? t : -10.0f);
    sum += v[i];
  }
  for (int i = 0; i < 16; ++i) v[i] /= sum;
}

/* comparator sequences of the sorting networks (descending, ties keep i) */
static const uint8_t kSort16[65][2] = {
  { 0, 1 },  { 2, 3 },   { 4, 5 },   { 6, 7 },   { 8, 9 },   { 10, 11 }, { 12, 13 },
  { 14, 15 }, { 0, 2 },  { 1, 3 },   { 4, 6 },   { 5, 7 },   { 8, 10 },  { 9, 11 },
  { 12, 14 }, { 13, 15 }, { 1, 2 },  { 5, 6 },   { 0, 4 },   { 3, 7 },   { 9, 10 },
  { 13, 14 }, { 8, 12 }, { 11, 15 }, { 1, 5 },   { 2, 6 },   { 9, 13 },  { 10, 14 },
  { 0, 8 },  { 7, 15 },  { 1, 4 },   { 3, 6 },   { 9, 12 },  { 11, 14 }, { 2, 4 },
  { 3, 5 },  { 10, 12 }, { 11, 13 }, { 1, 9 },   { 6, 14 },  { 3, 4 },   { 11, 12 },
  { 1, 8 },  { 2, 10 },  { 5, 13 },  { 7, 14 },  { 3, 11 },  { 2, 8 },   { 4, 12 },
  { 7, 13 }, { 3, 10 },  { 5, 12 },  { 3, 9 },   { 6, 12 },  { 3, 8 },   { 7, 12 },
  { 5, 9 },  { 6, 10 },  { 4, 8 },   { 7, 11 },  { 5, 8 },   { 7, 10 },  { 6, 8 },
  { 7, 9 },  { 7, 8 },
};
static const uint8_t kSort8[19][2] = {
  { 0, 1 }, { 2, 3 }, { 4, 5 }, { 6, 7 }, { 0, 2 }, { 1, 3 }, { 4, 6 },
  { 5, 7 }, { 1, 2 }, { 5, 6 }, { 0, 4 }, { 3, 7 }, { 1, 5 }, { 2, 6 },
  { 1, 4 }, { 3, 6 }, { 2, 4 }, { 3, 5 }, { 3, 4 },
};

static void orc_sort_network(float *k, int *v, const uint8_t (*pairs)[2], int n) {
  for (int p = 0; p < n; ++p) {
    const int i = pairs[p][0], j = pairs[p][1];
    const int ge = k[i] >= k[j];
    const float maxf = ge ? k[i] : k[j], minf = ge ? k[j] : k[i];
    const int maxi = ge ? v[i] : v[j], mini = ge ? v[j] : v[i];
    k[i] = maxf;
    k[j] = minf;
    v[i] = maxi;
    v[j] = mini;
  }
}

void orc_sort_fi32(float *k, int *v, int n) {
  if (n == 8) orc_sort_network(k, v, kSort8, 19);
  else orc_sort_network(k, v, kSort16, 65);
}

/* get_adaptive_thresholds' aggressiveness index; -1 when not applicable */
int orc_prune_aggressiveness(int tx_set_type, int prune_mode) {
  static const int aggr[5][2] = { { 4, 1 }, { 6, 3 }, { 9, 6 }, { 9, 6 }, { 12, 9 } };
  if (prune_mode < 1 || prune_mode > 5) return -1;
  if (tx_set_type == 5) return aggr[prune_mode - 1][0]; /* EXT_TX_SET_ALL16 */
  if (tx_set_type == 4) return aggr[prune_mode - 1][1]; /* EXT_TX_SET_DTT9_IDTX_1DDCT */
  return -1;
}

/* tx_type_table_2D (tx_search.c:1493-1498) as TX_TYPE values */
static const int kTable2D[16] = { 0, 2, 5, 10, 1, 3, 7, 12, 4, 8, 6, 14, 11, 13, 15, 9 };

/* one block: the body of prune_tx_2D after its feature extraction */
static void orc_prune_one(const float *hf, const float *vf, const OrcNNConfig *hor,
                          const OrcNNConfig *ver, float thresh, int prune_mode,
                          uint16_t *mask, uint8_t *map) {
  float hs[4], vs[4], raw[16];
  orc_nn_predict(hf, hor, 1, hs);
  orc_nn_predict(vf, ver, 1, vs);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) raw[i * 4 + j] = vs[i] * hs[j];
  orc_fast_softmax_16(raw);
  int max_i = 0, count = 0;
  float max_score = 0.0f, sum = 0.0f;
  uint16_t allow = 0;
  int allowed[16];
  float sc[16];
  for (int i = 0; i < 16; ++i) {
    allowed[i] = 255;
    sc[i] = -1;
  }
  for (int t = 0; t < 16; ++t) {
    if (!(*mask & (1 << kTable2D[t]))) continue;
    if (raw[t] > max_score) {
      max_score = raw[t];
      max_i = t;
    }
    if (raw[t] >= thresh) {
      allow |= (uint16_t)(1 << kTable2D[t]);
      sum += raw[t];
      sc[count] = raw[t];
      allowed[count] = kTable2D[t];
      count++;
    }
  }
  if (!(allow & (1 << kTable2D[max_i]))) {
    allow |= (uint16_t)(1 << kTable2D[max_i]);
    for (int i = 0; i < 16; ++i) map[i] = (uint8_t)kTable2D[i];
    *mask = allow;
    return;
  }
  orc_sort_fi32(sc, allowed, count <= 8 ? 8 : 16);
  if (prune_mode >= 4) {
    float temp = 0.0f, ratio = 0.0f;
    int t, n = 0;
    const float inv_sum = 100 / sum;
    for (t = 0; t < count; t++) {
      if (ratio > 30.0 && n >= 2) break;
      temp += sc[t];
      ratio = temp * inv_sum;
      n++;
    }
    for (; t < count; t++) allow &= (uint16_t)~(1 << allowed[t]);
  }
  for (int i = 0; i < 16; ++i) map[i] = (uint8_t)allowed[i];
  *mask = allow;
}

/* prune_tx_2D for every full bw x bh block of a residual plane (raster
 * order).  thresholds: the tx size's row of prune_2D_adaptive_thresholds
 * (NULL, or hor / ver NULL: no model -> masks pass through, identity map).
 * allowed_in: per block (or NULL: allowed_default for all). */
long orc_prune_tx_2d(const int16_t *residual, int stride, int width, int height, int bw, int bh,
                     int tx_set_type, int prune_mode, const float *thresholds,
                     const OrcNNConfig *hor, const OrcNNConfig *ver, const uint16_t *allowed_in,
                     uint16_t allowed_default, uint16_t *allowed_out, uint8_t *txk_map) {
  const int nbx = width / bw, nby = height / bh;
  const int hn = bw <= 8 ? bw : bw / 2, vn = bh <= 8 ? bh : bh / 2;
  const int ag = orc_prune_aggressiveness(tx_set_type, prune_mode);
  const int active = ag >= 0 && thresholds && hor && ver;
  for (int by = 0; by < nby; ++by)
    for (int bx = 0; bx < nbx; ++bx) {
      const long blk = (long)by * nbx + bx;
      uint16_t mask = allowed_in ? allowed_in[blk] : allowed_default;
      uint8_t *map = txk_map + blk * 16;
      for (int i = 0; i < 16; ++i) map[i] = (uint8_t)i;
      if (active) {
        float hf[16] = { 0 }, vf[16] = { 0 };
        const int16_t *d = residual + (size_t)by * bh * stride + (size_t)bx * bw;
        orc_energy_distribution_finer(d, stride, bw, bh, hf, vf);
        orc_horver_correlation_full(d, stride, bw, bh, &hf[hn - 1], &vf[vn - 1]);
        orc_prune_one(hf, vf, hor, ver, thresholds[ag], prune_mode, &mask, map);
      }
      allowed_out[blk] = mask;
    }
  return (long)nbx * nby;
}
