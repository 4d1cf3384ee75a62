/*
 * oracle_dsp.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Pixel-domain kernels of the reference, restated:
 *   sad / _skip / _avg          aom_dsp/sad.c:22-69, aom_comp_avg_pred_c
 *                               aom_dsp/variance.c:285-298
 *   highbd_sad                  aom_dsp/sad.c:240-256
 *   variance / MSE              aom_dsp/variance.c:38-55,123-130,230-238
 *   bilinear sub-pixel variance aom_dsp/variance.c:73-145,
 *                               bilinear_filters_2t aom_dsp/aom_filter.h:47-50
 *   highbd_variance64 + 8/10/12 aom_dsp/variance.c:321-408
 *   aom_sse_c / aom_highbd_sse_c   aom_dsp/sse.c:19-54
 *   aom_subtract_block(_c/highbd)  aom_dsp/subtract.c:20-54
 *   aom_sum_squares_2d_i16_c       aom_dsp/sum_squares.c:16-30
 *   aom_hadamard_{4x4,8x8,16x16,32x32}_c, aom_satd_c  aom_dsp/avg.c:102-348,509
 *   av1_block_error_c / highbd     av1/encoder/rdopt.c:635-682
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

unsigned int orc_sad(const uint8_t *a, int as, const uint8_t *b, int bs, int w,
                     int h) {
  unsigned int s = 0;
  for (int y = 0; y < h; ++y, a += as, b += bs)
    for (int x = 0; x < w; ++x) s += (unsigned)abs(a[x] - b[x]);
  return s;
}

unsigned int orc_sad_skip(const uint8_t *a, int as, const uint8_t *b, int bs,
                          int w, int h) {
  return 2 * orc_sad(a, 2 * as, b, 2 * bs, w, h / 2);
}

unsigned int orc_sad_avg(const uint8_t *src, int ss, const uint8_t *ref,
                         int rs, int w, int h, const uint8_t *second_pred) {
  uint8_t *comp = (uint8_t *)malloc((size_t)w * h);
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j)
      comp[i * w + j] =
          (uint8_t)((second_pred[i * w + j] + ref[i * rs + j] + 1) >> 1);
  const unsigned int s = orc_sad(src, ss, comp, w, w, h);
  free(comp);
  return s;
}

unsigned int orc_highbd_sad(const uint16_t *a, int as, const uint16_t *b,
                            int bs, int w, int h) {
  unsigned int s = 0;
  for (int y = 0; y < h; ++y, a += as, b += bs)
    for (int x = 0; x < w; ++x) s += (unsigned)abs(a[x] - b[x]);
  return s;
}

static void var_sums(const uint8_t *a, int as, const uint8_t *b, int bs, int w,
                     int h, uint32_t *sse, int *sum) {
  int s = 0;
  uint32_t q = 0;
  for (int i = 0; i < h; ++i, a += as, b += bs)
    for (int j = 0; j < w; ++j) {
      const int d = a[j] - b[j];
      s += d;
      q += (uint32_t)(d * d);
    }
  *sse = q;
  *sum = s;
}

unsigned int orc_variance(const uint8_t *a, int as, const uint8_t *b, int bs,
                          int w, int h, unsigned int *sse) {
  int sum;
  var_sums(a, as, b, bs, w, h, sse, &sum);
  return *sse - (uint32_t)(((int64_t)sum * sum) / (w * h));
}

unsigned int orc_mse(const uint8_t *a, int as, const uint8_t *b, int bs, int w,
                     int h, unsigned int *sse) {
  int sum;
  var_sums(a, as, b, bs, w, h, sse, &sum);
  return *sse;
}

static const uint8_t kBil[8][2] = { { 128, 0 }, { 112, 16 }, { 96, 32 },
                                    { 80, 48 }, { 64, 64 },  { 48, 80 },
                                    { 32, 96 }, { 16, 112 } };

unsigned int orc_sub_pixel_variance(const uint8_t *a, int as, int xo, int yo,
                                    const uint8_t *b, int bs, int w, int h,
                                    unsigned int *sse) {
  uint16_t *f = (uint16_t *)malloc(sizeof(uint16_t) * (h + 1) * w);
  uint8_t *t = (uint8_t *)malloc((size_t)h * w);
  for (int i = 0; i < h + 1; ++i)
    for (int j = 0; j < w; ++j) {
      const int v = a[i * as + j] * kBil[xo][0] + a[i * as + j + 1] * kBil[xo][1];
      f[i * w + j] = (uint16_t)((v + 64) >> 7);
    }
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) {
      const int v = f[i * w + j] * kBil[yo][0] + f[(i + 1) * w + j] * kBil[yo][1];
      t[i * w + j] = (uint8_t)((v + 64) >> 7);
    }
  const unsigned int r = orc_variance(t, w, b, bs, w, h, sse);
  free(f);
  free(t);
  return r;
}

/* aom_sub_pixel_avg_variance{W}x{H}_c (variance.c:132-145 + comp avg
 * aom_comp_avg_pred_c :285-298): filter as above, average with second_pred
 * (w x h, stride w), then variance against b. */
unsigned int orc_sub_pixel_avg_variance(const uint8_t *a, int as, int xo,
                                        int yo, const uint8_t *b, int bs,
                                        int w, int h, unsigned int *sse,
                                        const uint8_t *second_pred) {
  uint16_t *f = (uint16_t *)malloc(sizeof(uint16_t) * (h + 1) * w);
  uint8_t *t = (uint8_t *)malloc((size_t)h * w);
  for (int i = 0; i < h + 1; ++i)
    for (int j = 0; j < w; ++j) {
      const int v = a[i * as + j] * kBil[xo][0] + a[i * as + j + 1] * kBil[xo][1];
      f[i * w + j] = (uint16_t)((v + 64) >> 7);
    }
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) {
      const int v = f[i * w + j] * kBil[yo][0] + f[(i + 1) * w + j] * kBil[yo][1];
      const uint8_t p = (uint8_t)((v + 64) >> 7);
      t[i * w + j] = (uint8_t)((second_pred[i * w + j] + p + 1) >> 1);
    }
  const unsigned int r = orc_variance(t, w, b, bs, w, h, sse);
  free(f);
  free(t);
  return r;
}

unsigned int orc_highbd_variance(const uint16_t *a, int as, const uint16_t *b,
                                 int bs, int w, int h, int bd,
                                 unsigned int *sse) {
  int64_t tsum = 0;
  uint64_t tsse = 0;
  for (int i = 0; i < h; ++i, a += as, b += bs) {
    int32_t lsum = 0;
    for (int j = 0; j < w; ++j) {
      const int d = a[j] - b[j];
      lsum += d;
      tsse += (uint32_t)(d * d);
    }
    tsum += lsum;
  }
  int sum;
  if (bd == 8) {
    *sse = (uint32_t)tsse;
    sum = (int)tsum;
    return *sse - (uint32_t)(((int64_t)sum * sum) / (w * h));
  }
  const int ss = bd == 10 ? 4 : 8, sm = bd == 10 ? 2 : 4;
  *sse = (uint32_t)((tsse + ((1ull << ss) >> 1)) >> ss);
  sum = (int)((tsum + ((1ll << sm) >> 1)) >> sm);
  const int64_t var = (int64_t)(*sse) - (((int64_t)sum * sum) / (w * h));
  return var >= 0 ? (uint32_t)var : 0;
}

int64_t orc_sse(const uint8_t *a, int as, const uint8_t *b, int bs, int w,
                int h) {
  int64_t s = 0;
  for (int y = 0; y < h; ++y, a += as, b += bs)
    for (int x = 0; x < w; ++x) {
      const int32_t d = abs(a[x] - b[x]);
      s += d * d;
    }
  return s;
}

int64_t orc_highbd_sse(const uint16_t *a, int as, const uint16_t *b, int bs,
                       int w, int h) {
  int64_t s = 0;
  for (int y = 0; y < h; ++y, a += as, b += bs)
    for (int x = 0; x < w; ++x) {
      const int32_t d = (int32_t)a[x] - (int32_t)b[x];
      s += d * d;
    }
  return s;
}

void orc_subtract_block(int rows, int cols, int16_t *diff, ptrdiff_t ds,
                        const uint8_t *src, ptrdiff_t ss, const uint8_t *pred,
                        ptrdiff_t ps) {
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c)
      diff[r * ds + c] = (int16_t)(src[r * ss + c] - pred[r * ps + c]);
}

void orc_highbd_subtract_block(int rows, int cols, int16_t *diff,
                               ptrdiff_t ds, const uint16_t *src,
                               ptrdiff_t ss, const uint16_t *pred,
                               ptrdiff_t ps) {
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c)
      diff[r * ds + c] = (int16_t)(src[r * ss + c] - pred[r * ps + c]);
}

uint64_t orc_sum_squares_2d_i16(const int16_t *src, int stride, int w, int h) {
  uint64_t ss = 0;
  for (int r = 0; r < h; ++r)
    for (int c = 0; c < w; ++c) {
      const int16_t v = src[r * stride + c];
      ss += (uint64_t)(int64_t)(v * v);
    }
  return ss;
}

/* ---- Hadamard (int16 intermediates as in the reference) ---- */
static void had_col4(const int16_t *s, ptrdiff_t st, int16_t *o) {
  const int16_t b0 = (int16_t)((s[0] + s[st]) >> 1);
  const int16_t b1 = (int16_t)((s[0] - s[st]) >> 1);
  const int16_t b2 = (int16_t)((s[2 * st] + s[3 * st]) >> 1);
  const int16_t b3 = (int16_t)((s[2 * st] - s[3 * st]) >> 1);
  o[0] = (int16_t)(b0 + b2);
  o[1] = (int16_t)(b1 + b3);
  o[2] = (int16_t)(b0 - b2);
  o[3] = (int16_t)(b1 - b3);
}

static void had_col8(const int16_t *s, ptrdiff_t st, int16_t *o) {
  int16_t b[8], c[8];
  for (int k = 0; k < 4; ++k) {
    b[2 * k] = (int16_t)(s[2 * k * st] + s[(2 * k + 1) * st]);
    b[2 * k + 1] = (int16_t)(s[2 * k * st] - s[(2 * k + 1) * st]);
  }
  c[0] = (int16_t)(b[0] + b[2]);
  c[1] = (int16_t)(b[1] + b[3]);
  c[2] = (int16_t)(b[0] - b[2]);
  c[3] = (int16_t)(b[1] - b[3]);
  c[4] = (int16_t)(b[4] + b[6]);
  c[5] = (int16_t)(b[5] + b[7]);
  c[6] = (int16_t)(b[4] - b[6]);
  c[7] = (int16_t)(b[5] - b[7]);
  /* output order of avg.c:170-177 */
  o[0] = (int16_t)(c[0] + c[4]);
  o[7] = (int16_t)(c[1] + c[5]);
  o[3] = (int16_t)(c[2] + c[6]);
  o[4] = (int16_t)(c[3] + c[7]);
  o[2] = (int16_t)(c[0] - c[4]);
  o[6] = (int16_t)(c[1] - c[5]);
  o[1] = (int16_t)(c[2] - c[6]);
  o[5] = (int16_t)(c[3] - c[7]);
}

static void had_small(int n, const int16_t *src, ptrdiff_t st, int32_t *coeff) {
  int16_t b1[64], b2[64];
  for (int i = 0; i < n; ++i) {
    if (n == 4)
      had_col4(src + i, st, b1 + 4 * i);
    else
      had_col8(src + i, st, b1 + 8 * i);
  }
  for (int i = 0; i < n; ++i) {
    if (n == 4)
      had_col4(b1 + i, 4, b2 + 4 * i);
    else
      had_col8(b1 + i, 8, b2 + 8 * i);
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) coeff[i * n + j] = b2[j * n + i];
}

static void had16(const int16_t *src, ptrdiff_t st, int32_t *coeff) {
  for (int idx = 0; idx < 4; ++idx)
    had_small(8, src + (idx >> 1) * 8 * st + (idx & 1) * 8, st,
              coeff + idx * 64);
  for (int i = 0; i < 64; ++i) {
    const int32_t a0 = coeff[i], a1 = coeff[64 + i], a2 = coeff[128 + i],
                  a3 = coeff[192 + i];
    const int32_t b0 = (a0 + a1) >> 1, b1 = (a0 - a1) >> 1;
    const int32_t b2 = (a2 + a3) >> 1, b3 = (a2 - a3) >> 1;
    coeff[i] = b0 + b2;
    coeff[64 + i] = b1 + b3;
    coeff[128 + i] = b0 - b2;
    coeff[192 + i] = b1 - b3;
  }
  /* swap of 4-wide groups to match the AVX2 order (avg.c:281-287) */
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 4; ++j) {
      const int32_t t = coeff[i * 16 + 4 + j];
      coeff[i * 16 + 4 + j] = coeff[i * 16 + 8 + j];
      coeff[i * 16 + 8 + j] = t;
    }
}

void orc_hadamard(int n, const int16_t *src, ptrdiff_t st, int32_t *coeff) {
  if (n == 4 || n == 8) {
    had_small(n, src, st, coeff);
  } else if (n == 16) {
    had16(src, st, coeff);
  } else {
    for (int idx = 0; idx < 4; ++idx)
      had16(src + (idx >> 1) * 16 * st + (idx & 1) * 16, st, coeff + idx * 256);
    for (int i = 0; i < 256; ++i) {
      const int32_t a0 = coeff[i], a1 = coeff[256 + i], a2 = coeff[512 + i],
                    a3 = coeff[768 + i];
      const int32_t b0 = (a0 + a1) >> 2, b1 = (a0 - a1) >> 2;
      const int32_t b2 = (a2 + a3) >> 2, b3 = (a2 - a3) >> 2;
      coeff[i] = b0 + b2;
      coeff[256 + i] = b1 + b3;
      coeff[512 + i] = b0 - b2;
      coeff[768 + i] = b1 - b3;
    }
  }
}

int orc_satd(const int32_t *coeff, int length) {
  int s = 0;
  for (int i = 0; i < length; ++i) s += abs(coeff[i]);
  return s;
}

int64_t orc_block_error(const int32_t *coeff, const int32_t *dqcoeff,
                        intptr_t n, int64_t *ssz) {
  int64_t err = 0, sq = 0;
  for (intptr_t i = 0; i < n; ++i) {
    const int d = coeff[i] - dqcoeff[i];
    err += (int32_t)((uint32_t)d * (uint32_t)d);
    sq += (int32_t)((uint32_t)coeff[i] * (uint32_t)coeff[i]);
  }
  *ssz = sq;
  return err;
}

int64_t orc_highbd_block_error(const int32_t *coeff, const int32_t *dqcoeff,
                               intptr_t n, int64_t *ssz, int bd) {
  int64_t err = 0, sq = 0;
  const int shift = 2 * (bd - 8);
  const int rnd = shift > 0 ? 1 << (shift - 1) : 0;
  for (intptr_t i = 0; i < n; ++i) {
    const int64_t d = coeff[i] - dqcoeff[i];
    err += d * d;
    sq += (int64_t)coeff[i] * coeff[i];
  }
  *ssz = (sq + rnd) >> shift;
  return (err + rnd) >> shift;
}

/* aom_highbd_{8,10,12}_sub_pixel_variance / _avg_variance (variance.c:454-670):
 * u16 first pass (H+1 rows), u16 second pass, optional comp avg with
 * second_pred (nullable), then the bd variance against b. */
unsigned int orc_highbd_sub_pixel_variance(const uint16_t *a, int as, int xo,
                                           int yo, const uint16_t *b, int bs,
                                           int w, int h, int bd,
                                           unsigned int *sse,
                                           const uint16_t *second_pred) {
  uint16_t *f = (uint16_t *)malloc(sizeof(uint16_t) * (h + 1) * w);
  uint16_t *t = (uint16_t *)malloc(sizeof(uint16_t) * h * w);
  for (int i = 0; i < h + 1; ++i)
    for (int j = 0; j < w; ++j) {
      const int v = a[i * as + j] * kBil[xo][0] + a[i * as + j + 1] * kBil[xo][1];
      f[i * w + j] = (uint16_t)((v + 64) >> 7);
    }
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) {
      const int v = f[i * w + j] * kBil[yo][0] + f[(i + 1) * w + j] * kBil[yo][1];
      uint16_t p = (uint16_t)((v + 64) >> 7);
      if (second_pred) p = (uint16_t)((second_pred[i * w + j] + p + 1) >> 1);
      t[i * w + j] = p;
    }
  const unsigned int r = orc_highbd_variance(t, w, b, bs, w, h, bd, sse);
  free(f);
  free(t);
  return r;
}

/* aom_highbd_sad{W}x{H}_avg_c (sad.c:289-296, aom_highbd_comp_avg_pred) */
unsigned int orc_highbd_sad_avg(const uint16_t *src, int ss, const uint16_t *ref,
                                int rs, int w, int h,
                                const uint16_t *second_pred) {
  unsigned int s = 0;
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) {
      const int c = (second_pred[i * w + j] + ref[i * rs + j] + 1) >> 1;
      s += (unsigned)abs(src[i * ss + j] - c);
    }
  return s;
}

/* aom_highbd_hadamard_{8x8,16x16,32x32}_c (avg.c:350-507): int16 first
 * pass, int32 second pass, no output transpose and no 16x16 group swap. */
static void hbd_had8(const int16_t *src, ptrdiff_t st, int32_t *coeff) {
  int16_t b1[64];
  for (int i = 0; i < 8; ++i) had_col8(src + i, st, b1 + 8 * i);
  for (int i = 0; i < 8; ++i) {
    const int16_t *s = b1 + i;
    int32_t b[8], c[8];
    for (int k = 0; k < 4; ++k) {
      b[2 * k] = s[2 * k * 8] + s[(2 * k + 1) * 8];
      b[2 * k + 1] = s[2 * k * 8] - s[(2 * k + 1) * 8];
    }
    c[0] = b[0] + b[2];
    c[1] = b[1] + b[3];
    c[2] = b[0] - b[2];
    c[3] = b[1] - b[3];
    c[4] = b[4] + b[6];
    c[5] = b[5] + b[7];
    c[6] = b[4] - b[6];
    c[7] = b[5] - b[7];
    int32_t *o = coeff + 8 * i;
    o[0] = c[0] + c[4];
    o[7] = c[1] + c[5];
    o[3] = c[2] + c[6];
    o[4] = c[3] + c[7];
    o[2] = c[0] - c[4];
    o[6] = c[1] - c[5];
    o[1] = c[2] - c[6];
    o[5] = c[3] - c[7];
  }
}

static void hbd_had16(const int16_t *src, ptrdiff_t st, int32_t *coeff) {
  for (int idx = 0; idx < 4; ++idx)
    hbd_had8(src + (idx >> 1) * 8 * st + (idx & 1) * 8, st, coeff + idx * 64);
  for (int i = 0; i < 64; ++i) {
    const int32_t a0 = coeff[i], a1 = coeff[64 + i], a2 = coeff[128 + i],
                  a3 = coeff[192 + i];
    const int32_t b0 = (a0 + a1) >> 1, b1 = (a0 - a1) >> 1;
    const int32_t b2 = (a2 + a3) >> 1, b3 = (a2 - a3) >> 1;
    coeff[i] = b0 + b2;
    coeff[64 + i] = b1 + b3;
    coeff[128 + i] = b0 - b2;
    coeff[192 + i] = b1 - b3;
  }
}

void orc_highbd_hadamard(int n, const int16_t *src, ptrdiff_t st,
                         int32_t *coeff) {
  if (n == 8) {
    hbd_had8(src, st, coeff);
  } else if (n == 16) {
    hbd_had16(src, st, coeff);
  } else {
    for (int idx = 0; idx < 4; ++idx)
      hbd_had16(src + (idx >> 1) * 16 * st + (idx & 1) * 16, st,
                coeff + idx * 256);
    for (int i = 0; i < 256; ++i) {
      const int32_t a0 = coeff[i], a1 = coeff[256 + i], a2 = coeff[512 + i],
                    a3 = coeff[768 + i];
      const int32_t b0 = (a0 + a1) >> 2, b1 = (a0 - a1) >> 2;
      const int32_t b2 = (a2 + a3) >> 2, b3 = (a2 - a3) >> 2;
      coeff[i] = b0 + b2;
      coeff[256 + i] = b1 + b3;
      coeff[512 + i] = b0 - b2;
      coeff[768 + i] = b1 - b3;
    }
  }
}
