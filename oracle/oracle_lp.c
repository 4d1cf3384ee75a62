/* oracle_lp.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatements of the int16 ("low precision") Hadamard / SATD / block
 * error forms, the (sum, sse) helpers and the lossless 4x4 Walsh-Hadamard
 * transforms (the forward one, av1_fwht4x4, is orc_fwht4x4 in oracle_txfm.c):
 *   aom_hadamard_lp_8x8_c            aom_dsp/avg.c:207-236
 *   aom_hadamard_lp_16x16_c          aom_dsp/avg.c:289-316
 *   aom_satd_lp_c                    aom_dsp/avg.c:518-524
 *   av1_block_error_lp_c             av1/encoder/rdopt.c:650-660
 *   aom_sum_sse_2d_i16_c             aom_dsp/sum_squares.c:75-90
 *   aom_get_blk_sse_sum_c            aom_dsp/blk_sse_sum.c:14-27
 *   av1_highbd_iwht4x4_16_add_c / _1 av1/common/av1_inv_txfm2d.c:20-107,
 *                                    dispatch av1/common/idct.c:34-40
 * Pinned by tests/golden/fix_pixel.npz (the reference's own bodies executed).
 */
#include <stdlib.h>

#include "oracle.h"

/* 8x8 lp = the lowbd 8x8 butterflies + transpose (orc_hadamard), as int16 */
void orc_hadamard_lp(int n, const int16_t *src, ptrdiff_t st, int16_t *coeff) {
  int32_t c[256];
  if (n == 8) {
    orc_hadamard(8, src, st, c);
    for (int i = 0; i < 64; ++i) coeff[i] = (int16_t)c[i];
    return;
  }
  /* 16x16: four lp 8x8 blocks, then the int16 combine -- no AVX2 swap */
  for (int idx = 0; idx < 4; ++idx)
    orc_hadamard_lp(8, src + (idx >> 1) * 8 * st + (idx & 1) * 8, st, coeff + idx * 64);
  for (int i = 0; i < 64; ++i) {
    const int16_t a0 = coeff[i], a1 = coeff[64 + i], a2 = coeff[128 + i], a3 = coeff[192 + i];
    const int16_t b0 = (int16_t)((a0 + a1) >> 1), b1 = (int16_t)((a0 - a1) >> 1);
    const int16_t b2 = (int16_t)((a2 + a3) >> 1), b3 = (int16_t)((a2 - a3) >> 1);
    coeff[i] = (int16_t)(b0 + b2);
    coeff[64 + i] = (int16_t)(b1 + b3);
    coeff[128 + i] = (int16_t)(b0 - b2);
    coeff[192 + i] = (int16_t)(b1 - b3);
  }
}

int orc_satd_lp(const int16_t *coeff, int length) {
  int s = 0;
  for (int i = 0; i < length; ++i) s += abs(coeff[i]);
  return s;
}

int64_t orc_block_error_lp(const int16_t *coeff, const int16_t *dqcoeff, intptr_t n) {
  int64_t err = 0;
  for (intptr_t i = 0; i < n; ++i) {
    const int d = coeff[i] - dqcoeff[i];
    err += (int32_t)((uint32_t)d * (uint32_t)d); /* int * int */
  }
  return err;
}

/* (sum, sse) of an int16 block; aom_sum_sse_2d_i16 adds the sum into *sum */
void orc_sum_sse(const int16_t *src, int stride, int w, int h, int *sum, int64_t *sse) {
  int s = 0;
  int64_t ss = 0;
  for (int r = 0; r < h; ++r)
    for (int c = 0; c < w; ++c) {
      const int v = src[r * stride + c];
      ss += v * v;
      s += v;
    }
  *sum = s;
  *sse = ss;
}

static uint16_t clip_add(uint16_t p, int32_t v, int bd) {
  const int x = (int)p + v, mx = (1 << bd) - 1;
  return (uint16_t)(x < 0 ? 0 : (x > mx ? mx : x));
}

void orc_iwht4x4_add(const int32_t *in, uint16_t *dst, int stride, int eob, int bd) {
  if (eob > 1) {
    int32_t o[16];
    for (int i = 0; i < 4; ++i) {
      int32_t a1 = in[i] >> 2, c1 = in[4 + i] >> 2, d1 = in[8 + i] >> 2, b1 = in[12 + i] >> 2;
      a1 += c1;
      d1 -= b1;
      const int32_t e1 = (a1 - d1) >> 1;
      b1 = e1 - b1;
      c1 = e1 - c1;
      a1 -= b1;
      d1 += c1;
      o[i] = a1;
      o[4 + i] = b1;
      o[8 + i] = c1;
      o[12 + i] = d1;
    }
    for (int i = 0; i < 4; ++i) {
      int32_t a1 = o[4 * i], c1 = o[4 * i + 1], d1 = o[4 * i + 2], b1 = o[4 * i + 3];
      a1 += c1;
      d1 -= b1;
      const int32_t e1 = (a1 - d1) >> 1;
      b1 = e1 - b1;
      c1 = e1 - c1;
      a1 -= b1;
      d1 += c1;
      dst[0 * stride + i] = clip_add(dst[0 * stride + i], a1, bd);
      dst[1 * stride + i] = clip_add(dst[1 * stride + i], b1, bd);
      dst[2 * stride + i] = clip_add(dst[2 * stride + i], c1, bd);
      dst[3 * stride + i] = clip_add(dst[3 * stride + i], d1, bd);
    }
  } else {
    int32_t a1 = in[0] >> 2;
    int32_t e1 = a1 >> 1;
    a1 -= e1;
    const int32_t t[4] = {a1, e1, e1, e1};
    for (int i = 0; i < 4; ++i) {
      const int32_t e = t[i] >> 1, a = t[i] - e;
      dst[0 * stride + i] = clip_add(dst[0 * stride + i], a, bd);
      dst[1 * stride + i] = clip_add(dst[1 * stride + i], e, bd);
      dst[2 * stride + i] = clip_add(dst[2 * stride + i], e, bd);
      dst[3 * stride + i] = clip_add(dst[3 * stride + i], e, bd);
    }
  }
}
