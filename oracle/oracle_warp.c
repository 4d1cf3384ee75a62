/* oracle_warp.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the affine warp predictor of av1/common/warped_motion.c:
 *   av1_get_shear_params (:218-247) with resolve_divisor_32 (:187-201) and
 *   the shear validity test (:203-215);
 *   av1_warp_affine_c (:538-666) and av1_highbd_warp_affine_c (:264-388) in
 *   one routine over u8 / u16 samples: per 8x8 output block, the block
 *   centre projected through the matrix (luma coordinates when subsampled),
 *   15 horizontally filtered rows of 8 (per-pixel filter phase sx4 + alpha l
 *   + beta k, edge-clamped samples, offset 2^(bd+6), round by the horizontal
 *   reduce bits), then 8 vertical taps per output (phase sy4 + gamma l +
 *   delta k) and the single / compound (plain or distance-weighted average)
 *   write-out.  Filter taps and the divisor LUT: warp_tables.h (checked
 *   against the reference text by tests/test_capi_cpu.py).
 */
#include <stdint.h>
#include <stdlib.h>

#include "oracle.h"
#include "warp_tables.h"

#define WM_BITS 16     /* WARPEDMODEL_PREC_BITS (mv.h:96) */
#define WD_BITS 10     /* WARPEDDIFF_PREC_BITS = 16 - WARPEDPIXEL_PREC_BITS */
#define WP_SHIFTS 64   /* WARPEDPIXEL_PREC_SHIFTS */
#define WR_BITS 6      /* WARP_PARAM_REDUCE_BITS */
#define F_BITS 7       /* FILTER_BITS */

static int64_t rshift_signed64(int64_t v, int n) { /* ROUND_POWER_OF_TWO_SIGNED_64 */
  return v < 0 ? -((-v + (((int64_t)1 << n) >> 1)) >> n) : (v + (((int64_t)1 << n) >> 1)) >> n;
}
static int rshift_signed(int v, int n) { /* ROUND_POWER_OF_TWO_SIGNED */
  return v < 0 ? -((-v + ((1 << n) >> 1)) >> n) : (v + ((1 << n) >> 1)) >> n;
}
static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static int msb32(uint32_t v) {
  int n = 0;
  while (v >>= 1) ++n;
  return n;
}

int orc_get_shear_params(const int32_t mat[6], int16_t out[4]) {
  if (mat[2] <= 0) return 0;
  int alpha = clampi(mat[2] - (1 << WM_BITS), INT16_MIN, INT16_MAX);
  int beta = clampi(mat[3], INT16_MIN, INT16_MAX);
  /* 1 / mat[2] = y / 2^shift: 8 bits of the mantissa index the LUT */
  const uint32_t D = (uint32_t)abs(mat[2]);
  int shift = msb32(D);
  const int32_t e = (int32_t)(D - ((uint32_t)1 << shift));
  const int32_t f = shift > 8 ? (e + ((1 << (shift - 8)) >> 1)) >> (shift - 8) : e << (8 - shift);
  shift += 14; /* DIV_LUT_PREC_BITS */
  const int y = kDivLut[f] * (mat[2] < 0 ? -1 : 1);
  int64_t v = ((int64_t)mat[4] * (1 << WM_BITS)) * y;
  int gamma = clampi((int)rshift_signed64(v, shift), INT16_MIN, INT16_MAX);
  v = ((int64_t)mat[3] * mat[4]) * y;
  int delta = clampi(mat[5] - (int)rshift_signed64(v, shift) - (1 << WM_BITS), INT16_MIN,
                     INT16_MAX);
  alpha = rshift_signed(alpha, WR_BITS) * (1 << WR_BITS);
  beta = rshift_signed(beta, WR_BITS) * (1 << WR_BITS);
  gamma = rshift_signed(gamma, WR_BITS) * (1 << WR_BITS);
  delta = rshift_signed(delta, WR_BITS) * (1 << WR_BITS);
  out[0] = (int16_t)alpha;
  out[1] = (int16_t)beta;
  out[2] = (int16_t)gamma;
  out[3] = (int16_t)delta;
  if (4 * abs(alpha) + 7 * abs(beta) >= (1 << WM_BITS) ||
      4 * abs(gamma) + 4 * abs(delta) >= (1 << WM_BITS))
    return 0;
  return 1;
}

static int px(const void *p, long i, int hbd) {
  return hbd ? ((const uint16_t *)p)[i] : ((const uint8_t *)p)[i];
}

void orc_warp_affine(const int32_t mat[6], const void *ref, int width, int height, int stride,
                     void *pred, int p_col, int p_row, int p_width, int p_height, int p_stride,
                     int ss_x, int ss_y, int bd, int hbd, const OrcConvParams *cp,
                     uint16_t *conv_dst, int dst_stride, int alpha, int beta, int gamma,
                     int delta) {
  /* the lowbd function fixes reduce_bits_horiz = round_0 */
  const int rh = hbd ? cp->round_0 + (bd + F_BITS - cp->round_0 - 14 > 0
                                          ? bd + F_BITS - cp->round_0 - 14 : 0)
                     : cp->round_0;
  const int rv = cp->is_compound ? cp->round_1 : 2 * F_BITS - rh;
  const int off_h = bd + F_BITS - 1, off_v = bd + 2 * F_BITS - rh;
  const int round_bits = 2 * F_BITS - cp->round_0 - cp->round_1;
  const int off_bits = bd + 2 * F_BITS - cp->round_0;
  const int pmax = (1 << bd) - 1;
  int32_t t[15][8];
  for (int i = p_row; i < p_row + p_height; i += 8) {
    for (int j = p_col; j < p_col + p_width; j += 8) {
      const int64_t cx = (int64_t)((j + 4) << ss_x), cy = (int64_t)((i + 4) << ss_y);
      const int64_t x4 = (mat[2] * cx + mat[3] * cy + mat[0]) >> ss_x;
      const int64_t y4 = (mat[4] * cx + mat[5] * cy + mat[1]) >> ss_y;
      const int ix4 = (int)(x4 >> WM_BITS), iy4 = (int)(y4 >> WM_BITS);
      int sx4 = (int)(x4 & ((1 << WM_BITS) - 1)), sy4 = (int)(y4 & ((1 << WM_BITS) - 1));
      sx4 = (sx4 - 4 * alpha - 4 * beta) & ~((1 << WR_BITS) - 1);
      sy4 = (sy4 - 4 * gamma - 4 * delta) & ~((1 << WR_BITS) - 1);
      for (int r = 0; r < 15; ++r) { /* k = r - 7 */
        const long row = (long)clampi(iy4 + r - 7, 0, height - 1) * stride;
        for (int c = 0; c < 8; ++c) { /* l = c - 4 */
          const int sx = sx4 + beta * (r - 3) + alpha * c;
          const int16_t *f = kWarpedFilter[((sx + (1 << (WD_BITS - 1))) >> WD_BITS) + WP_SHIFTS];
          int32_t s = 1 << off_h;
          for (int m = 0; m < 8; ++m) s += px(ref, row + clampi(ix4 + c - 7 + m, 0, width - 1), hbd) * f[m];
          t[r][c] = (s + ((1 << rh) >> 1)) >> rh;
        }
      }
      const int rows = p_row + p_height - i < 8 ? p_row + p_height - i : 8;
      const int cols = p_col + p_width - j < 8 ? p_col + p_width - j : 8;
      for (int r = 0; r < rows; ++r) {   /* k = r - 4 */
        for (int c = 0; c < cols; ++c) { /* l = c - 4 */
          const int sy = sy4 + delta * r + gamma * c;
          const int16_t *f = kWarpedFilter[((sy + (1 << (WD_BITS - 1))) >> WD_BITS) + WP_SHIFTS];
          int32_t s = 1 << off_v;
          for (int m = 0; m < 8; ++m) s += t[r + m][c] * f[m];
          s = (s + ((1 << rv) >> 1)) >> rv;
          const long po = (long)(i - p_row + r) * p_stride + (j - p_col + c);
          int out;
          if (cp->is_compound) {
            uint16_t *d = conv_dst + (long)(i - p_row + r) * dst_stride + (j - p_col + c);
            if (!cp->do_average) {
              *d = (uint16_t)s;
              continue;
            }
            int32_t a = *d;
            a = cp->use_dist_wtd_comp_avg ? (a * cp->fwd_offset + s * cp->bck_offset) >> 4
                                          : (a + s) >> 1; /* DIST_PRECISION_BITS 4 */
            a -= (1 << (off_bits - cp->round_1)) + (1 << (off_bits - cp->round_1 - 1));
            out = (a + ((1 << round_bits) >> 1)) >> round_bits;
          } else {
            out = s - (1 << (bd - 1)) - (1 << bd);
          }
          out = clampi(out, 0, pmax);
          if (hbd) ((uint16_t *)pred)[po] = (uint16_t)out;
          else ((uint8_t *)pred)[po] = (uint8_t)out;
        }
      }
    }
  }
}

/* Batch driver for the `warp` bench workload's CPU baseline: jobs in the
 * LavishWarpJob layout (one block each), one conv form, over pthreads. */
#include <pthread.h>

typedef struct {
  int32_t mat[6];
  int16_t alpha, beta, gamma, delta;
  int32_t p_col, p_row, p_width, p_height;
  int64_t ref_off, pred_off, dst_off;
} WarpJob;

typedef struct {
  const void *ref;
  void *pred;
  uint16_t *dst;
  const WarpJob *jobs;
  const OrcConvParams *cp;
  int width, height, stride, p_stride, dst_stride, ss_x, ss_y, bd, hbd;
  long lo, hi;
} WarpArg;

static void *warp_worker(void *p) {
  const WarpArg *a = (const WarpArg *)p;
  const int es = a->hbd ? 2 : 1;
  for (long j = a->lo; j < a->hi; ++j) {
    const WarpJob *jb = &a->jobs[j];
    orc_warp_affine(jb->mat, (const char *)a->ref + jb->ref_off * es, a->width, a->height,
                    a->stride, (char *)a->pred + jb->pred_off * es, jb->p_col, jb->p_row,
                    jb->p_width, jb->p_height, a->p_stride, a->ss_x, a->ss_y, a->bd, a->hbd,
                    a->cp, a->dst ? a->dst + jb->dst_off : NULL, a->dst_stride, jb->alpha,
                    jb->beta, jb->gamma, jb->delta);
  }
  return NULL;
}

void orc_warp_batch(const void *ref, int width, int height, int stride, void *pred,
                    int p_stride, uint16_t *dst, int dst_stride, const void *jobs, long njobs,
                    int ss_x, int ss_y, int bd, int hbd, const OrcConvParams *cp, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  WarpArg args[256];
  for (int t = 0; t < threads; ++t) {
    WarpArg *a = &args[t];
    a->ref = ref;
    a->pred = pred;
    a->dst = dst;
    a->jobs = (const WarpJob *)jobs;
    a->cp = cp;
    a->width = width;
    a->height = height;
    a->stride = stride;
    a->p_stride = p_stride;
    a->dst_stride = dst_stride;
    a->ss_x = ss_x;
    a->ss_y = ss_y;
    a->bd = bd;
    a->hbd = hbd;
    a->lo = njobs * t / threads;
    a->hi = njobs * (t + 1) / threads;
    if (threads > 1) pthread_create(&tid[t], NULL, warp_worker, a);
    else warp_worker(a);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}
