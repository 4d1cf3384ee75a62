/* oracle_scale.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the scaled convolution of the reference:
 *   av1_convolve_2d_scale_c         av1/common/convolve.c:488-574
 *   av1_highbd_convolve_2d_scale_c  av1/common/convolve.c:992-1078
 * (the inter predictor of a scaled reference: convolve_2d_scale_wrapper,
 * :576-588).  Positions step in 1/1024 pel (SCALE_SUBPEL_BITS 10); the
 * kernel phase of a position is its top 4 sub-pel bits (SCALE_EXTRA_BITS 6).
 * fx / fy: the 16 kernel rows of the InterpFilterParams (taps each), as
 * av1_get_interp_filter_subpel_kernel reads them.  Pinned by
 * tests/golden/fix_scale.npz (both functions executed from the reference).
 */
#include <stdlib.h>

#include "oracle.h"

#define SCALE_BITS 10
#define SCALE_MASK ((1 << SCALE_BITS) - 1)
#define SCALE_EXTRA 6
#define FBITS 7
#define RPOT(v, n) (((v) + ((1 << (n)) >> 1)) >> (n))

static inline int px_get(const void *p, ptrdiff_t i, int hbd) {
  return hbd ? ((const uint16_t *)p)[i] : ((const uint8_t *)p)[i];
}
static inline void px_put(void *p, ptrdiff_t i, int v, int hbd) {
  if (hbd) ((uint16_t *)p)[i] = (uint16_t)v;
  else ((uint8_t *)p)[i] = (uint8_t)v;
}
static inline int clip_bd(int v, int bd) {
  const int mx = (1 << bd) - 1;
  return v < 0 ? 0 : v > mx ? mx : v;
}

/* One w x h block; src at its integer position.  hbd 0: the lowbd
 * function (its bd is 8); the compound forms read / write conv (CONV_BUF). */
void orc_convolve_2d_scale(const void *src, int src_stride, void *dst, int dst_stride, int w,
                           int h, const int16_t *fx, int tx, const int16_t *fy, int ty,
                           int subpel_x_qn, int x_step_qn, int subpel_y_qn, int y_step_qn,
                           const OrcConvParams *cp, uint16_t *conv, int conv_stride, int bd,
                           int hbd) {
  if (!hbd) bd = 8;
  const int im_h = (((h - 1) * y_step_qn + subpel_y_qn) >> SCALE_BITS) + ty;
  int16_t *im = (int16_t *)malloc(sizeof(int16_t) * (size_t)im_h * w);
  const int fo_vert = ty / 2 - 1, fo_horiz = tx / 2 - 1;
  const int bits = 2 * FBITS - cp->round_0 - cp->round_1;
  /* horizontal filter: im_h rows from fo_vert above the block */
  for (int y = 0; y < im_h; ++y) {
    const ptrdiff_t row = (ptrdiff_t)(y - fo_vert) * src_stride;
    int x_qn = subpel_x_qn;
    for (int x = 0; x < w; ++x, x_qn += x_step_qn) {
      const ptrdiff_t sx = row + (x_qn >> SCALE_BITS);
      const int16_t *f = fx + tx * ((x_qn & SCALE_MASK) >> SCALE_EXTRA);
      int32_t sum = 1 << (bd + FBITS - 1);
      for (int k = 0; k < tx; ++k) sum += f[k] * px_get(src, sx + k - fo_horiz, hbd);
      im[y * w + x] = (int16_t)RPOT(sum, cp->round_0);
    }
  }
  /* vertical filter */
  const int offset_bits = bd + 2 * FBITS - cp->round_0;
  const int round_offset =
      (1 << (offset_bits - cp->round_1)) + (1 << (offset_bits - cp->round_1 - 1));
  for (int x = 0; x < w; ++x) {
    int y_qn = subpel_y_qn;
    for (int y = 0; y < h; ++y, y_qn += y_step_qn) {
      const int r0 = y_qn >> SCALE_BITS; /* src_vert = im + fo_vert rows */
      const int16_t *f = fy + ty * ((y_qn & SCALE_MASK) >> SCALE_EXTRA);
      int32_t sum = 1 << offset_bits;
      for (int k = 0; k < ty; ++k) sum += f[k] * im[(r0 + k) * w + x];
      const int32_t res = (uint16_t)RPOT(sum, cp->round_1); /* CONV_BUF_TYPE */
      if (cp->is_compound) {
        uint16_t *c = conv + (ptrdiff_t)y * conv_stride + x;
        if (cp->do_average) {
          int32_t tmp = *c;
          if (cp->use_dist_wtd_comp_avg)
            tmp = (tmp * cp->fwd_offset + res * cp->bck_offset) >> 4; /* DIST_PRECISION_BITS */
          else
            tmp = (tmp + res) >> 1;
          tmp -= round_offset;
          px_put(dst, (ptrdiff_t)y * dst_stride + x, clip_bd(RPOT(tmp, bits), bd), hbd);
        } else {
          *c = (uint16_t)res;
        }
      } else {
        const int32_t tmp = res - round_offset;
        px_put(dst, (ptrdiff_t)y * dst_stride + x, clip_bd(RPOT(tmp, bits), bd), hbd);
      }
    }
  }
  free(im);
}

/* Batch driver for the `scale` bench workload's CPU baseline: jobs in the
 * LavishScaleJob layout (one w x h block each), one conv form, over
 * pthreads. */
#include <pthread.h>

typedef struct {
  int64_t src_off, dst_off, conv_off;
  int32_t subpel_x_qn, x_step_qn, subpel_y_qn, y_step_qn;
} ScaleJob;

typedef struct {
  const void *src;
  void *dst;
  uint16_t *conv;
  const ScaleJob *jobs;
  const int16_t *fx, *fy;
  const OrcConvParams *cp;
  int src_stride, dst_stride, conv_stride, w, h, tx, ty, bd, hbd;
  long lo, hi;
} ScaleArg;

static void *scale_worker(void *p) {
  const ScaleArg *a = (const ScaleArg *)p;
  const int es = a->hbd ? 2 : 1;
  for (long j = a->lo; j < a->hi; ++j) {
    const ScaleJob *jb = &a->jobs[j];
    orc_convolve_2d_scale((const char *)a->src + jb->src_off * es, a->src_stride,
                          a->dst ? (char *)a->dst + jb->dst_off * es : NULL, a->dst_stride, a->w,
                          a->h, a->fx, a->tx, a->fy, a->ty, jb->subpel_x_qn, jb->x_step_qn,
                          jb->subpel_y_qn, jb->y_step_qn, a->cp,
                          a->conv ? a->conv + jb->conv_off : NULL, a->conv_stride, a->bd, a->hbd);
  }
  return NULL;
}

void orc_convolve_2d_scale_batch(const void *src, int src_stride, void *dst, int dst_stride,
                                 uint16_t *conv, int conv_stride, int w, int h, const void *jobs,
                                 long njobs, const int16_t *fx, int tx, const int16_t *fy, int ty,
                                 const OrcConvParams *cp, int bd, int hbd, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  ScaleArg args[256];
  for (int t = 0; t < threads; ++t) {
    ScaleArg *a = &args[t];
    a->src = src;
    a->dst = dst;
    a->conv = conv;
    a->jobs = (const ScaleJob *)jobs;
    a->fx = fx;
    a->fy = fy;
    a->cp = cp;
    a->src_stride = src_stride;
    a->dst_stride = dst_stride;
    a->conv_stride = conv_stride;
    a->w = w;
    a->h = h;
    a->tx = tx;
    a->ty = ty;
    a->bd = bd;
    a->hbd = hbd;
    a->lo = njobs * t / threads;
    a->hi = njobs * (t + 1) / threads;
    if (threads > 1) pthread_create(&tid[t], NULL, scale_worker, a);
    else scale_worker(a);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}
