/* oracle_compound.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the compound (CONV_BUF) convolutions of
 * av1/common/convolve.c, lowbd and highbd in one routine:
 *   path 0 av1_dist_wtd_convolve_2d_copy_c (:453-489) / highbd (:955-988)
 *   path 1 av1_dist_wtd_convolve_x_c (:406-451) / highbd (:859-905)
 *   path 2 av1_dist_wtd_convolve_y_c (:359-404) / highbd (:907-953)
 *   path 3 av1_dist_wtd_convolve_2d_c (:291-357) / highbd (:790-857)
 * (the selection of convolve_2d_facade_compound, :590-612, is path =
 * (subpel_x != 0) + 2 (subpel_y != 0)).  Every form produces the offset
 * CONV_BUF value res; do_average 0 stores it, do_average 1 averages it with
 * the buffer (plain or distance-weighted, DIST_PRECISION_BITS 4), removes
 * the offset, rounds and clips into dst.  fx / fy: the subpel kernel rows
 * (tx / ty taps), src at the block's integer position.
 */
#include <stdint.h>

#include "oracle.h"

#define FB 7 /* FILTER_BITS */

static int pget(const void *p, long i, int hbd) {
  return hbd ? ((const uint16_t *)p)[i] : ((const uint8_t *)p)[i];
}
static int rpot(int v, int n) { return (v + ((1 << n) >> 1)) >> n; }

void orc_dist_wtd_convolve(int path, const void *src, int src_stride, void *dst, int dst_stride,
                           int w, int h, const int16_t *fx, int tx, const int16_t *fy, int ty,
                           const OrcConvParams *cp, uint16_t *conv, int conv_stride, int bd,
                           int hbd) {
  const int r0 = cp->round_0, r1 = cp->round_1;
  const int offset_bits = bd + 2 * FB - r0;
  const int round_offset = (1 << (offset_bits - r1)) + (1 << (offset_bits - r1 - 1));
  const int round_bits = 2 * FB - r0 - r1;
  const int fo_x = tx / 2 - 1, fo_y = ty / 2 - 1;
  const int pmax = (1 << bd) - 1;
  /* path 3: the (h + ty - 1) x w horizontally filtered rows first (int16,
   * as im_block) */
  int16_t im[(128 + 11) * 128];
  if (path == 3)
    for (int y = 0; y < h + ty - 1; ++y) {
      const long row = (long)(y - fo_y) * src_stride;
      for (int x = 0; x < w; ++x) {
        int32_t hs = 1 << (bd + FB - 1);
        for (int m = 0; m < tx; ++m) hs += fx[m] * pget(src, row + x - fo_x + m, hbd);
        im[y * w + x] = (int16_t)rpot(hs, r0);
      }
    }
  for (int y = 0; y < h; ++y) {
    for (int x = 0; x < w; ++x) {
      int32_t res;
      if (path == 0) {
        res = (uint16_t)((pget(src, (long)y * src_stride + x, hbd) << round_bits) + round_offset);
      } else if (path == 1) {
        int32_t s = 0;
        for (int k = 0; k < tx; ++k) s += fx[k] * pget(src, (long)y * src_stride + x - fo_x + k, hbd);
        res = (1 << (FB - r1)) * rpot(s, r0) + round_offset;
      } else if (path == 2) {
        int32_t s = 0;
        for (int k = 0; k < ty; ++k)
          s += fy[k] * pget(src, (long)(y - fo_y + k) * src_stride + x, hbd);
        res = rpot(s * (1 << (FB - r0)), r1) + round_offset;
      } else {
        /* the intermediate rows y .. y + ty - 1 (source rows y - fo_y ..) */
        int32_t s = 1 << offset_bits;
        for (int k = 0; k < ty; ++k) s += fy[k] * im[(y + k) * w + x];
        res = (uint16_t)rpot(s, r1);
      }
      uint16_t *c = conv + (long)y * conv_stride + x;
      if (!cp->do_average) {
        *c = (uint16_t)res;
        continue;
      }
      int32_t t = *c;
      t = cp->use_dist_wtd_comp_avg ? (t * cp->fwd_offset + res * cp->bck_offset) >> 4
                                    : (t + res) >> 1;
      t -= round_offset;
      int v = rpot(t, round_bits);
      v = v < 0 ? 0 : (v > pmax ? pmax : v);
      if (hbd) ((uint16_t *)dst)[(long)y * dst_stride + x] = (uint16_t)v;
      else ((uint8_t *)dst)[(long)y * dst_stride + x] = (uint8_t)v;
    }
  }
}

/* Batch driver for the `compound` bench workload's CPU baseline: jobs in the
 * LavishCompoundJob layout, the x / y kernel tables [16][taps] shared, the
 * path per job from its sub-pel phases, over pthreads. */
#include <pthread.h>

typedef struct {
  int64_t src_off, dst_off, conv_off;
  int32_t sx, sy;
} CompJob;

typedef struct {
  const void *src;
  void *dst;
  uint16_t *conv;
  const CompJob *jobs;
  const int16_t *fx, *fy;
  const OrcConvParams *cp;
  int src_stride, dst_stride, conv_stride, w, h, tx, ty, bd, hbd;
  long lo, hi;
} CompArg;

static void *comp_worker(void *p) {
  const CompArg *a = (const CompArg *)p;
  const int es = a->hbd ? 2 : 1;
  for (long j = a->lo; j < a->hi; ++j) {
    const CompJob *jb = &a->jobs[j];
    const int sx = jb->sx & 15, sy = jb->sy & 15;
    orc_dist_wtd_convolve((sx != 0) + 2 * (sy != 0), (const char *)a->src + jb->src_off * es,
                          a->src_stride, (char *)a->dst + jb->dst_off * es, a->dst_stride, a->w,
                          a->h, a->fx + sx * a->tx, a->tx, a->fy + sy * a->ty, a->ty, a->cp,
                          a->conv + jb->conv_off, a->conv_stride, a->bd, a->hbd);
  }
  return NULL;
}

void orc_dist_wtd_batch(const void *src, int src_stride, void *dst, int dst_stride,
                        uint16_t *conv, int conv_stride, int w, int h, const void *jobs,
                        long njobs, const int16_t *fx, int tx, const int16_t *fy, int ty,
                        const OrcConvParams *cp, int bd, int hbd, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  CompArg args[256];
  for (int t = 0; t < threads; ++t) {
    CompArg *a = &args[t];
    a->src = src;
    a->dst = dst;
    a->conv = conv;
    a->jobs = (const CompJob *)jobs;
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
    if (threads > 1) pthread_create(&tid[t], NULL, comp_worker, a);
    else comp_worker(a);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}
