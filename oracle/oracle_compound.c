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
        /* the intermediate rows y - fo_y .. y - fo_y + ty - 1 at column x */
        int32_t s = 1 << offset_bits;
        for (int k = 0; k < ty; ++k) {
          const long row = (long)(y - fo_y + k) * src_stride;
          int32_t hs = 1 << (bd + FB - 1);
          for (int m = 0; m < tx; ++m) hs += fx[m] * pget(src, row + x - fo_x + m, hbd);
          s += fy[k] * (int16_t)rpot(hs, r0);
        }
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
