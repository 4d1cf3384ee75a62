/* oracle_convolve.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of single-reference translational inter prediction
 * ("inter prediction"):
 *   av1_enc_build_one_inter_predictor   av1/encoder/reconinter_enc.c:31-51
 *     -> enc_calc_subpel_params / init_subpel_params
 *                                       av1/common/reconinter.h:131-165
 *        (unscaled: av1_unscaled_value, scale.h:54-57; clamp to the
 *         AOM_LEFT_TOP_MARGIN_SCALED / (size + AOM_INTERP_EXTEND) window)
 *     -> av1_get_interp_filter_params_with_block_size  filter.h:253-259
 *     -> inter_predictor / highbd_inter_predictor      reconinter.h:252-291
 *        (revert_scale_extra_bits :241-250)
 *     -> convolve_2d_facade_single / highbd_...        convolve.c:614-634,1106-1128
 *   av1_convolve_x_sr_c / _y_sr_c / _2d_sr_c           convolve.c:76-188
 *   av1_highbd_convolve_x_sr_c / _y_sr_c / _2d_sr_c    convolve.c:687-787
 *   aom_convolve_copy_c / aom_highbd_convolve_copy_c   aom_dsp/aom_convolve.c:156-180
 *   get_conv_params_no_round (single prediction)       convolve.h:63-95
 * The lowbd and highbd C functions differ only in the clip and the pixel
 * type (the lowbd 2-D filter runs with bd = 8), so one routine covers both.
 * Filter tables: filter.h:111-243; their values are pinned against the
 * reference's source by tests/golden (ref_tables.json "interp_filters").
 */
#include <string.h>

#include "oracle.h"

/* [kind][subpel][tap]: 0 REGULAR, 1 SMOOTH, 2 SHARP, 3 BILINEAR (8-tap
 * layouts), 4 REGULAR 4-tap, 5 SMOOTH 4-tap (used for sizes <= 4) */
static const int16_t kern8[6][16][8] = {
  { { 0, 0, 0, 128, 0, 0, 0, 0 }, { 0, 2, -6, 126, 8, -2, 0, 0 },
    { 0, 2, -10, 122, 18, -4, 0, 0 }, { 0, 2, -12, 116, 28, -8, 2, 0 },
    { 0, 2, -14, 110, 38, -10, 2, 0 }, { 0, 2, -14, 102, 48, -12, 2, 0 },
    { 0, 2, -16, 94, 58, -12, 2, 0 }, { 0, 2, -14, 84, 66, -12, 2, 0 },
    { 0, 2, -14, 76, 76, -14, 2, 0 }, { 0, 2, -12, 66, 84, -14, 2, 0 },
    { 0, 2, -12, 58, 94, -16, 2, 0 }, { 0, 2, -12, 48, 102, -14, 2, 0 },
    { 0, 2, -10, 38, 110, -14, 2, 0 }, { 0, 2, -8, 28, 116, -12, 2, 0 },
    { 0, 0, -4, 18, 122, -10, 2, 0 }, { 0, 0, -2, 8, 126, -6, 2, 0 } },
  { { 0, 0, 0, 128, 0, 0, 0, 0 }, { 0, 2, 28, 62, 34, 2, 0, 0 },
    { 0, 0, 26, 62, 36, 4, 0, 0 }, { 0, 0, 22, 62, 40, 4, 0, 0 },
    { 0, 0, 20, 60, 42, 6, 0, 0 }, { 0, 0, 18, 58, 44, 8, 0, 0 },
    { 0, 0, 16, 56, 46, 10, 0, 0 }, { 0, -2, 16, 54, 48, 12, 0, 0 },
    { 0, -2, 14, 52, 52, 14, -2, 0 }, { 0, 0, 12, 48, 54, 16, -2, 0 },
    { 0, 0, 10, 46, 56, 16, 0, 0 }, { 0, 0, 8, 44, 58, 18, 0, 0 },
    { 0, 0, 6, 42, 60, 20, 0, 0 }, { 0, 0, 4, 40, 62, 22, 0, 0 },
    { 0, 0, 4, 36, 62, 26, 0, 0 }, { 0, 0, 2, 34, 62, 28, 2, 0 } },
  { { 0, 0, 0, 128, 0, 0, 0, 0 }, { -2, 2, -6, 126, 8, -2, 2, 0 },
    { -2, 6, -12, 124, 16, -6, 4, -2 }, { -2, 8, -18, 120, 26, -10, 6, -2 },
    { -4, 10, -22, 116, 38, -14, 6, -2 }, { -4, 10, -22, 108, 48, -18, 8, -2 },
    { -4, 10, -24, 100, 60, -20, 8, -2 }, { -4, 10, -24, 90, 70, -22, 10, -2 },
    { -4, 12, -24, 80, 80, -24, 12, -4 }, { -2, 10, -22, 70, 90, -24, 10, -4 },
    { -2, 8, -20, 60, 100, -24, 10, -4 }, { -2, 8, -18, 48, 108, -22, 10, -4 },
    { -2, 6, -14, 38, 116, -22, 10, -4 }, { -2, 6, -10, 26, 120, -18, 8, -2 },
    { -2, 4, -6, 16, 124, -12, 6, -2 }, { 0, 2, -2, 8, 126, -6, 2, -2 } },
  { { 0, 0, 0, 128, 0, 0, 0, 0 }, { 0, 0, 0, 120, 8, 0, 0, 0 },
    { 0, 0, 0, 112, 16, 0, 0, 0 }, { 0, 0, 0, 104, 24, 0, 0, 0 },
    { 0, 0, 0, 96, 32, 0, 0, 0 }, { 0, 0, 0, 88, 40, 0, 0, 0 },
    { 0, 0, 0, 80, 48, 0, 0, 0 }, { 0, 0, 0, 72, 56, 0, 0, 0 },
    { 0, 0, 0, 64, 64, 0, 0, 0 }, { 0, 0, 0, 56, 72, 0, 0, 0 },
    { 0, 0, 0, 48, 80, 0, 0, 0 }, { 0, 0, 0, 40, 88, 0, 0, 0 },
    { 0, 0, 0, 32, 96, 0, 0, 0 }, { 0, 0, 0, 24, 104, 0, 0, 0 },
    { 0, 0, 0, 16, 112, 0, 0, 0 }, { 0, 0, 0, 8, 120, 0, 0, 0 } },
  { { 0, 0, 0, 128, 0, 0, 0, 0 }, { 0, 0, -4, 126, 8, -2, 0, 0 },
    { 0, 0, -8, 122, 18, -4, 0, 0 }, { 0, 0, -10, 116, 28, -6, 0, 0 },
    { 0, 0, -12, 110, 38, -8, 0, 0 }, { 0, 0, -12, 102, 48, -10, 0, 0 },
    { 0, 0, -14, 94, 58, -10, 0, 0 }, { 0, 0, -12, 84, 66, -10, 0, 0 },
    { 0, 0, -12, 76, 76, -12, 0, 0 }, { 0, 0, -10, 66, 84, -12, 0, 0 },
    { 0, 0, -10, 58, 94, -14, 0, 0 }, { 0, 0, -10, 48, 102, -12, 0, 0 },
    { 0, 0, -8, 38, 110, -12, 0, 0 }, { 0, 0, -6, 28, 116, -10, 0, 0 },
    { 0, 0, -4, 18, 122, -8, 0, 0 }, { 0, 0, -2, 8, 126, -4, 0, 0 } },
  { { 0, 0, 0, 128, 0, 0, 0, 0 }, { 0, 0, 30, 62, 34, 2, 0, 0 },
    { 0, 0, 26, 62, 36, 4, 0, 0 }, { 0, 0, 22, 62, 40, 4, 0, 0 },
    { 0, 0, 20, 60, 42, 6, 0, 0 }, { 0, 0, 18, 58, 44, 8, 0, 0 },
    { 0, 0, 16, 56, 46, 10, 0, 0 }, { 0, 0, 14, 54, 48, 12, 0, 0 },
    { 0, 0, 12, 52, 52, 12, 0, 0 }, { 0, 0, 12, 48, 54, 14, 0, 0 },
    { 0, 0, 10, 46, 56, 16, 0, 0 }, { 0, 0, 8, 44, 58, 18, 0, 0 },
    { 0, 0, 6, 42, 60, 20, 0, 0 }, { 0, 0, 4, 40, 62, 22, 0, 0 },
    { 0, 0, 4, 36, 62, 26, 0, 0 }, { 0, 0, 2, 34, 62, 30, 0, 0 } },
};

/* MULTITAP_SHARP2 (12 taps, encoder-only: temporal filtering) */
static const int16_t kern12[16][12] = {
  { 0, 0, 0, 0, 0, 128, 0, 0, 0, 0, 0, 0 },
  { 0, 1, -2, 3, -7, 127, 8, -4, 2, -1, 1, 0 },
  { -1, 2, -3, 6, -13, 124, 18, -8, 4, -2, 2, -1 },
  { -1, 3, -4, 8, -18, 120, 28, -12, 7, -4, 2, -1 },
  { -1, 3, -6, 10, -21, 115, 38, -15, 8, -5, 3, -1 },
  { -2, 4, -6, 12, -24, 108, 49, -18, 10, -6, 3, -2 },
  { -2, 4, -7, 13, -25, 100, 60, -21, 11, -7, 4, -2 },
  { -2, 4, -7, 13, -26, 91, 71, -24, 13, -7, 4, -2 },
  { -2, 4, -7, 13, -25, 81, 81, -25, 13, -7, 4, -2 },
  { -2, 4, -7, 13, -24, 71, 91, -26, 13, -7, 4, -2 },
  { -2, 4, -7, 11, -21, 60, 100, -25, 13, -7, 4, -2 },
  { -2, 3, -6, 10, -18, 49, 108, -24, 12, -6, 4, -2 },
  { -1, 3, -5, 8, -15, 38, 115, -21, 10, -6, 3, -1 },
  { -1, 2, -4, 7, -12, 28, 120, -18, 8, -4, 3, -1 },
  { -1, 2, -2, 4, -8, 18, 124, -13, 6, -3, 2, -1 },
  { 0, 1, -1, 2, -4, 8, 127, -7, 3, -2, 1, 0 },
};

/* av1_get_interp_filter_params_with_block_size + ..._subpel_kernel: the
 * kernel row of interp_filter (InterpFilter 0..4) for a block dimension of
 * `size` at `subpel` (0..15); returns the tap count (8 or 12). */
int orc_interp_kernel(int interp_filter, int size, int subpel, int16_t *out) {
  if (interp_filter == 4) {
    memcpy(out, kern12[subpel], 12 * sizeof(int16_t));
    return 12;
  }
  int kind = interp_filter;
  if (size <= 4) kind = interp_filter == 1 ? 5 : interp_filter == 3 ? 3 : 4;
  memcpy(out, kern8[kind][subpel], 8 * sizeof(int16_t));
  return 8;
}

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
#define RPOT(v, n) (((v) + ((1 << (n)) >> 1)) >> (n))

/* One block through the chosen convolve function.  path: 0 copy, 1 x_sr,
 * 2 y_sr, 3 2d_sr.  src points at the block's integer position; fx / fy are
 * the kernel rows already selected for the sub-pel phase. */
void orc_convolve_block(const void *src, ptrdiff_t ss, void *dst, ptrdiff_t ds, int w, int h,
                        int path, const int16_t *fx, int tx, const int16_t *fy, int ty,
                        int round_0, int round_1, int bd, int hbd) {
  if (path == 0) {
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) px_put(dst, y * ds + x, px_get(src, y * ss + x, hbd), hbd);
  } else if (path == 1) { /* convolve.c:156-188, 687-713 */
    const int fo = tx / 2 - 1, bits = FILTER_BITS_ORC - round_0;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        int32_t res = 0;
        for (int k = 0; k < tx; ++k) res += fx[k] * px_get(src, y * ss + x - fo + k, hbd);
        res = RPOT(res, round_0);
        px_put(dst, y * ds + x, clip_bd(RPOT(res, bits), bd), hbd);
      }
  } else if (path == 2) { /* convolve.c:135-154, 715-733 */
    const int fo = ty / 2 - 1;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        int32_t res = 0;
        for (int k = 0; k < ty; ++k) res += fy[k] * px_get(src, (y - fo + k) * ss + x, hbd);
        px_put(dst, y * ds + x, clip_bd(RPOT(res, FILTER_BITS_ORC), bd), hbd);
      }
  } else { /* convolve.c:76-133, 735-787 */
    static __thread int16_t im[(128 + 11) * 128];
    const int im_h = h + ty - 1, fov = ty / 2 - 1, foh = tx / 2 - 1;
    const int bits = 2 * FILTER_BITS_ORC - round_0 - round_1;
    for (int y = 0; y < im_h; ++y)
      for (int x = 0; x < w; ++x) {
        int32_t sum = 1 << (bd + FILTER_BITS_ORC - 1);
        for (int k = 0; k < tx; ++k)
          sum += fx[k] * px_get(src, (y - fov) * ss + x - foh + k, hbd);
        im[y * w + x] = (int16_t)RPOT(sum, round_0);
      }
    const int offset_bits = bd + 2 * FILTER_BITS_ORC - round_0;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        int32_t sum = 1 << offset_bits;
        for (int k = 0; k < ty; ++k) sum += fy[k] * im[(y + k) * w + x];
        const int32_t res = RPOT(sum, round_1) - ((1 << (offset_bits - round_1)) +
                                                  (1 << (offset_bits - round_1 - 1)));
        px_put(dst, y * ds + x, clip_bd(RPOT(res, bits), bd), hbd);
      }
  }
}

/* get_conv_params_no_round(0, plane, NULL, 0, 0, bd): round_0 / round_1 */
void orc_conv_rounds(int bd, int *round_0, int *round_1) {
  int r0 = 3, r1 = 2 * FILTER_BITS_ORC - 3;
  const int intbufrange = bd + FILTER_BITS_ORC - r0 + 2;
  if (intbufrange > 16) {
    r0 += intbufrange - 16;
    r1 -= intbufrange - 16;
  }
  *round_0 = r0;
  *round_1 = r1;
}

/* av1_enc_build_one_inter_predictor for every job (TRANSLATION_PRED,
 * UNIFORM_SINGLE, unscaled reference, not intrabc).  mvs (optional)
 * overrides each job's mv with a sub-pel search result. */
long orc_build_inter_pred_batch(const void *ref, int ref_stride, int ref_width, int ref_height,
                                int ss_x, int ss_y, int w, int h, const OrcInterPredJob *jobs,
                                long njobs, const OrcSubpelResult *mvs, void *dst,
                                int dst_stride, int bd, int hbd) {
  int r0, r1;
  orc_conv_rounds(hbd ? bd : 8, &r0, &r1);
  const int pbd = hbd ? bd : 8;
  const size_t es = hbd ? 2 : 1;
  for (long j = 0; j < njobs; ++j) {
    const OrcInterPredJob *jb = &jobs[j];
    const int mv_row = mvs ? mvs[j].best_row : jb->mv_row;
    const int mv_col = mvs ? mvs[j].best_col : jb->mv_col;
    /* init_subpel_params, unscaled */
    int pos_y = ((jb->pix_row << 4) + mv_row * (1 << (1 - ss_y))) * (1 << 6) + 32;
    int pos_x = ((jb->pix_col << 4) + mv_col * (1 << (1 - ss_x))) * (1 << 6) + 32;
    const int top = -(((288 >> ss_y) - 4) << 10), left = -(((288 >> ss_x) - 4) << 10);
    const int bottom = (ref_height + 4) << 10, right = (ref_width + 4) << 10;
    pos_y = pos_y < top ? top : pos_y > bottom ? bottom : pos_y;
    pos_x = pos_x < left ? left : pos_x > right ? right : pos_x;
    const int sx = (pos_x & 1023) >> 6, sy = (pos_y & 1023) >> 6;
    const char *src = (const char *)ref +
                      (jb->ref_off + (ptrdiff_t)(pos_y >> 10) * ref_stride + (pos_x >> 10)) * es;
    char *d = (char *)dst + jb->dst_off * es;
    int16_t fx[12], fy[12];
    const int tx = orc_interp_kernel(jb->filter_x, w, sx, fx);
    const int ty = orc_interp_kernel(jb->filter_y, h, sy, fy);
    const int path = (sx ? 1 : 0) + (sy ? 2 : 0);
    orc_convolve_block(src, ref_stride, d, dst_stride, w, h, path, fx, tx, fy, ty, r0, r1, pbd,
                       hbd);
  }
  return njobs;
}
