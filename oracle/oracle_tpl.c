/* oracle_tpl.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the TPL model's per-block transform leg
 * (av1/encoder/tpl_model.c): for every block and prediction,
 * tpl_get_satd_cost (:199-210: av1_subtract_block, av1_quick_txfm with
 * use_hadamard 0 = DCT_DCT 2-D, aom_satd); the cheapest prediction (strictly
 * lower cost wins); then txfm_quant_rdcost (:225-247): get_quantize_error
 * (:98-135: FP quantizer, log_scale of the size, DCT_DCT scan, block error
 * and sse >> (TX_32X32 ? 0 : 2) clamped to >= 1), rate_estimator (:212-223)
 * and av1_inverse_transform_block into the prediction.  Built from the
 * oracle's pinned pieces (orc_fwd_txfm2d, orc_quantize_fp, orc_block_error,
 * orc_inv_txfm2d_add).
 */
#include <limits.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  const void *src, *preds;
  long pred_plane;
  int src_stride, pred_stride, nrefs, nbx, bsize, bd, recon_stride;
  const OrcQuant *q;
  OrcTplBlock *out;
  void *recon;
  int32_t *ref_costs;
  long lo, hi;
} TplArg;

static int px(const void *p, long off, int hbd) {
  return hbd ? ((const uint16_t *)p)[off] : ((const uint8_t *)p)[off];
}

static int msb(unsigned v) { /* get_msb */
  int n = 0;
  while (v >>= 1) ++n;
  return n;
}

static void *tpl_worker(void *v) {
  const TplArg *a = (const TplArg *)v;
  const int N = a->bsize, n = N * N, hbd = a->bd > 8;
  const int ts = N == 8 ? 1 : N == 16 ? 2 : 3; /* TX_8X8 / 16X16 / 32X32 */
  const int ls = (n > 256) + (n > 1024);
  const int shift = ts == 3 ? 0 : 2;
  const int16_t *scan = orc_scan(ts, 0), *iscan = orc_iscan(ts, 0);
  int16_t diff[32 * 32];
  int32_t coeff[32 * 32], best[32 * 32], qc[32 * 32], dq[32 * 32];
  uint16_t rec[32 * 32];
  for (long blk = a->lo; blk < a->hi; ++blk) {
    const long bx = (blk % a->nbx) * N, by = (blk / a->nbx) * N;
    int best_k = -1, best_cost = 0x7FFFFFFF;
    for (int k = 0; k < a->nrefs; ++k) {
      const long pb = k * a->pred_plane + by * a->pred_stride + bx;
      for (int r = 0; r < N; ++r)
        for (int c = 0; c < N; ++c)
          diff[r * N + c] = (int16_t)(px(a->src, (by + r) * a->src_stride + bx + c, hbd) -
                                      px(a->preds, pb + (long)r * a->pred_stride + c, hbd));
      orc_fwd_txfm2d(diff, coeff, N, 0, ts, a->bd);
      int satd = 0;
      for (int i = 0; i < n; ++i) satd += abs(coeff[i]);
      if (a->ref_costs) a->ref_costs[blk * a->nrefs + k] = satd;
      if (satd < best_cost) {
        best_cost = satd;
        best_k = k;
        memcpy(best, coeff, sizeof(int32_t) * n);
      }
    }
    uint16_t eob;
    if (hbd)
      orc_highbd_quantize_fp(best, n, a->q->zbin, a->q->round_fp, a->q->quant_fp,
                             a->q->quant_shift, qc, dq, a->q->dequant, &eob, scan, iscan, ls);
    else
      orc_quantize_fp(best, n, a->q->zbin, a->q->round_fp, a->q->quant_fp, a->q->quant_shift,
                      qc, dq, a->q->dequant, &eob, scan, iscan, ls);
    int64_t sse;
    int64_t err = hbd ? orc_highbd_block_error(best, dq, n, &sse, a->bd)
                      : orc_block_error(best, dq, n, &sse);
    err >>= shift;
    sse >>= shift;
    int rate = 1;
    for (int i = 0; i < eob; ++i) {
      const unsigned al = (unsigned)abs(qc[scan[i]]);
      rate += msb(al + 1) + 1 + (al > 0);
    }
    const long pb = (long)best_k * a->pred_plane + by * a->pred_stride + bx;
    for (int r = 0; r < N; ++r)
      for (int c = 0; c < N; ++c)
        rec[r * N + c] = (uint16_t)px(a->preds, pb + (long)r * a->pred_stride + c, hbd);
    if (eob) orc_inv_txfm2d_add(dq, rec, N, 0, ts, a->bd);
    for (int r = 0; r < N; ++r)
      for (int c = 0; c < N; ++c) {
        const long o = (by + r) * a->recon_stride + bx + c;
        if (hbd) ((uint16_t *)a->recon)[o] = rec[r * N + c];
        else ((uint8_t *)a->recon)[o] = (uint8_t)rec[r * N + c];
      }
    OrcTplBlock *o = &a->out[blk];
    o->best_ref = best_k;
    o->inter_cost = best_cost;
    o->rate_cost = rate << 9;
    o->eob = eob;
    o->recon_error = err > 1 ? err : 1;
    o->sse = sse > 1 ? sse : 1;
  }
  return NULL;
}

void orc_tpl_block_batch(const void *src, int src_stride, const void *preds, long pred_plane,
                         int pred_stride, int nrefs, int width, int height, int bsize, int bd,
                         const OrcQuant *q, OrcTplBlock *out, void *recon, int recon_stride,
                         int32_t *ref_costs, int threads) {
  const long nblocks = (long)(width / bsize) * (height / bsize);
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t tid[64];
  TplArg args[64];
  for (int t = 0; t < threads; ++t) {
    args[t] = (TplArg){ src, preds, pred_plane, src_stride, pred_stride, nrefs, width / bsize,
                        bsize, bd, recon_stride, q, out, recon, ref_costs,
                        nblocks * t / threads, nblocks * (t + 1) / threads };
    if (threads > 1) pthread_create(&tid[t], NULL, tpl_worker, &args[t]);
    else tpl_worker(&args[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}

/* ---- TPL motion search with start-mv candidates ------------------------
 * mode_estimation's per-reference loop (av1/encoder/tpl_model.c:632-743)
 * over a frame of TPL blocks in raster order, one thread per reference (the
 * references are independent; within one the blocks are sequential, as in
 * the reference's row-synchronised walk):
 *   center_mvs = {zero}; above (:656-664), left (:666-674), above-right
 *   (:676-685) tpl mvs of the same reference unless is_alike_mv (:319-333);
 *   the third-pass mv into slot 0 (:687-703); prune_starting_mv (:705-728):
 *   sdf at the clamped full-pel centres, qsort by compare_sad (:310-317;
 *   insertion sort here: stable, as glibc's qsort is for <= 4 entries),
 *   the cut to 4 - prune_starting_mv, the SAD-gap cut; motion_estimation
 *   (:249-303) per centre: av1_full_pixel_search from get_fullmv_from_mv
 *   (centre) with ref_mv = centre (av1_make_default_fullpel_ms_params ->
 *   av1_set_mv_search_range, mcomp.c:95-164,206-234) and, at
 *   subpel_force_stop FULL_PEL, the sub-pel step's setup_center_error: the
 *   variance at the full-pel best (MV_COST_NONE); strict < keeps the first
 *   best (:736-739). */
typedef struct {
  const uint8_t *src, *ref;
  int ss, rs, cols, rows, method, step_param, skip, prune, thr, nrefs;
  const OrcMvCost *cost;
  const OrcDiamondJob *jobs;
  const int32_t *third;
  int32_t *mvs, *cls, *centers;
  OrcDiamondResult *out;
  int ref_idx;
} TplMvArg;

static int rawpel_mv(int x) { return (x + 3 + (x >= 0)) >> 3; } /* GET_MV_RAWPEL, mv.h:28 */
static int mvr(int32_t m) { return (int16_t)(m & 0xFFFF); }
static int mvc(int32_t m) { return (int16_t)((uint32_t)m >> 16); }
static int32_t mvpack(int r, int c) { return (int32_t)(((uint32_t)(uint16_t)c << 16) | (uint16_t)r); }

typedef struct {
  int row, col, sad;
} CenterMv; /* center_mv_t */

static int is_alike(int r, int c, const CenterMv *cm, int n, int thr) {
  for (int i = 0; i < n; ++i)
    if (abs(cm[i].col - c) < thr && abs(cm[i].row - r) < thr) return 1;
  return 0;
}

/* AOMMIN(reduce_first_step_size, MAX_MVSEARCH_STEPS - 2) (:270-271) */
#define MAX_TPL_STEP 9

static void *tpl_mv_worker(void *v) {
  const TplMvArg *a = (const TplMvArg *)v;
  const int k = a->ref_idx;
  const long nb = (long)a->rows * a->cols;
  int32_t *mvs = a->mvs + k * nb;
  for (int r = 0; r < a->rows; ++r)
    for (int c = 0; c < a->cols; ++c) {
      const long bi = (long)r * a->cols + c, j = k * nb + bi;
      const OrcDiamondJob *jb = &a->jobs[j];
      CenterMv cm[4] = { { 0, 0, INT_MAX }, { 0, 0, INT_MAX }, { 0, 0, INT_MAX },
                         { 0, 0, INT_MAX } };
      int n = 1;
      int32_t cand[3];
      int nc = 0;
      if (r > 0) cand[nc++] = mvs[bi - a->cols];
      if (c > 0) cand[nc++] = mvs[bi - 1];
      if (r > 0 && c + 1 < a->cols) cand[nc++] = mvs[bi - a->cols + 1];
      for (int i = 0; i < nc; ++i)
        if (!is_alike(mvr(cand[i]), mvc(cand[i]), cm, n, a->thr)) {
          cm[n].row = mvr(cand[i]);
          cm[n].col = mvc(cand[i]);
          ++n;
        }
      if (a->third && a->third[j] != (int32_t)0x80008000 &&
          !is_alike(mvr(a->third[j]), mvc(a->third[j]), cm + 1, n - 1, a->thr)) {
        cm[0].row = mvr(a->third[j]);
        cm[0].col = mvc(a->third[j]);
      }
      const uint8_t *sb = a->src + jb->src_off, *rb = a->ref + jb->ref_off;
      if (a->prune) {
        for (int i = 0; i < n; ++i) {
          int fr = rawpel_mv(cm[i].row), fc = rawpel_mv(cm[i].col);
          fr = fr < jb->row_min ? jb->row_min : fr > jb->row_max ? jb->row_max : fr;
          fc = fc < jb->col_min ? jb->col_min : fc > jb->col_max ? jb->col_max : fc;
          cm[i].sad = (int)orc_sad(sb, a->ss, rb + (long)fr * a->rs + fc, a->rs, 16, 16);
        }
        for (int i = 1; i < n; ++i) {
          const CenterMv x = cm[i];
          int q = i;
          while (q > 0 && cm[q - 1].sad > x.sad) {
            cm[q] = cm[q - 1];
            --q;
          }
          cm[q] = x;
        }
        if (n > 4 - a->prune) n = 4 - a->prune;
        if (n > 1 && (cm[n - 1].sad - cm[n - 2].sad) * 5 > cm[n - 2].sad) --n;
      }
      unsigned bestsme = 0xFFFFFFFFu;
      int best_r = 0, best_c = 0;
      for (int i = 0; i < n; ++i) {
        OrcMsParams p = { sb, a->ss, rb, a->rs, 16, 16, jb->col_min, jb->col_max, jb->row_min,
                          jb->row_max, cm[i].row, cm[i].col, a->cost->mv_cost_type, a->skip,
                          a->cost };
        /* av1_set_mv_search_range (MAX_FULL_PEL_VAL 1023, MV_LOW/UPP -/+2^14) */
        int t;
        t = ((cm[i].col + 7) >> 3) - 1023; t = t > -2047 ? t : -2047;
        if (p.col_min < t) p.col_min = t;
        t = ((cm[i].row + 7) >> 3) - 1023; t = t > -2047 ? t : -2047;
        if (p.row_min < t) p.row_min = t;
        t = (cm[i].col >> 3) + 1023; t = t < 2047 ? t : 2047;
        if (p.col_max > t) p.col_max = t;
        t = (cm[i].row >> 3) + 1023; t = t < 2047 ? t : 2047;
        if (p.row_max > t) p.row_max = t;
        if (p.col_max < p.col_min) p.col_max = p.col_min;
        if (p.row_max < p.row_min) p.row_max = p.row_min;
        int cl[5], br, bc, steps = 0;
        const int sme = orc_full_pixel_search(&p, a->method, rawpel_mv(cm[i].row),
                                              rawpel_mv(cm[i].col), a->step_param,
                                              a->cls ? cl : NULL, &br, &bc, &steps);
        unsigned sse;
        const unsigned thissme =
            orc_variance(sb, a->ss, rb + (long)br * a->rs + bc, a->rs, 16, 16, &sse);
        if (thissme < bestsme) {
          bestsme = thissme;
          best_r = br;
          best_c = bc;
          a->out[j].best_row = (int16_t)br;
          a->out[j].best_col = (int16_t)bc;
          a->out[j].bestsme = sme;
          a->out[j].steps = steps;
          a->out[j].reserved = 0;
          if (a->cls) memcpy(a->cls + 5 * j, cl, sizeof(cl));
          if (a->centers) a->centers[j] = mvpack(cm[i].row, cm[i].col);
        }
      }
      mvs[bi] = mvpack(8 * best_r, 8 * best_c);
    }
  return NULL;
}

void orc_tpl_motion_search(const uint8_t *src, int src_stride, const uint8_t *ref,
                           int ref_stride, const OrcDiamondJob *jobs, int cols, int rows,
                           int nrefs, int method, int step_param, int skip_sad,
                           int prune_starting_mv, int skip_alike_starting_mv,
                           const OrcMvCost *cost, const int32_t *third, int32_t *mvs,
                           OrcDiamondResult *out, int32_t *cost_lists, int32_t *centers) {
  static const int thr[3] = { 1, 8 << 3, 16 << 3 }; /* mv_diff_thr (:322) */
  if (nrefs > 64) nrefs = 64;
  pthread_t tid[64];
  TplMvArg args[64];
  const int sp = step_param < MAX_TPL_STEP ? step_param : MAX_TPL_STEP;
  for (int k = 0; k < nrefs; ++k) {
    args[k] = (TplMvArg){ src, ref, src_stride, ref_stride, cols, rows, method, sp, skip_sad,
                          prune_starting_mv, thr[skip_alike_starting_mv], nrefs, cost, jobs,
                          third, mvs, cost_lists, centers, out, k };
    if (nrefs > 1) pthread_create(&tid[k], NULL, tpl_mv_worker, &args[k]);
    else tpl_mv_worker(&args[k]);
  }
  if (nrefs > 1)
    for (int k = 0; k < nrefs; ++k) pthread_join(tid[k], NULL);
}
