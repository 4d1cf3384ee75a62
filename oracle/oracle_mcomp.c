/* oracle_mcomp.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the DIAMOND full-pixel motion search of the reference:
 *   av1_init_dsmotion_compensation   av1/encoder/mcomp.c:369-404 (level 0)
 *   mvsad_err_cost / mv_err_cost     av1/encoder/mcomp.c:257-360 (L1 / none)
 *   diamond_search_sad               av1/encoder/mcomp.c:1318-1477
 *   full_pixel_diamond               av1/encoder/mcomp.c:1479-1526
 *   downsampled-SAD quality recheck  av1/encoder/mcomp.c:1840-1867
 *   FAST_BIGDIA (pattern_search)     av1/encoder/mcomp.c:498-550,1017-1316
 * with sdf/sdx4df = aom_sad / aom_sad_skip and vf = aom_variance of the
 * block size (oracle_dsp.c).  MV_COST_ENTROPY (needs the entropy context's
 * mv cost tables) and mesh refinement are not restated.
 */
#include <stdlib.h>

#include "oracle.h"

#define MAX_STEPS 11 /* MAX_MVSEARCH_STEPS, mcomp_structs.h:19 */

static int sad_lambda(int type) {
  return type == 1 ? 32 : type == 2 ? 15 : type == 3 ? 8 : 0;
}
static int sse_lambda(int type) {
  return type == 1 ? 2 : type == 2 ? 0 : type == 3 ? 1 : 0;
}

static int rawpel(int x) { return (x + 3 + (x >= 0)) >> 3; } /* mv.h:28 */

static unsigned mvsad_cost(const OrcMsParams *p, int row, int col) {
  if (p->mv_cost_type < 1 || p->mv_cost_type > 3) return 0;
  const int dr = (row - rawpel(p->ref_mv_row)) * 8;
  const int dc = (col - rawpel(p->ref_mv_col)) * 8;
  return (unsigned)((sad_lambda(p->mv_cost_type) * (abs(dr) + abs(dc))) >> 3);
}

static int mv_cost(const OrcMsParams *p, int row, int col) {
  if (p->mv_cost_type < 1 || p->mv_cost_type > 3) return 0;
  const int dr = row * 8 - p->ref_mv_row, dc = col * 8 - p->ref_mv_col;
  return (sse_lambda(p->mv_cost_type) * (abs(dr) + abs(dc))) >> 3;
}

static int in_range(const OrcMsParams *p, int row, int col) {
  return col >= p->col_min && col <= p->col_max && row >= p->row_min &&
         row <= p->row_max;
}

static unsigned block_sad(const OrcMsParams *p, int row, int col, int skip) {
  const uint8_t *r = p->ref + (ptrdiff_t)row * p->ref_stride + col;
  return skip ? orc_sad_skip(p->src, p->src_stride, r, p->ref_stride, p->w, p->h)
              : orc_sad(p->src, p->src_stride, r, p->ref_stride, p->w, p->h);
}

static int var_cost(const OrcMsParams *p, int row, int col) {
  unsigned sse;
  const uint8_t *r = p->ref + (ptrdiff_t)row * p->ref_stride + col;
  const int v = (int)orc_variance(p->src, p->src_stride, r, p->ref_stride, p->w, p->h, &sse);
  return v + mv_cost(p, row, col);
}

/* diamond_search_sad without second_pred / mask: returns bestsad, writes
 * the best mv and num00 (center steps).  *steps counts evaluated steps. */
static unsigned diamond(const OrcMsParams *p, int srow, int scol, int search_step, int skip,
                        int *brow, int *bcol, int *num00, int *steps) {
  static const int kDr[9] = { 0, -1, 1, 0, 0, -1, 1, -1, 1 };
  static const int kDc[9] = { 0, 0, 0, -1, 1, -1, 1, 1, -1 };
  if (scol < p->col_min) scol = p->col_min;
  if (scol > p->col_max) scol = p->col_max;
  if (srow < p->row_min) srow = p->row_min;
  if (srow > p->row_max) srow = p->row_max;
  int row = srow, col = scol, off_center = 0, center_steps = 0;
  unsigned best = mvsad_cost(p, row, col) + block_sad(p, row, col, skip);
  const int tot = MAX_STEPS - search_step;
  for (int step = tot - 1; step >= 0; --step) {
    const int rad = 1 << step; /* cfg->radius[step] at level 0 */
    int best_site = 0;
    const int all_in = row - rad >= p->row_min && row + rad <= p->row_max &&
                       col - rad >= p->col_min && col + rad <= p->col_max;
    for (int i = 1; i <= 8; ++i) {
      const int r = row + kDr[i] * rad, c = col + kDc[i] * rad;
      if (!all_in && !in_range(p, r, c)) continue;
      const unsigned s = block_sad(p, r, c, skip);
      if (s < best) {
        const unsigned t = s + mvsad_cost(p, r, c);
        if (t < best) {
          best = t;
          best_site = i;
        }
      }
    }
    ++*steps;
    if (best_site) {
      row += kDr[best_site] * rad;
      col += kDc[best_site] * rad;
      off_center = 1;
    }
    if (!off_center) ++center_steps;
  }
  *brow = row;
  *bcol = col;
  *num00 = center_steps;
  return best;
}

static int full_pixel_diamond(const OrcMsParams *p, int srow, int scol, int step_param, int skip,
                              int *brow, int *bcol, int *steps) {
  int n, num00 = 0;
  diamond(p, srow, scol, step_param, skip, brow, bcol, &n, steps);
  int bestsme = var_cost(p, *brow, *bcol);
  const int further = MAX_STEPS - 1 - step_param;
  while (n < further) {
    ++n;
    int tr, tc;
    diamond(p, srow, scol, step_param + n, skip, &tr, &tc, &num00, steps);
    const int sme = var_cost(p, tr, tc);
    if (sme < bestsme) {
      bestsme = sme;
      *brow = tr;
      *bcol = tc;
    }
    if (num00) {
      n += num00;
      num00 = 0;
    }
  }
  return bestsme;
}

int orc_full_pixel_search_diamond(const OrcMsParams *p, int start_row, int start_col,
                                  int step_param, int *best_row, int *best_col,
                                  int *steps) {
  *steps = 0;
  /* use_downsampled_sad only for blocks >= 16 high (mcomp.c:132-133) */
  const int skip = p->skip_sad && p->h >= 16;
  int var = full_pixel_diamond(p, start_row, start_col, step_param, skip, best_row, best_col,
                               steps);
  if (skip) {
    const uint8_t *r = p->ref + (ptrdiff_t)*best_row * p->ref_stride + *best_col;
    const int sad = (int)orc_sad(p->src, p->src_stride, r, p->ref_stride, p->w, p->h);
    const int ssad = (int)orc_sad_skip(p->src, p->src_stride, r, p->ref_stride, p->w, p->h);
    const int thresh = (p->w >> 2) * (p->h >> 2); /* 1 << (mi_w_log2 + mi_h_log2) */
    const int big = sad > 1 ? sad : 1;
    if (sad > thresh && abs(ssad - sad) * 10 >= big * 9)
      var = full_pixel_diamond(p, start_row, start_col, step_param, 0, best_row, best_col,
                               steps);
  }
  return var;
}

/* ---- FAST_BIGDIA: fast_bigdia_search -> bigdia_search -> pattern_search
 * (mcomp.c:1017-1245, 1266-1316) with do_init_search 0, sites of
 * av1_init_motion_compensation_bigdia (mcomp.c:498-550), candidate updates
 * update_mvs_and_sad (mcomp.c:858-877) in site order.  Written in the
 * reference's cost_list == NULL form; with a cost list the reference finishes
 * scale 0 in a separate block whose mv result is identical for
 * do_init_search 0.  *steps counts candidate rounds (full or 3-point). */
static void bigdia_site(int s, int i, int *dr, int *dc) {
  static const int k0r[4] = { 0, 1, 0, -1 }, k0c[4] = { -1, 0, 1, 0 };
  static const int kr[8] = { -1, 0, 1, 2, 1, 0, -1, -2 }, kc[8] = { -1, -2, -1, 0, 1, 2, 1, 0 };
  if (s == 0) {
    *dr = k0r[i];
    *dc = k0c[i];
  } else {
    const int r = 1 << (s - 1);
    *dr = kr[i] * r;
    *dc = kc[i] * r;
  }
}

/* update_mvs_and_sad without raw / second-best tracking */
static int bd_update(const OrcMsParams *p, unsigned thissad, int r, int c, unsigned *best) {
  if (thissad >= *best) return 0;
  const unsigned sad = thissad + mvsad_cost(p, r, c);
  if (sad < *best) {
    *best = sad;
    return 1;
  }
  return 0;
}

static int fast_bigdia(const OrcMsParams *p, int srow, int scol, int step_param, int skip,
                       int *brow, int *bcol, int *steps) {
  int search_step = step_param > MAX_STEPS - 3 ? step_param : MAX_STEPS - 3;
  if (search_step > MAX_STEPS - 1) search_step = MAX_STEPS - 1;
  int s = MAX_STEPS - 1 - search_step; /* search_steps[search_step] */
  if (scol < p->col_min) scol = p->col_min;
  if (scol > p->col_max) scol = p->col_max;
  if (srow < p->row_min) srow = p->row_min;
  if (srow > p->row_max) srow = p->row_max;
  int br = srow, bc = scol, k = -1;
  unsigned best = block_sad(p, br, bc, skip) + mvsad_cost(p, br, bc);
  int best_site = -1;
  for (; s >= 0; s--) {
    const int n = s == 0 ? 4 : 8;
    const int all_in = br - (1 << s) >= p->row_min && br + (1 << s) <= p->row_max &&
                       bc - (1 << s) >= p->col_min && bc + (1 << s) <= p->col_max;
    for (int i = 0; i < n; ++i) { /* calc_sad4_update_bestmv / calc_sad_update_bestmv */
      int dr, dc;
      bigdia_site(s, i, &dr, &dc);
      if (!all_in && !in_range(p, br + dr, bc + dc)) continue;
      if (bd_update(p, block_sad(p, br + dr, bc + dc, skip), br + dr, bc + dc, &best))
        best_site = i;
    }
    ++*steps;
    if (best_site == -1) continue;
    {
      int dr, dc;
      bigdia_site(s, best_site, &dr, &dc);
      br += dr;
      bc += dc;
      k = best_site;
    }
    do {
      int idx[3];
      best_site = -1;
      idx[0] = (k == 0) ? n - 1 : k - 1;
      idx[1] = k;
      idx[2] = (k == n - 1) ? 0 : k + 1;
      const int in3 = br - (1 << s) >= p->row_min && br + (1 << s) <= p->row_max &&
                      bc - (1 << s) >= p->col_min && bc + (1 << s) <= p->col_max;
      for (int j = 0; j < 3; ++j) { /* calc_sad3_update_bestmv / _with_indices */
        int dr, dc;
        bigdia_site(s, idx[j], &dr, &dc);
        if (!in3 && !in_range(p, br + dr, bc + dc)) continue;
        if (bd_update(p, block_sad(p, br + dr, bc + dc, skip), br + dr, bc + dc, &best))
          best_site = j;
      }
      ++*steps;
      if (best_site != -1) {
        k = idx[best_site];
        int dr, dc;
        bigdia_site(s, k, &dr, &dc);
        br += dr;
        bc += dc;
      }
    } while (best_site != -1);
  }
  *brow = br;
  *bcol = bc;
  return var_cost(p, br, bc); /* get_mvpred_var_cost */
}

int orc_full_pixel_search_bigdia(const OrcMsParams *p, int start_row, int start_col,
                                 int step_param, int *best_row, int *best_col, int *steps) {
  *steps = 0;
  const int skip = p->skip_sad && p->h >= 16;
  int var = fast_bigdia(p, start_row, start_col, step_param, skip, best_row, best_col, steps);
  if (skip) { /* av1_full_pixel_search quality recheck, mcomp.c:1840-1873 */
    const uint8_t *r = p->ref + (ptrdiff_t)*best_row * p->ref_stride + *best_col;
    const int sad = (int)orc_sad(p->src, p->src_stride, r, p->ref_stride, p->w, p->h);
    const int ssad = (int)orc_sad_skip(p->src, p->src_stride, r, p->ref_stride, p->w, p->h);
    const int thresh = (p->w >> 2) * (p->h >> 2);
    const int big = sad > 1 ? sad : 1;
    if (sad > thresh && abs(ssad - sad) * 10 >= big * 9)
      var = fast_bigdia(p, start_row, start_col, step_param, 0, best_row, best_col, steps);
  }
  return var;
}

/* ---- batch driver (pthreads over job ranges) ---- */
#include <pthread.h>

typedef struct {
  const uint8_t *src, *ref;
  int ss, rs, w, h, step_param, cost, skip, method;
  const OrcDiamondJob *jobs;
  OrcDiamondResult *out;
  long lo, hi;
} BatchArg;

static void *batch_worker(void *v) {
  const BatchArg *a = (const BatchArg *)v;
  for (long j = a->lo; j < a->hi; ++j) {
    const OrcDiamondJob *jb = &a->jobs[j];
    OrcMsParams p = { a->src + jb->src_off, a->ss, a->ref + jb->ref_off, a->rs, a->w, a->h,
                      jb->col_min, jb->col_max, jb->row_min, jb->row_max, jb->ref_mv_row,
                      jb->ref_mv_col, a->cost, a->skip };
    int br, bc, steps;
    a->out[j].bestsme =
        a->method ? orc_full_pixel_search_bigdia(&p, jb->start_row, jb->start_col, a->step_param,
                                                 &br, &bc, &steps)
                  : orc_full_pixel_search_diamond(&p, jb->start_row, jb->start_col,
                                                  a->step_param, &br, &bc, &steps);
    a->out[j].best_row = (int16_t)br;
    a->out[j].best_col = (int16_t)bc;
    a->out[j].steps = steps;
    a->out[j].reserved = 0;
  }
  return NULL;
}

static void fullpel_batch(const uint8_t *src, int src_stride, const uint8_t *ref,
                          int ref_stride, int w, int h, const OrcDiamondJob *jobs, long njobs,
                          int step_param, int mv_cost_type, int skip_sad, int method,
                          OrcDiamondResult *out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t tid[64];
  BatchArg args[64];
  for (int t = 0; t < threads; ++t) {
    args[t] = (BatchArg){ src, ref, src_stride, ref_stride, w, h, step_param, mv_cost_type,
                          skip_sad, method, jobs, out, njobs * t / threads,
                          njobs * (t + 1) / threads };
    if (threads > 1) pthread_create(&tid[t], NULL, batch_worker, &args[t]);
    else batch_worker(&args[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}

void orc_diamond_batch(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride,
                       int w, int h, const OrcDiamondJob *jobs, long njobs, int step_param,
                       int mv_cost_type, int skip_sad, OrcDiamondResult *out, int threads) {
  fullpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, step_param, mv_cost_type,
                skip_sad, 0, out, threads);
}

void orc_bigdia_batch(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride,
                      int w, int h, const OrcDiamondJob *jobs, long njobs, int step_param,
                      int mv_cost_type, int skip_sad, OrcDiamondResult *out, int threads) {
  fullpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, step_param, mv_cost_type,
                skip_sad, 1, out, threads);
}
