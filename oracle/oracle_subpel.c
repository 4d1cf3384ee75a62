/* oracle_subpel.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the sub-pixel motion refinement the encoder runs after
 * the full-pel search at speed >= 4:
 *   av1_find_best_sub_pixel_tree_pruned_more  av1/encoder/mcomp.c:2907-2981
 *     (cost_list NULL, last_mv_search_list NULL, unscaled reference)
 *   setup_center_error                        mcomp.c:2781-2838 (vf at the
 *                                             full-pel start, no second_pred)
 *   two_level_checks_fast                     mcomp.c:2675-2686
 *   first_level_check_fast                    mcomp.c:2566-2604
 *   second_level_check_fast                   mcomp.c:2608-2669
 *   check_better_fast / estimated_pref_error  mcomp.c:2496-2523, 2368-2397
 *     (svf = aom_sub_pixel_variance: the bilinear estimate)
 *   get_best_diag_step                        mcomp.c:2555-2562
 *   mv_err_cost_ (L1 types / none)            mcomp.c:290-323
 *   av1_is_subpelmv_in_range                  mcomp.h:375-379
 * 8-bit planes.  MVs in 1/8 pel; the reference block at mv is at
 * ref + (row >> 3) * stride + (col >> 3) with offsets (col & 7, row & 7).
 */
#include <limits.h>
#include <pthread.h>
#include <stdlib.h>

#include "oracle.h"

typedef struct {
  const uint8_t *src, *ref;
  int ss, rs, w, h, cost_type;
  const OrcSubpelJob *jb;
} SpCtx;

static int sp_lambda(int t) { return t == 1 ? 2 : t == 2 ? 0 : t == 3 ? 1 : 0; }

/* mv_err_cost_ for MV_COST_L1_* / MV_COST_NONE (mcomp.c:290-323) */
static int sp_mv_cost(const SpCtx *c, int row, int col) {
  if (c->cost_type < 1 || c->cost_type > 3) return 0;
  const int dr = abs(row - c->jb->ref_mv_row), dc = abs(col - c->jb->ref_mv_col);
  return (sp_lambda(c->cost_type) * (dr + dc)) >> 3;
}

static int sp_in_range(const SpCtx *c, int row, int col) {
  return col >= c->jb->col_min && col <= c->jb->col_max && row >= c->jb->row_min &&
         row <= c->jb->row_max;
}

static unsigned sp_svf(const SpCtx *c, int row, int col, unsigned *sse) {
  const uint8_t *r = c->ref + c->jb->ref_off + (ptrdiff_t)(row >> 3) * c->rs + (col >> 3);
  return orc_sub_pixel_variance(r, c->rs, col & 7, row & 7, c->src + c->jb->src_off, c->ss,
                                c->w, c->h, sse);
}

typedef struct {
  int row, col;
  unsigned besterr, sse1;
  int distortion;
} SpBest;

/* check_better_fast: returns the candidate's cost, INT_MAX when out of range */
static unsigned sp_check(const SpCtx *c, int row, int col, SpBest *b) {
  if (!sp_in_range(c, row, col)) return INT_MAX;
  unsigned sse;
  const int thismse = (int)sp_svf(c, row, col, &sse);
  unsigned cost = (unsigned)sp_mv_cost(c, row, col);
  cost += (unsigned)thismse;
  if (cost < b->besterr) {
    b->besterr = cost;
    b->row = row;
    b->col = col;
    b->distortion = thismse;
    b->sse1 = sse;
  }
  return cost;
}

static void sp_two_level(const SpCtx *c, int tr, int tc, int hstep, int iters, SpBest *b) {
  const unsigned left = sp_check(c, tr, tc - hstep, b);
  const unsigned right = sp_check(c, tr, tc + hstep, b);
  const unsigned up = sp_check(c, tr - hstep, tc, b);
  const unsigned down = sp_check(c, tr + hstep, tc, b);
  const int dr = up <= down ? -hstep : hstep, dc = left <= right ? -hstep : hstep;
  sp_check(c, tr + dr, tc + dc, b);
  if (iters <= 1) return;
  const int br = b->row, bc = b->col;
  if (tr != br && tc != bc) {
    sp_check(c, br, bc + dc, b);
    sp_check(c, br + dr, bc, b);
  } else if (tr == br && tc != bc) {
    sp_check(c, br + hstep, bc + dc, b);
    sp_check(c, br - hstep, bc + dc, b);
    sp_check(c, br - dr, bc, b);
  } else if (tr != br && tc == bc) {
    sp_check(c, br + dr, bc + hstep, b);
    sp_check(c, br + dr, bc - hstep, b);
    sp_check(c, br, bc - dc, b);
  }
}

/* forced_stop: 0 EIGHTH_PEL, 1 QUARTER_PEL, 2 HALF_PEL, 3 FULL_PEL */
static void sp_search(const SpCtx *c, int forced_stop, int allow_hp, int iters,
                      OrcSubpelResult *out) {
  SpBest b;
  b.row = c->jb->start_row;
  b.col = c->jb->start_col;
  /* setup_center_error: vf at the (full-pel) start */
  unsigned sse;
  const uint8_t *r = c->ref + c->jb->ref_off + (ptrdiff_t)(b.row >> 3) * c->rs + (b.col >> 3);
  const unsigned v = orc_variance(r, c->rs, c->src + c->jb->src_off, c->ss, c->w, c->h, &sse);
  b.distortion = (int)v;
  b.sse1 = sse;
  b.besterr = v + (unsigned)sp_mv_cost(c, b.row, b.col);
  if (forced_stop != 3) {
    int hstep = 4; /* INIT_SUBPEL_STEP_SIZE */
    sp_two_level(c, c->jb->start_row, c->jb->start_col, hstep, iters, &b);
    if (forced_stop < 2) {
      hstep >>= 1;
      sp_two_level(c, b.row, b.col, hstep, iters, &b);
    }
    if (allow_hp && forced_stop == 0) {
      hstep >>= 1;
      sp_two_level(c, b.row, b.col, hstep, iters, &b);
    }
  }
  out->best_row = (int16_t)b.row;
  out->best_col = (int16_t)b.col;
  out->besterr = b.besterr;
  out->distortion = b.distortion;
  out->sse = b.sse1;
}

typedef struct {
  SpCtx base;
  const OrcSubpelJob *jobs;
  OrcSubpelResult *out;
  int forced_stop, allow_hp, iters;
  long lo, hi;
} SpArg;

static void *sp_worker(void *v) {
  SpArg *a = (SpArg *)v;
  for (long j = a->lo; j < a->hi; ++j) {
    SpCtx c = a->base;
    c.jb = &a->jobs[j];
    sp_search(&c, a->forced_stop, a->allow_hp, a->iters, &a->out[j]);
  }
  return NULL;
}

void orc_subpel_batch(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride,
                      int w, int h, const OrcSubpelJob *jobs, long njobs, int forced_stop,
                      int allow_hp, int iters_per_step, int mv_cost_type, OrcSubpelResult *out,
                      int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t tid[64];
  SpArg args[64];
  for (int t = 0; t < threads; ++t) {
    args[t].base = (SpCtx){ src, ref, src_stride, ref_stride, w, h, mv_cost_type, NULL };
    args[t].jobs = jobs;
    args[t].out = out;
    args[t].forced_stop = forced_stop;
    args[t].allow_hp = allow_hp;
    args[t].iters = iters_per_step;
    args[t].lo = njobs * t / threads;
    args[t].hi = njobs * (t + 1) / threads;
    if (threads > 1) pthread_create(&tid[t], NULL, sp_worker, &args[t]);
    else sp_worker(&args[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}
