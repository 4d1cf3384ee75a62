/* oracle_subpel.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the sub-pixel motion refinement the encoder runs after
 * the full-pel search:
 *   av1_find_best_sub_pixel_tree_pruned_more  av1/encoder/mcomp.c:2907-2990
 *   av1_find_best_sub_pixel_tree_pruned       av1/encoder/mcomp.c:2992-3126
 *     (last_mv_search_list NULL, unscaled reference), with the full-pel
 *     search's cost list: is_cost_list_wellbehaved / get_cost_surf_min
 *     (:2857-2876) for pruned_more, the whichdir quadrant for pruned
 *   setup_center_error                        mcomp.c:2781-2838 (vf at the
 *                                             full-pel start, no second_pred)
 *   two_level_checks_fast                     mcomp.c:2675-2686
 *   first_level_check_fast                    mcomp.c:2566-2604
 *   second_level_check_fast                   mcomp.c:2608-2669
 *   check_better_fast / estimated_pref_error  mcomp.c:2496-2523, 2368-2397
 *     (svf = aom_sub_pixel_variance: the bilinear estimate)
 *   get_best_diag_step                        mcomp.c:2555-2562
 *   mv_err_cost_ (entropy / L1 / none)        mcomp.c:290-323
 *   av1_is_subpelmv_in_range                  mcomp.h:375-379
 *   SUBPEL_TREE with subpel_search_type != USE_2_TAPS_ORIG: first_level_check
 *     / check_better / upsampled_pref_error (mcomp.c:2402-2491,2528-2551,
 *     2689-2723), second_level_check_v2's check_better branch (:2752-2762),
 *     aom_upsampled_pred_c (reconinter_enc.c:424-496, unscaled) through
 *     aom_convolve8_horiz_c / _vert_c (aom_dsp/aom_convolve.c:36-113) with
 *     av1_get_filter (filter.h:276-285)
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
  const OrcMvCost *cost; /* MV_COST_ENTROPY tables and error_per_bit */
  int search_type;       /* SUBPEL_SEARCH_TYPE of SUBPEL_TREE: 0 USE_2_TAPS_ORIG .. 3 USE_8_TAPS */
} SpCtx;

static int sp_lambda(int t) { return t == 1 ? 2 : t == 2 ? 0 : t == 3 ? 1 : 0; }

/* mv_err_cost_ (mcomp.c:290-323) */
static int sp_mv_cost(const SpCtx *c, int row, int col) {
  const int dr = row - c->jb->ref_mv_row, dc = col - c->jb->ref_mv_col;
  if (c->cost_type == 0) {
    const OrcMvCost *m = c->cost;
    const int joint = (dc != 0) | ((dr != 0) << 1);
    const int rate = m->mvjcost[joint] + m->mvcost[0][dr] + m->mvcost[1][dc];
    return (int)(((int64_t)rate * m->error_per_bit + 8192) >> 14);
  }
  if (c->cost_type < 1 || c->cost_type > 3) return 0;
  return (sp_lambda(c->cost_type) * (abs(dr) + abs(dc))) >> 3;
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

static uint8_t clip8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* upsampled_pref_error (mcomp.c:2402-2491) for an unscaled reference, no
 * second_pred: aom_upsampled_pred_c's prediction at mv, then vf.  The kernel
 * row is av1_get_filter(subpel_search) at phase 2 * q3: USE_2_TAPS the
 * bilinear, USE_4_TAPS the 4-tap regular, USE_8_TAPS the 8-tap regular
 * kernels, all in the 8-tap layout; each aom_convolve8 pass rounds by
 * FILTER_BITS and clips to 8 bits, the 2-D case filtering rows -3 .. h + 4
 * horizontally into a temporary first. */
static unsigned sp_upsampled(const SpCtx *c, int row, int col, unsigned *sse) {
  const int w = c->w, h = c->h, sx = col & 7, sy = row & 7;
  const uint8_t *r = c->ref + c->jb->ref_off + (ptrdiff_t)(row >> 3) * c->rs + (col >> 3);
  const int filt = c->search_type == 1 ? 3 : 0;    /* BILINEAR : EIGHTTAP_REGULAR */
  const int size = c->search_type == 2 ? 4 : 8;    /* a size of 4 selects the 4-tap kernels */
  int16_t kx[8], ky[8];
  orc_interp_kernel(filt, size, 2 * sx, kx);
  orc_interp_kernel(filt, size, 2 * sy, ky);
  static __thread uint8_t pred[128 * 128], tmp[(128 + 7) * 128];
  if (!sx && !sy) {
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) pred[y * w + x] = r[(ptrdiff_t)y * c->rs + x];
  } else if (!sy) {
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        int sum = 0;
        for (int k = 0; k < 8; ++k) sum += r[(ptrdiff_t)y * c->rs + x - 3 + k] * kx[k];
        pred[y * w + x] = clip8((sum + 64) >> 7);
      }
  } else if (!sx) {
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        int sum = 0;
        for (int k = 0; k < 8; ++k) sum += r[(ptrdiff_t)(y - 3 + k) * c->rs + x] * ky[k];
        pred[y * w + x] = clip8((sum + 64) >> 7);
      }
  } else {
    for (int y = 0; y < h + 7; ++y)
      for (int x = 0; x < w; ++x) {
        int sum = 0;
        for (int k = 0; k < 8; ++k) sum += r[(ptrdiff_t)(y - 3) * c->rs + x - 3 + k] * kx[k];
        tmp[y * w + x] = clip8((sum + 64) >> 7);
      }
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        int sum = 0;
        for (int k = 0; k < 8; ++k) sum += tmp[(y + k) * w + x] * ky[k];
        pred[y * w + x] = clip8((sum + 64) >> 7);
      }
  }
  return orc_variance(pred, w, c->src + c->jb->src_off, c->ss, w, h, sse);
}

typedef struct {
  int row, col;
  unsigned besterr, sse1;
  int distortion;
} SpBest;

/* check_better_fast (the svf estimate) or, for SUBPEL_TREE with a
 * subpel_search_type other than USE_2_TAPS_ORIG, check_better (the upsampled
 * prediction): returns the candidate's cost, INT_MAX when out of range */
static unsigned sp_check(const SpCtx *c, int row, int col, SpBest *b) {
  if (!sp_in_range(c, row, col)) return INT_MAX;
  unsigned sse;
  const int thismse =
      (int)(c->search_type ? sp_upsampled(c, row, col, &sse) : sp_svf(c, row, col, &sse));
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

/* one SUBPEL_TREE level with the bilinear error (USE_2_TAPS_ORIG):
 * first_level_check_fast (mcomp.c:2566-2606) around the current best, then
 * with iters_per_step > 1 and a moved best second_level_check_v2
 * (:2728-2779): the row / column bias points away from the diagonal step when
 * the diagonal did not win, and the diagonal bias point only if one of them
 * improved */
static void sp_tree_level(const SpCtx *c, int hstep, int iters, SpBest *b) {
  const int tr = b->row, tc = b->col;
  const unsigned left = sp_check(c, tr, tc - hstep, b);
  const unsigned right = sp_check(c, tr, tc + hstep, b);
  const unsigned up = sp_check(c, tr - hstep, tc, b);
  const unsigned down = sp_check(c, tr + hstep, tc, b);
  int dr = up <= down ? -hstep : hstep, dc = left <= right ? -hstep : hstep;
  sp_check(c, tr + dr, tc + dc, b);
  if (iters <= 1) return;
  const int br = b->row, bc = b->col;
  if (br == tr && bc == tc) return;
  if (tr == br) dr = -dr;
  else if (tc == bc) dc = -dc;
  const unsigned before = b->besterr;
  sp_check(c, br + dr, bc, b);
  sp_check(c, br, bc + dc, b);
  if (b->besterr != before) sp_check(c, br + dr, bc + dc, b);
}

static int div_round(int n, int d) { /* divide_and_round, mcomp.c:2853-2855 */
  return ((n < 0) ^ (d < 0)) ? ((n - d / 2) / d) : ((n + d / 2) / d);
}

/* forced_stop: 0 EIGHTH_PEL, 1 QUARTER_PEL, 2 HALF_PEL, 3 FULL_PEL;
 * method 0 SUBPEL_TREE (bilinear error, USE_2_TAPS_ORIG), 1 SUBPEL_TREE_PRUNED,
 * 2 SUBPEL_TREE_PRUNED_MORE; cl NULL or the
 * full-pel cost list */
static void sp_search(const SpCtx *c, int method, int forced_stop, int allow_hp, int iters,
                      const int32_t *cl, OrcSubpelResult *out) {
  SpBest b;
  const int sr = c->jb->start_row, sc = c->jb->start_col;
  b.row = sr;
  b.col = sc;
  /* setup_center_error: vf at the (full-pel) start */
  unsigned sse;
  const uint8_t *r = c->ref + c->jb->ref_off + (ptrdiff_t)(b.row >> 3) * c->rs + (b.col >> 3);
  const unsigned v = orc_variance(r, c->rs, c->src + c->jb->src_off, c->ss, c->w, c->h, &sse);
  b.distortion = (int)v;
  b.sse1 = sse;
  b.besterr = v + (unsigned)sp_mv_cost(c, b.row, b.col);
  if (method == 0) { /* av1_find_best_sub_pixel_tree (mcomp.c:3128-3194), no repeat list */
    const int round = (3 - forced_stop) < (3 - !allow_hp) ? 3 - forced_stop : 3 - !allow_hp;
    int hstep = 4;
    for (int it = 0; it < round; ++it, hstep >>= 1) sp_tree_level(c, hstep, iters, &b);
  } else if (forced_stop != 3) {
    int hstep = 4; /* INIT_SUBPEL_STEP_SIZE */
    const int cl_ok = cl && cl[0] != INT_MAX && cl[1] != INT_MAX && cl[2] != INT_MAX &&
                      cl[3] != INT_MAX && cl[4] != INT_MAX;
    if (method == 2 && cl_ok && cl[0] < cl[1] && cl[0] < cl[2] && cl[0] < cl[3] &&
        cl[0] < cl[4]) {
      /* get_cost_surf_min(bits 1), one check at the modelled minimum */
      const int ic = div_round(cl[1] - cl[3], cl[1] - 2 * cl[0] + cl[3]);
      const int ir = div_round(cl[4] - cl[2], cl[4] - 2 * cl[0] + cl[2]);
      if (ir != 0 || ic != 0) sp_check(c, sr + ir * hstep, sc + ic * hstep, &b);
    } else if (method == 1 && cl_ok) {
      /* whichdir: the quadrant of the cheaper full-pel neighbours */
      const int dc = cl[1] < cl[3] ? -hstep : hstep; /* left : right */
      const int dr = cl[2] < cl[4] ? hstep : -hstep; /* bottom : top */
      sp_check(c, sr, sc + dc, &b);
      sp_check(c, sr + dr, sc, &b);
      sp_check(c, sr + dr, sc + dc, &b);
    } else {
      sp_two_level(c, sr, sc, hstep, iters, &b);
    }
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
  const int32_t *cls;
  int method, forced_stop, allow_hp, iters;
  long lo, hi;
} SpArg;

static void *sp_worker(void *v) {
  SpArg *a = (SpArg *)v;
  for (long j = a->lo; j < a->hi; ++j) {
    SpCtx c = a->base;
    c.jb = &a->jobs[j];
    sp_search(&c, a->method, a->forced_stop, a->allow_hp, a->iters,
              a->cls ? a->cls + 5 * j : NULL, &a->out[j]);
  }
  return NULL;
}

void orc_subpel_search_batch_ex(const uint8_t *src, int src_stride, const uint8_t *ref,
                                int ref_stride, int w, int h, const OrcSubpelJob *jobs,
                                long njobs, int subpel_method, int subpel_search_type,
                                int forced_stop, int allow_hp, int iters_per_step,
                                const OrcMvCost *cost, const int32_t *cost_lists,
                                OrcSubpelResult *out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  /* only SUBPEL_TREE takes the upsampled error (the pruned searches use
   * check_better_fast, which for an unscaled reference is the svf) */
  const int st = subpel_method == 0 ? subpel_search_type : 0;
  pthread_t tid[64];
  SpArg args[64];
  for (int t = 0; t < threads; ++t) {
    args[t].base =
        (SpCtx){ src, ref, src_stride, ref_stride, w, h, cost->mv_cost_type, NULL, cost, st };
    args[t].jobs = jobs;
    args[t].out = out;
    args[t].cls = cost_lists;
    args[t].method = subpel_method;
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

void orc_subpel_search_batch(const uint8_t *src, int src_stride, const uint8_t *ref,
                             int ref_stride, int w, int h, const OrcSubpelJob *jobs, long njobs,
                             int subpel_method, int forced_stop, int allow_hp,
                             int iters_per_step, const OrcMvCost *cost,
                             const int32_t *cost_lists, OrcSubpelResult *out, int threads) {
  orc_subpel_search_batch_ex(src, src_stride, ref, ref_stride, w, h, jobs, njobs, subpel_method,
                             0, forced_stop, allow_hp, iters_per_step, cost, cost_lists, out,
                             threads);
}

void orc_subpel_batch(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride,
                      int w, int h, const OrcSubpelJob *jobs, long njobs, int forced_stop,
                      int allow_hp, int iters_per_step, int mv_cost_type, OrcSubpelResult *out,
                      int threads) {
  const OrcMvCost c = { mv_cost_type, 0, 0, NULL, { NULL, NULL } };
  orc_subpel_search_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, 2, forced_stop,
                          allow_hp, iters_per_step, &c, NULL, out, threads);
}
