/* oracle_mcomp.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the full-pixel motion search of the reference:
 *   av1_init_dsmotion_compensation     av1/encoder/mcomp.c:369-404 (level 0)
 *   av1_init_motion_compensation_bigdia av1/encoder/mcomp.c:498-550
 *   av1_init_motion_compensation_nstep  av1/encoder/mcomp.c:450-494 (NSTEP, NSTEP_8PT)
 *   av1_init_motion_compensation_square av1/encoder/mcomp.c:552-604
 *   av1_init_motion_compensation_hex    av1/encoder/mcomp.c:606-653 (HEX, FAST_HEX)
 *   mv_cost / mv_err_cost / mvsad_err_cost (entropy, L1, none)
 *                                      av1/encoder/mcomp.c:255-360
 *   av1_get_mv_joint                   av1/encoder/encodemv.h:49-55
 *   diamond_search_sad                 av1/encoder/mcomp.c:1318-1477
 *   full_pixel_diamond                 av1/encoder/mcomp.c:1479-1526
 *   pattern_search (BIGDIA / HEX / SQUARE do_init_search 1, FAST_BIGDIA /
 *   FAST_DIAMOND / VFAST_DIAMOND / FAST_HEX 0, cost lists)
 *                                      av1/encoder/mcomp.c:858-1245,1258-1316
 *   calc_int_sad_list                  av1/encoder/mcomp.c:789-838
 *   av1_full_pixel_search: method switch, downsampled-SAD quality recheck
 *                                      av1/encoder/mcomp.c:1755-1873
 * with sdf/sdx4df = aom_sad / aom_sad_skip and vf = aom_variance of the
 * block size (oracle_dsp.c), and the mesh refinement:
 *   exhaustive_mesh_search             av1/encoder/mcomp.c:1529-1601
 *   full_pixel_exhaustive              av1/encoder/mcomp.c:1603-1680
 *   av1_full_pixel_search mesh tail    av1/encoder/mcomp.c:1818-1838,1875-1893
 * Pinned by tests/golden/fix_mcomp*.npz, made by executing the reference's
 * own av1_full_pixel_search.
 */
#include <limits.h>
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

/* mv_cost (mcomp.c:268-272) of a 1/8-pel diff */
static int mv_rate(const OrcMvCost *c, int dr, int dc) {
  const int joint = (dc != 0) | ((dr != 0) << 1);
  return c->mvjcost[joint] + c->mvcost[0][dr] + c->mvcost[1][dc];
}

static unsigned mvsad_cost(const OrcMsParams *p, int row, int col) {
  const int dr = (row - rawpel(p->ref_mv_row)) * 8;
  const int dc = (col - rawpel(p->ref_mv_col)) * 8;
  if (p->mv_cost_type == 0) /* ROUND_POWER_OF_TWO(unsigned, AV1_PROB_COST_SHIFT) */
    return ((unsigned)mv_rate(p->cost, dr, dc) * (unsigned)p->cost->sad_per_bit + 256u) >> 9;
  if (p->mv_cost_type < 1 || p->mv_cost_type > 3) return 0;
  return (unsigned)((sad_lambda(p->mv_cost_type) * (abs(dr) + abs(dc))) >> 3);
}

static int mv_cost(const OrcMsParams *p, int row, int col) {
  const int dr = row * 8 - p->ref_mv_row, dc = col * 8 - p->ref_mv_col;
  if (p->mv_cost_type == 0) /* ROUND_POWER_OF_TWO_64(., 7 + 9 - 6 + 4) */
    return (int)(((int64_t)mv_rate(p->cost, dr, dc) * p->cost->error_per_bit + 8192) >> 14);
  if (p->mv_cost_type < 1 || p->mv_cost_type > 3) return 0;
  return (sse_lambda(p->mv_cost_type) * (abs(dr) + abs(dc))) >> 3;
}

static int in_range(const OrcMsParams *p, int row, int col) {
  return col >= p->col_min && col <= p->col_max && row >= p->row_min &&
         row <= p->row_max;
}

static int bounds_ok(const OrcMsParams *p, int row, int col, int r) {
  return row - r >= p->row_min && row + r <= p->row_max && col - r >= p->col_min &&
         col + r <= p->col_max;
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

/* calc_int_sad_list (mcomp.c:789-838): neighbours left, bottom, right, top */
static void int_sad_list(const OrcMsParams *p, int br, int bc, int skip, int *cl,
                         int has_sad) {
  static const int nr[4] = { 0, 1, 0, -1 }, nc[4] = { -1, 0, 1, 0 };
  if (!has_sad) {
    cl[0] = (int)block_sad(p, br, bc, skip);
    const int all = bounds_ok(p, br, bc, 1);
    for (int i = 0; i < 4; ++i) {
      if (!all && !in_range(p, br + nr[i], bc + nc[i]))
        cl[i + 1] = INT_MAX;
      else
        cl[i + 1] = (int)block_sad(p, br + nr[i], bc + nc[i], skip);
    }
  }
  cl[0] += (int)mvsad_cost(p, br, bc);
  for (int i = 0; i < 4; ++i)
    if (cl[i + 1] != INT_MAX) cl[i + 1] += (int)mvsad_cost(p, br + nr[i], bc + nc[i]);
}

/* a diamond_search_sad site configuration: per step its radius and search
 * points (site 0 = the centre), num_search_steps */
typedef struct {
  int nsteps;
  int radius[16], npts[16];
  int dr[16][13], dc[16][13];
} DiaCfg;

/* av1_init_dsmotion_compensation (level 0): 11 steps, radius 2^step, the
 * 8 points (-r,0) (r,0) (0,-r) (0,r) (-r,-r) (r,r) (-r,r) (r,-r) */
static void dia_cfg_ds(DiaCfg *c) {
  static const int kDr[9] = { 0, -1, 1, 0, 0, -1, 1, -1, 1 };
  static const int kDc[9] = { 0, 0, 0, -1, 1, -1, 1, 1, -1 };
  c->nsteps = MAX_STEPS;
  for (int st = 0; st < MAX_STEPS; ++st) {
    const int r = 1 << st;
    c->radius[st] = r;
    c->npts[st] = 8;
    for (int i = 0; i <= 8; ++i) {
      c->dr[st][i] = kDr[i] * r;
      c->dc[st][i] = kDc[i] * r;
    }
  }
}

/* av1_init_motion_compensation_nstep (mcomp.c:452-494): level 0 (NSTEP) 15
 * stages, 12 points at radius > 5 with tan_radius = max((int)(0.41 r), 1);
 * level 1 (NSTEP_8PT) 16 stages of 8 points; the radius grows to
 * max((int)(1.5 r + 0.5), r + 1) after each of the first 12 stages */
static void dia_cfg_nstep(DiaCfg *c, int level) {
  c->nsteps = level > 0 ? 16 : 15;
  int radius = 1;
  for (int st = 0; st < c->nsteps; ++st) {
    int tan = (int)(0.41 * radius);
    if (tan < 1) tan = 1;
    int n = 12;
    if (radius <= 5 || level > 0) {
      tan = radius;
      n = 8;
    }
    const int r = radius, t = tan;
    const int mr[13] = { 0, -r, r, 0, 0, -r, r, -t, t, -r, r, t, -t };
    const int mc[13] = { 0, 0, 0, -r, r, -t, t, r, -r, t, -t, r, -r };
    for (int i = 0; i <= n; ++i) {
      c->dr[st][i] = mr[i];
      c->dc[st][i] = mc[i];
    }
    c->npts[st] = n;
    c->radius[st] = radius;
    if (st < 12) {
      const int g = (int)(radius * 1.5 + 0.5);
      radius = g > radius + 1 ? g : radius + 1;
    }
  }
}

/* diamond_search_sad without second_pred / mask: returns bestsad, writes
 * the best mv and num00 (center steps).  *steps counts evaluated steps. */
static unsigned diamond(const OrcMsParams *p, const DiaCfg *cfg, int srow, int scol,
                        int search_step, int skip, int *brow, int *bcol, int *num00, int *steps) {
  if (scol < p->col_min) scol = p->col_min;
  if (scol > p->col_max) scol = p->col_max;
  if (srow < p->row_min) srow = p->row_min;
  if (srow > p->row_max) srow = p->row_max;
  int row = srow, col = scol, off_center = 0, center_steps = 0;
  unsigned best = mvsad_cost(p, row, col) + block_sad(p, row, col, skip);
  const int tot = cfg->nsteps - search_step;
  for (int step = tot - 1; step >= 0; --step) {
    const int rad = cfg->radius[step];
    int best_site = 0;
    /* all_in: sites 1..4 (the axis points at the radius) in range */
    const int all_in = bounds_ok(p, row, col, rad);
    for (int i = 1; i <= cfg->npts[step]; ++i) {
      const int r = row + cfg->dr[step][i], c = col + cfg->dc[step][i];
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
    /* UPDATE_SEARCH_STEP (mcomp.c:1322-1342) */
    if (best_site) {
      row += cfg->dr[step][best_site];
      col += cfg->dc[step][best_site];
      off_center = 1;
    }
    if (!off_center) ++center_steps;
    if (best_site == 0 && step > 2) {  /* steps of an equal radius below are skipped */
      int next = cfg->radius[step - 1];
      while (next == cfg->radius[step] && step > 2) {
        ++center_steps;
        --step;
        next = cfg->radius[step - 1];
      }
    }
  }
  *brow = row;
  *bcol = col;
  *num00 = center_steps;
  return best;
}

static int full_pixel_diamond(const OrcMsParams *p, const DiaCfg *cfg, int srow, int scol,
                              int step_param, int skip, int *cl, int *brow, int *bcol,
                              int *steps) {
  int n, num00 = 0;
  diamond(p, cfg, srow, scol, step_param, skip, brow, bcol, &n, steps);
  int bestsme = var_cost(p, *brow, *bcol);
  const int further = cfg->nsteps - 1 - step_param;
  while (n < further) {
    ++n;
    int tr, tc;
    diamond(p, cfg, srow, scol, step_param + n, skip, &tr, &tc, &num00, steps);
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
  if (cl) int_sad_list(p, *brow, *bcol, skip, cl, 0);
  return bestsme;
}

/* ---- pattern_search (mcomp.c:1017-1245) over the BIGDIA, SQUARE and HEX
 * sites (kind 0 / 1 / 2) ---- */
enum { PAT_BIGDIA = 0, PAT_SQUARE = 1, PAT_HEX = 2 };
#if defined(__GNUC__)
#define ORC_TLS __thread
#else
#define ORC_TLS
#endif
static ORC_TLS int t_kind;
static void bigdia_site(int s, int i, int *dr, int *dc) {
  /* BIGDIA: scale 0 the 4 nearest, scale s >= 1 8 points of r = 2^(s-1) / 2r */
  static const int k0r[4] = { 0, 1, 0, -1 }, k0c[4] = { -1, 0, 1, 0 };
  static const int kr[8] = { -1, 0, 1, 2, 1, 0, -1, -2 }, kc[8] = { -1, -2, -1, 0, 1, 2, 1, 0 };
  /* SQUARE (and HEX scale 0): 8 points of r = 2^s */
  static const int sr[8] = { -1, 0, 1, 1, 1, 0, -1, -1 }, sc[8] = { -1, -1, -1, 0, 1, 1, 1, 0 };
  /* HEX scale s >= 1: 6 points (-r,-2r) (r,-2r) (2r,0) (r,2r) (-r,2r) (-2r,0), r = 2^(s-1) */
  static const int hr[6] = { -1, 1, 2, 1, -1, -2 }, hc[6] = { -2, -2, 0, 2, 2, 0 };
  if (t_kind == PAT_SQUARE || (t_kind == PAT_HEX && s == 0)) {
    *dr = sr[i] << s;
    *dc = sc[i] << s;
  } else if (t_kind == PAT_HEX) {
    *dr = hr[i] << (s - 1);
    *dc = hc[i] << (s - 1);
  } else if (s == 0) {
    *dr = k0r[i];
    *dc = k0c[i];
  } else {
    const int r = 1 << (s - 1);
    *dr = kr[i] * r;
    *dc = kc[i] * r;
  }
}
static int ncand(int s) {
  return t_kind == PAT_BIGDIA ? (s == 0 ? 4 : 8) : t_kind == PAT_HEX ? (s == 0 ? 8 : 6) : 8;
}

typedef struct {
  const OrcMsParams *p;
  int skip;
  unsigned best, raw_best;
  int *cl;
  int *steps;
} PState;

/* update_mvs_and_sad (mcomp.c:858-877) */
static int upd(PState *st, unsigned thissad, int r, int c) {
  if (thissad >= st->best) return 0;
  const unsigned sad = thissad + mvsad_cost(st->p, r, c);
  if (sad < st->best) {
    st->raw_best = thissad;
    st->best = sad;
    return 1;
  }
  return 0;
}

/* calc_sad4 / calc_sad_update_bestmv over candidates [0, n) of scale s
 * around (br, bc); cost list entries get the raw SADs (sad4: all four; the
 * bounds-checked form: in-range ones only).  Returns the best site or -1.
 * With every candidate in bounds the reference runs calc_sad4 over the
 * groups of four and then calc_sad_update_bestmv(num_candidates =
 * n % 4, cand_start = n & ~3), whose loop (i = cand_start; i <
 * num_candidates) never runs: HEX's 6-point scales evaluate only their first
 * four candidates (mcomp.c:1064-1077,1108-1122,964). */
static int scan_all(PState *st, int s, int br, int bc, int *cl) {
  const OrcMsParams *p = st->p;
  int best_site = -1;
  const int all = bounds_ok(p, br, bc, 1 << s);
  const int n = all ? (ncand(s) & ~3) : ncand(s);
  for (int i = 0; i < n; ++i) {
    int dr, dc;
    bigdia_site(s, i, &dr, &dc);
    if (!all && !in_range(p, br + dr, bc + dc)) continue;
    const unsigned sad = block_sad(p, br + dr, bc + dc, st->skip);
    if (cl) cl[i + 1] = (int)sad;
    if (upd(st, sad, br + dr, bc + dc)) best_site = i;
  }
  ++*st->steps;
  return best_site;
}

/* calc_sad3_update_bestmv / _with_indices: returns j of idx[j] or -1 */
static int scan3(PState *st, int s, int br, int bc, const int *idx, int *cl) {
  const OrcMsParams *p = st->p;
  int best_site = -1;
  const int all = bounds_ok(p, br, bc, 1 << s);
  for (int j = 0; j < 3; ++j) {
    int dr, dc;
    bigdia_site(s, idx[j], &dr, &dc);
    if (!all && !in_range(p, br + dr, bc + dc)) {
      if (cl) cl[idx[j] + 1] = INT_MAX;
      continue;
    }
    const unsigned sad = block_sad(p, br + dr, bc + dc, st->skip);
    if (cl) cl[idx[j] + 1] = (int)sad;
    if (upd(st, sad, br + dr, bc + dc)) best_site = j;
  }
  ++*st->steps;
  return best_site;
}

static void next3(int k, int n, int *idx) {
  idx[0] = (k == 0) ? n - 1 : k - 1;
  idx[1] = k;
  idx[2] = (k == n - 1) ? 0 : k + 1;
}

static int pattern_search(const OrcMsParams *p, int kind, int srow, int scol, int search_step,
                          int do_init, int skip, int *cl, int *brow, int *bcol, int *steps) {
  PState st = { p, skip, UINT_MAX, UINT_MAX, cl, steps };
  t_kind = kind;
  if (search_step > MAX_STEPS - 1) search_step = MAX_STEPS - 1;
  int best_init_s = MAX_STEPS - 1 - search_step; /* search_steps[search_step] */
  if (scol < p->col_min) scol = p->col_min;
  if (scol > p->col_max) scol = p->col_max;
  if (srow < p->row_min) srow = p->row_min;
  if (srow > p->row_max) srow = p->row_max;
  int br = srow, bc = scol, k = -1, s;
  if (cl) cl[0] = cl[1] = cl[2] = cl[3] = cl[4] = INT_MAX;
  int costlist_has_sad = 0;
  st.raw_best = block_sad(p, br, bc, skip);
  st.best = st.raw_best + mvsad_cost(p, br, bc);
  if (do_init) {
    s = best_init_s;
    best_init_s = -1;
    for (int t = 0; t <= s; ++t) { /* every scale around the fixed start */
      const int bs = scan_all(&st, t, br, bc, NULL);
      if (bs == -1) continue;
      best_init_s = t;
      k = bs;
    }
    if (best_init_s != -1) {
      int dr, dc;
      bigdia_site(best_init_s, k, &dr, &dc);
      br += dr;
      bc += dc;
    }
  }
  if (best_init_s != -1) {
    /* last_is_4 && cost_list: num_candidates[0] == 4 only for BIGDIA */
    const int last_s = kind == PAT_BIGDIA && cl != NULL;
    int best_site = -1;
    s = best_init_s;
    for (; s >= last_s; s--) {
      if (!do_init || s != best_init_s) {
        best_site = scan_all(&st, s, br, bc, NULL);
        if (best_site == -1) continue;
        int dr, dc;
        bigdia_site(s, best_site, &dr, &dc);
        br += dr;
        bc += dc;
        k = best_site;
      }
      do {
        int idx[3];
        next3(k, ncand(s), idx);
        best_site = scan3(&st, s, br, bc, idx, NULL);
        if (best_site != -1) {
          k = idx[best_site];
          int dr, dc;
          bigdia_site(s, k, &dr, &dc);
          br += dr;
          bc += dc;
        }
      } while (best_site != -1);
    }
    if (s == 0) { /* only BIGDIA with a cost list (last_s == 1) */
      cl[0] = (int)st.raw_best;
      costlist_has_sad = 1;
      if (!do_init || s != best_init_s) {
        best_site = scan_all(&st, 0, br, bc, cl);
        if (best_site != -1) {
          int dr, dc;
          bigdia_site(0, best_site, &dr, &dc);
          br += dr;
          bc += dc;
          k = best_site;
        }
      }
      while (best_site != -1) {
        int idx[3];
        next3(k, 4, idx);
        cl[1] = cl[2] = cl[3] = cl[4] = INT_MAX;
        cl[((k + 2) % 4) + 1] = cl[0];
        cl[0] = (int)st.raw_best;
        best_site = scan3(&st, 0, br, bc, idx, cl);
        if (best_site != -1) {
          k = idx[best_site];
          int dr, dc;
          bigdia_site(0, k, &dr, &dc);
          br += dr;
          bc += dc;
        }
      }
    }
  }
  *brow = br;
  *bcol = bc;
  if (cl) int_sad_list(p, br, bc, skip, cl, costlist_has_sad);
  return var_cost(p, br, bc); /* get_mvpred_var_cost */
}

/* exhaustive_mesh_search (mcomp.c:1529-1601): every (step)-th row and column
 * (column step 4 when step is 1, then 4 positions per call; the last partial
 * group of a row stops one short of end_col) within range of the clamped
 * start, sequential strict-< update of sad + mvsad_err_cost; returns best_sad */
static unsigned mesh_pass(const OrcMsParams *p, int srow, int scol, int range, int step,
                          int skip, int *brow, int *bcol) {
  const int col_step = step > 1 ? step : 4;
  srow = srow < p->row_min ? p->row_min : srow > p->row_max ? p->row_max : srow;
  scol = scol < p->col_min ? p->col_min : scol > p->col_max ? p->col_max : scol;
  *brow = srow;
  *bcol = scol;
  unsigned best = block_sad(p, srow, scol, skip) + mvsad_cost(p, srow, scol);
  const int r0 = -range > p->row_min - srow ? -range : p->row_min - srow;
  const int c0 = -range > p->col_min - scol ? -range : p->col_min - scol;
  const int r1 = range < p->row_max - srow ? range : p->row_max - srow;
  const int c1 = range < p->col_max - scol ? range : p->col_max - scol;
  for (int r = r0; r <= r1; r += step) {
    for (int c = c0; c <= c1; c += col_step) {
      const int n = step > 1 ? 1 : (c + 3 <= c1 ? 4 : c1 - c);
      for (int i = 0; i < n; ++i) {
        const int row = srow + r, col = scol + c + i;
        const unsigned sad = block_sad(p, row, col, skip);
        if (sad >= best) continue; /* update_mvs_and_sad, mcomp.c:858-877 */
        const unsigned cost = sad + mvsad_cost(p, row, col);
        if (cost < best) {
          best = cost;
          *brow = row;
          *bcol = col;
        }
      }
    }
  }
  return best;
}

static int ilog2i(int v) {
  int l = 0;
  while ((1 << (l + 1)) <= v) ++l;
  return l;
}

/* full_pixel_exhaustive (mcomp.c:1603-1680): INT_MAX for an illegal first
 * pattern (cost list untouched), else the var cost at the mesh's best and
 * the cost list around it */
static int mesh_exhaustive(const OrcMsParams *p, const OrcMeshParams *m, int srow, int scol,
                           int skip, int *cl, int *brow, int *bcol) {
  int interval = m->interval[0], range = m->range[0];
  *brow = srow;
  *bcol = scol;
  if (range < 7 || range > 256 || interval < 1 || interval > range) return INT_MAX;
  const int div = range / interval;
  const int mag = abs(srow) > abs(scol) ? abs(srow) : abs(scol);
  if (5 * mag / 4 > range) range = 5 * mag / 4;
  if (range > 256) range = 256;
  if (range / div > interval) interval = range / div;
  if (m->fine_search_interval && interval > 4) interval = 4;
  mesh_pass(p, srow, scol, range, interval, skip, brow, bcol);
  if (interval > 1 && range > 7) {
    for (int i = 1; i < 4; ++i) {
      mesh_pass(p, *brow, *bcol, m->range[i], m->interval[i], skip, brow, bcol);
      if (m->interval[i] == 1) break;
    }
  }
  if (cl) int_sad_list(p, *brow, *bcol, skip, cl, 0);
  return var_cost(p, *brow, *bcol);
}

/* the mesh tail of av1_full_pixel_search (mcomp.c:1818-1838, 1875-1893):
 * forced after NSTEP / NSTEP_8PT when the variance passes force_mesh_thresh
 * scaled to the block, pruned when the search moved little */
static int mesh_tail(const OrcMsParams *p, const OrcMeshParams *m, int method, int start_row,
                     int start_col, int skip, int var, int *cl, int *best_row, int *best_col) {
  int run = m->run_mesh_search;
  if (!run && (method == ORC_NSTEP || method == ORC_NSTEP_8PT)) {
    const int thr = m->force_mesh_thresh >> (10 - (ilog2i(p->w >> 2) + ilog2i(p->h >> 2)));
    if (var > thr) run = 1;
  }
  if (!m->is_intra_mode && m->prune_mesh_search) {
    const int dr = abs(start_row - *best_row), dc = abs(start_col - *best_col);
    if ((dr > dc ? dr : dc) <= m->mesh_search_mv_diff_threshold) run = 0;
  }
  if (!run) return var;
  int tr, tc;
  const int var_ex = mesh_exhaustive(p, m, *best_row, *best_col, skip, cl, &tr, &tc);
  if (var_ex < var) {
    var = var_ex;
    *best_row = tr;
    *best_col = tc;
  }
  return var;
}

/* av1_full_pixel_search (mcomp.c:1755-1893); mesh NULL: no mesh refinement */
int orc_full_pixel_search_ex(const OrcMsParams *p, int method, int start_row, int start_col,
                             int step_param, int *cl, int *best_row, int *best_col, int *steps,
                             const OrcMeshParams *mesh) {
  /* use_downsampled_sad only for blocks >= 16 high (mcomp.c:132-133) */
  int skip = p->skip_sad && p->h >= 16;
  for (;;) {
    if (cl) cl[0] = cl[1] = cl[2] = cl[3] = cl[4] = INT_MAX;
    int var;
    if (method == ORC_DIAMOND || method == ORC_NSTEP || method == ORC_NSTEP_8PT) {
      DiaCfg cfg;
      if (method == ORC_DIAMOND) dia_cfg_ds(&cfg);
      else dia_cfg_nstep(&cfg, method == ORC_NSTEP_8PT);
      var = full_pixel_diamond(p, &cfg, start_row, start_col, step_param, skip, cl, best_row,
                               best_col, steps);
    } else {
      /* bigdia / hex / square_search: step_param, do_init 1; fast_dia /
       * vfast_dia / fast_bigdia / fast_hex: AOMMAX(MAX_MVSEARCH_STEPS - 2 /
       * 1 / 3 / 2, step_param), do_init 0 (mcomp.c:1258-1316) */
      const int floor = method == ORC_FAST_DIAMOND || method == ORC_FAST_HEX ? MAX_STEPS - 2
                        : method == ORC_VFAST_DIAMOND ? MAX_STEPS - 1
                        : MAX_STEPS - 3;
      const int init = method == ORC_BIGDIA || method == ORC_HEX || method == ORC_SQUARE;
      const int kind = method == ORC_HEX || method == ORC_FAST_HEX ? PAT_HEX
                       : method == ORC_SQUARE ? PAT_SQUARE : PAT_BIGDIA;
      const int ss = init ? step_param : (step_param > floor ? step_param : floor);
      var = pattern_search(p, kind, start_row, start_col, ss, init, skip, cl, best_row, best_col,
                           steps);
    }
    if (!skip)
      return mesh ? mesh_tail(p, mesh, method, start_row, start_col, skip, var, cl, best_row,
                              best_col)
                  : var;
    /* quality check of the row-skipping search (mcomp.c:1840-1867) */
    const uint8_t *r = p->ref + (ptrdiff_t)*best_row * p->ref_stride + *best_col;
    const int sad = (int)orc_sad(p->src, p->src_stride, r, p->ref_stride, p->w, p->h);
    const int ssad = (int)orc_sad_skip(p->src, p->src_stride, r, p->ref_stride, p->w, p->h);
    const int thresh = (p->w >> 2) * (p->h >> 2); /* 1 << (mi_w_log2 + mi_h_log2) */
    const int big = sad > 1 ? sad : 1;
    if (!(sad > thresh && abs(ssad - sad) * 10 >= big * 9))
      return mesh ? mesh_tail(p, mesh, method, start_row, start_col, skip, var, cl, best_row,
                              best_col)
                  : var;
    skip = 0; /* redo the whole search with the full SAD */
  }
}

int orc_full_pixel_search(const OrcMsParams *p, int method, int start_row, int start_col,
                          int step_param, int *cl, int *best_row, int *best_col, int *steps) {
  return orc_full_pixel_search_ex(p, method, start_row, start_col, step_param, cl, best_row,
                                  best_col, steps, NULL);
}

int orc_full_pixel_search_diamond(const OrcMsParams *p, int start_row, int start_col,
                                  int step_param, int *best_row, int *best_col, int *steps) {
  *steps = 0;
  return orc_full_pixel_search(p, ORC_DIAMOND, start_row, start_col, step_param, NULL, best_row,
                               best_col, steps);
}

int orc_full_pixel_search_bigdia(const OrcMsParams *p, int start_row, int start_col,
                                 int step_param, int *best_row, int *best_col, int *steps) {
  *steps = 0;
  return orc_full_pixel_search(p, ORC_FAST_BIGDIA, start_row, start_col, step_param, NULL,
                               best_row, best_col, steps);
}

/* ---- batch driver (pthreads over job ranges) ---- */
#include <pthread.h>

typedef struct {
  const uint8_t *src, *ref;
  int ss, rs, w, h, step_param, skip, method;
  const OrcMvCost *cost;
  const OrcMeshParams *mesh;
  const OrcDiamondJob *jobs;
  OrcDiamondResult *out;
  int32_t *cls;
  long lo, hi;
} BatchArg;

static void *batch_worker(void *v) {
  const BatchArg *a = (const BatchArg *)v;
  for (long j = a->lo; j < a->hi; ++j) {
    const OrcDiamondJob *jb = &a->jobs[j];
    OrcMsParams p = { a->src + jb->src_off, a->ss, a->ref + jb->ref_off, a->rs, a->w, a->h,
                      jb->col_min, jb->col_max, jb->row_min, jb->row_max, jb->ref_mv_row,
                      jb->ref_mv_col, a->cost->mv_cost_type, a->skip, a->cost };
    int br, bc, steps = 0;
    a->out[j].bestsme = orc_full_pixel_search_ex(&p, a->method, jb->start_row, jb->start_col,
                                                 a->step_param, a->cls ? a->cls + 5 * j : NULL,
                                                 &br, &bc, &steps, a->mesh);
    a->out[j].best_row = (int16_t)br;
    a->out[j].best_col = (int16_t)bc;
    a->out[j].steps = steps;
    a->out[j].reserved = 0;
  }
  return NULL;
}

void orc_full_pixel_search_batch_ex(const uint8_t *src, int src_stride, const uint8_t *ref,
                                    int ref_stride, int w, int h, const OrcDiamondJob *jobs,
                                    long njobs, int method, int step_param,
                                    const OrcMvCost *cost, int skip_sad, int32_t *cost_lists,
                                    OrcDiamondResult *out, int threads,
                                    const OrcMeshParams *mesh) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t tid[64];
  BatchArg args[64];
  for (int t = 0; t < threads; ++t) {
    args[t] = (BatchArg){ src, ref, src_stride, ref_stride, w, h, step_param, skip_sad, method,
                          cost, mesh, jobs, out, cost_lists, njobs * t / threads,
                          njobs * (t + 1) / threads };
    if (threads > 1) pthread_create(&tid[t], NULL, batch_worker, &args[t]);
    else batch_worker(&args[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}

void orc_full_pixel_search_batch(const uint8_t *src, int src_stride, const uint8_t *ref,
                                 int ref_stride, int w, int h, const OrcDiamondJob *jobs,
                                 long njobs, int method, int step_param, const OrcMvCost *cost,
                                 int skip_sad, int32_t *cost_lists, OrcDiamondResult *out,
                                 int threads) {
  orc_full_pixel_search_batch_ex(src, src_stride, ref, ref_stride, w, h, jobs, njobs, method,
                                 step_param, cost, skip_sad, cost_lists, out, threads, NULL);
}

void orc_diamond_batch(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride,
                       int w, int h, const OrcDiamondJob *jobs, long njobs, int step_param,
                       int mv_cost_type, int skip_sad, OrcDiamondResult *out, int threads) {
  const OrcMvCost c = { mv_cost_type, 0, 0, NULL, { NULL, NULL } };
  orc_full_pixel_search_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, ORC_DIAMOND,
                              step_param, &c, skip_sad, NULL, out, threads);
}

void orc_bigdia_batch(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride,
                      int w, int h, const OrcDiamondJob *jobs, long njobs, int step_param,
                      int mv_cost_type, int skip_sad, OrcDiamondResult *out, int threads) {
  const OrcMvCost c = { mv_cost_type, 0, 0, NULL, { NULL, NULL } };
  orc_full_pixel_search_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs,
                              ORC_FAST_BIGDIA, step_param, &c, skip_sad, NULL, out, threads);
}
