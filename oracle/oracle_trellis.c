/* oracle_trellis.c -- CPU restatement of the coefficient trellis
 * (TEST INFRASTRUCTURE: only tests/, smoke() and bench.py's cpu_baseline use
 * it, as the checker).
 *
 * av1_optimize_b (av1/encoder/encodemb.c:87-103) -> av1_optimize_txb
 * (av1/encoder/txb_rdopt.c:326-449), no quantization matrix (the default
 * PSNR metric: qmatrix NULL; a flat iqmatrix changes nothing), in the
 * reference's order: the last coefficient (update_coeff_general or the
 * eob-cost form), update_coeff_eob while at most 2 nonzeros are kept
 * (:128-244), update_skip (:246-262), update_coeff_simple down to scan index
 * 1 (:75-126), update_coeff_general at DC (:17-73); then the skip /
 * non-skip + tx-type cost and av1_get_txb_entropy_context (encodetxb.c:
 * 451-467).  Cost helpers: txb_rdopt_utils.h:39-194; contexts as
 * oracle_costcoeffs.c.  Pinned by tests/golden/fix_trellis.npz
 * (av1_optimize_b executed from the reference).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define PAD 4

static int lg2i(int v) {
  int r = 0;
  while ((1 << (r + 1)) <= v) ++r;
  return r;
}

static int clsof(int tx_type) { return tx_type < 10 ? 0 : ((tx_type & 1) ? 1 : 2); }
static int mn3(int v) { return v < 3 ? v : 3; }

typedef struct {
  const OrcCoeffCost *c;
  const OrcEobCost *e;
  int w, h, bhl, stride, cls, txw, txh, dc_sign_ctx, sharpness, shift;
  int64_t rdmult;
  uint8_t *lv;
} Tr;

/* RDCOST (av1/encoder/rd.h:31-33) */
static int64_t rdcost(int64_t rm, int64_t r, int64_t d) { return ((r * rm + 256) >> 9) + d * 128; }

/* get_coeff_dist, no qmatrix (txb_rdopt_utils.h:48-66) */
static int64_t cdist(int32_t t, int32_t d, int shift) {
  const int64_t diff = (int64_t)(int32_t)((t - d) * (1 << shift));
  return diff * diff;
}

static int nzoff(int w, int h, int col, int row) {
  if (w < h) {
    if (row < 2) return 11;
  } else if (w > h) {
    if (col < 2) return 16;
  }
  if (row + col < 2) return 1;
  if (row + col < 4) return 6;
  return 21;
}

/* get_lower_levels_ctx (txb_common.h:251-258) */
static int lower_ctx(const Tr *t, int ci) {
  const int col = ci >> t->bhl, row = ci - (col << t->bhl);
  const uint8_t *l = t->lv + col * t->stride + row;
  const int s = t->stride;
  int mag = mn3(l[s]) + mn3(l[1]);
  if (t->cls == 0) mag += mn3(l[s + 1]) + mn3(l[2 * s]) + mn3(l[2]);
  else if (t->cls == 2) mag += mn3(l[2]) + mn3(l[3]) + mn3(l[4]);
  else mag += mn3(l[2 * s]) + mn3(l[3 * s]) + mn3(l[4 * s]);
  if (t->cls == 0 && ci == 0) return 0;
  int ctx = (mag + 1) >> 1;
  if (ctx > 4) ctx = 4;
  if (t->cls == 0) return ctx + nzoff(t->txw, t->txh, col, row);
  const int idx = t->cls == 1 ? col : row;
  return ctx + 26 + (idx == 0 ? 0 : (idx == 1 ? 5 : 10));
}

/* get_lower_levels_ctx_eob (txb_common.h:229-234) */
static int eob_ctx(const Tr *t, int si) {
  const int n = t->w * t->h;
  if (si == 0) return 0;
  if (si <= n / 8) return 1;
  if (si <= n / 4) return 2;
  return 3;
}

static int br_ctx(const Tr *t, int ci) {
  const int col = ci >> t->bhl, row = ci - (col << t->bhl);
  const uint8_t *l = t->lv + col * t->stride + row;
  const int s = t->stride;
  int mag = l[1] + l[s], near;
  if (t->cls == 0) {
    mag += l[s + 1];
    near = row < 2 && col < 2;
  } else if (t->cls == 1) {
    mag += l[2 * s];
    near = col == 0;
  } else {
    mag += l[2];
    near = row == 0;
  }
  mag = (mag + 1) >> 1;
  if (mag > 6) mag = 6;
  if (ci == 0) return mag;
  return near ? mag + 7 : mag + 14;
}

static int br_ctx_eob(const Tr *t, int ci) {
  const int col = ci >> t->bhl, row = ci - (col << t->bhl);
  if (ci == 0) return 0;
  if ((t->cls == 0 && row < 2 && col < 2) || (t->cls == 1 && col == 0) ||
      (t->cls == 2 && row == 0))
    return 7;
  return 14;
}

static int golomb(int level) {
  if (level < 15) return 0;
  return (2 * (lg2i(level - 14) + 1) - 1) * 512;
}

static int br_cost(int level, const int32_t *lps) {
  int br = level - 3;
  if (br > 12) br = 12;
  return lps[br] + golomb(level);
}

/* get_br_cost_with_diff (txb_rdopt_utils.h:106-128) */
static int br_cost_diff(int level, const int32_t *lps, int *diff) {
  int br = level - 3;
  if (br > 12) br = 12;
  int bits = 0;
  if (level <= 15) *diff += lps[br + 13];
  if (level >= 15) {
    const int r = level - 14;
    bits = golomb(level);
    *diff += r == 1 ? 512 : ((r & (r - 1)) == 0 ? 1024 : 0);
  }
  return lps[br] + bits;
}

/* get_coeff_cost_eob / get_coeff_cost_general (txb_rdopt_utils.h:155-194) */
static int cost_eob(const Tr *t, int ci, int abs_qc, int sign, int ctx) {
  int cost = t->c->base_eob_cost[ctx][(abs_qc < 3 ? abs_qc : 3) - 1];
  if (abs_qc) {
    cost += ci == 0 ? t->c->dc_sign_cost[t->dc_sign_ctx][sign] : 512;
    if (abs_qc > 2) cost += br_cost(abs_qc, t->c->lps_cost[br_ctx_eob(t, ci)]);
  }
  return cost;
}

static int cost_general(const Tr *t, int is_last, int ci, int abs_qc, int sign, int ctx) {
  if (is_last) return cost_eob(t, ci, abs_qc, sign, ctx);
  int cost = t->c->base_cost[ctx][abs_qc < 3 ? abs_qc : 3];
  if (abs_qc) {
    cost += ci == 0 ? t->c->dc_sign_cost[t->dc_sign_ctx][sign] : 512;
    if (abs_qc > 2) cost += br_cost(abs_qc, t->c->lps_cost[br_ctx(t, ci)]);
  }
  return cost;
}

/* get_eob_cost (txb_rdopt_utils.h:70-84) */
static int eob_cost(const Tr *t, int eob) {
  static const int start[12] = {0, 1, 2, 3, 5, 9, 17, 33, 65, 129, 257, 513};
  int pt = 0;
  while (pt < 11 && start[pt + 1] <= eob) ++pt;
  const int extra = eob - start[pt];
  int cost = t->e->eob_cost[t->cls == 0 ? 0 : 1][pt - 1];
  const int bits = pt >= 3 ? pt - 2 : 0;
  if (bits > 0) {
    cost += t->c->eob_extra_cost[pt - 3][(extra >> (bits - 1)) & 1];
    if (bits > 1) cost += (bits - 1) * 512;
  }
  return cost;
}

static int dqv_of(const int16_t *dq, int ci) { return dq[ci != 0]; }

static void set_level(Tr *t, int ci, int v) {
  const int col = ci >> t->bhl, row = ci - (col << t->bhl);
  t->lv[col * t->stride + row] = (uint8_t)(v > 127 ? 127 : v);
}

/* update_coeff_general (txb_rdopt.c:17-73) */
static void upd_general(Tr *t, int *accu_rate, int64_t *accu_dist, int si, int eob,
                        const int16_t *scan, const int16_t *dq, const int32_t *tc, int32_t *qc,
                        int32_t *dqc) {
  const int ci = scan[si];
  const int dqv = dqv_of(dq, ci);
  const int32_t q = qc[ci];
  const int is_last = si == eob - 1;
  const int ctx = is_last ? eob_ctx(t, si) : lower_ctx(t, ci);
  if (q == 0) {
    *accu_rate += t->c->base_cost[ctx][0];
    return;
  }
  const int sign = q < 0;
  const int abs_qc = abs(q);
  const int64_t dist = cdist(tc[ci], dqc[ci], t->shift);
  const int64_t dist0 = cdist(tc[ci], 0, t->shift);
  const int rate = cost_general(t, is_last, ci, abs_qc, sign, ctx);
  const int64_t rd = rdcost(t->rdmult, rate, dist);
  int32_t qlow = 0, dqlow = 0;
  int abs_low = 0, rate_low;
  int64_t dist_low;
  if (abs_qc == 1) {
    dist_low = dist0;
    rate_low = t->c->base_cost[ctx][0];
  } else {
    abs_low = abs_qc - 1;
    const int32_t adq = (abs_low * dqv) >> t->shift;
    qlow = sign ? -abs_low : abs_low;
    dqlow = sign ? -adq : adq;
    dist_low = cdist(tc[ci], dqlow, t->shift);
    rate_low = cost_general(t, is_last, ci, abs_low, sign, ctx);
  }
  const int64_t rd_low = rdcost(t->rdmult, rate_low, dist_low);
  if (rd_low < rd) {
    qc[ci] = qlow;
    dqc[ci] = dqlow;
    set_level(t, ci, abs_low);
    *accu_rate += rate_low;
    *accu_dist += dist_low - dist0;
  } else {
    *accu_rate += rate;
    *accu_dist += dist - dist0;
  }
}

/* update_coeff_simple (txb_rdopt.c:75-126) */
static void upd_simple(Tr *t, int *accu_rate, int si, const int16_t *scan, const int16_t *dq,
                       const int32_t *tc, int32_t *qc, int32_t *dqc) {
  const int ci = scan[si];
  const int dqv = dqv_of(dq, ci);
  const int32_t q = qc[ci];
  const int ctx = lower_ctx(t, ci);
  if (q == 0) {
    *accu_rate += t->c->base_cost[ctx][0];
    return;
  }
  const int abs_qc = abs(q);
  const int32_t abs_tqc = abs(tc[ci]), abs_dqc = abs(dqc[ci]);
  /* get_two_coeff_cost_simple (txb_rdopt_utils.h:130-153) */
  int cost = t->c->base_cost[ctx][abs_qc < 3 ? abs_qc : 3];
  int diff = abs_qc <= 3 ? t->c->base_cost[ctx][abs_qc + 4] : 0;
  cost += 512;
  if (abs_qc > 2) {
    int bd = 0;
    cost += br_cost_diff(abs_qc, t->c->lps_cost[br_ctx(t, ci)], &bd);
    diff += bd;
  }
  const int rate_low = cost - diff;
  if (abs_dqc < abs_tqc) {
    *accu_rate += cost;
    return;
  }
  const int64_t dist = cdist(abs_tqc, abs_dqc, t->shift);
  const int64_t rd = rdcost(t->rdmult, cost, dist);
  const int abs_low = abs_qc - 1;
  const int32_t abs_dqlow = (abs_low * dqv) >> t->shift;
  const int64_t dist_low = cdist(abs_tqc, abs_dqlow, t->shift);
  const int64_t rd_low = rdcost(t->rdmult, rate_low, dist_low);
  if (rd_low < rd) {
    const int sign = q < 0;
    qc[ci] = sign ? -abs_low : abs_low;
    dqc[ci] = sign ? -abs_dqlow : abs_dqlow;
    set_level(t, ci, abs_low);
    *accu_rate += rate_low;
  } else {
    *accu_rate += cost;
  }
}

/* update_coeff_eob (txb_rdopt.c:128-244) */
static void upd_eob(Tr *t, int *accu_rate, int64_t *accu_dist, int *eob, int *nz_num, int *nz_ci,
                    int si, const int16_t *scan, const int16_t *dq, const int32_t *tc, int32_t *qc,
                    int32_t *dqc) {
  const int ci = scan[si];
  const int dqv = dqv_of(dq, ci);
  const int32_t q = qc[ci];
  const int ctx = lower_ctx(t, ci);
  if (q == 0) {
    *accu_rate += t->c->base_cost[ctx][0];
    return;
  }
  int lower = 0;
  const int abs_qc = abs(q);
  const int sign = q < 0;
  const int64_t dist0 = cdist(tc[ci], 0, t->shift);
  int64_t dist = cdist(tc[ci], dqc[ci], t->shift) - dist0;
  int rate = cost_general(t, 0, ci, abs_qc, sign, ctx);
  int64_t rd = rdcost(t->rdmult, *accu_rate + rate, *accu_dist + dist);
  int32_t qlow = 0, dqlow = 0;
  int abs_low = 0, rate_low;
  int64_t dist_low, rd_low;
  if (abs_qc == 1) {
    dist_low = 0;
    rate_low = t->c->base_cost[ctx][0];
    rd_low = rdcost(t->rdmult, *accu_rate + rate_low, *accu_dist);
  } else {
    abs_low = abs_qc - 1;
    const int32_t adq = (abs_low * dqv) >> t->shift;
    qlow = sign ? -abs_low : abs_low;
    dqlow = sign ? -adq : adq;
    dist_low = cdist(tc[ci], dqlow, t->shift) - dist0;
    rate_low = cost_general(t, 0, ci, abs_low, sign, ctx);
    rd_low = rdcost(t->rdmult, *accu_rate + rate_low, *accu_dist + dist_low);
  }
  int lower_new_eob = 0;
  const int new_eob = si + 1;
  const int ctx_new_eob = eob_ctx(t, si);
  const int new_eob_cost = eob_cost(t, new_eob);
  int rate_eob = new_eob_cost + cost_eob(t, ci, abs_qc, sign, ctx_new_eob);
  int64_t dist_new_eob = dist;
  int64_t rd_new_eob = rdcost(t->rdmult, rate_eob, dist_new_eob);
  if (abs_low > 0) {
    const int rate_eob_low = new_eob_cost + cost_eob(t, ci, abs_low, sign, ctx_new_eob);
    const int64_t rd_low_eob = rdcost(t->rdmult, rate_eob_low, dist_low);
    if (rd_low_eob < rd_new_eob) {
      lower_new_eob = 1;
      rd_new_eob = rd_low_eob;
      rate_eob = rate_eob_low;
      dist_new_eob = dist_low;
    }
  }
  if (t->sharpness == 0 || abs_qc > 1) {
    if (rd_low < rd) {
      lower = 1;
      rd = rd_low;
      rate = rate_low;
      dist = dist_low;
    }
  }
  if (t->sharpness == 0 && rd_new_eob < rd) {
    for (int i = 0; i < *nz_num; ++i) {
      const int lc = nz_ci[i];
      set_level(t, lc, 0);
      qc[lc] = 0;
      dqc[lc] = 0;
    }
    *eob = new_eob;
    *nz_num = 0;
    *accu_rate = rate_eob;
    *accu_dist = dist_new_eob;
    lower = lower_new_eob;
  } else {
    *accu_rate += rate;
    *accu_dist += dist;
  }
  if (lower) {
    qc[ci] = qlow;
    dqc[ci] = dqlow;
    set_level(t, ci, abs_low);
  }
  if (qc[ci]) nz_ci[(*nz_num)++] = ci;
}

int orc_optimize_b(const OrcCoeffCosts *cc, const int32_t *tcoeff, int32_t *qcoeff,
                   int32_t *dqcoeff, int eob, int plane, int tx_size, int tx_type, int bd,
                   int is_inter, int x_rdmult, int sharpness, const int16_t dequant[2],
                   int txb_skip_ctx, int dc_sign_ctx, int tx_type_cost, int *rate_cost,
                   uint8_t *entropy_ctx) {
  static const int plane_rd_mult[2][2] = {{17, 13}, {16, 10}}; /* encodetxb.h:266-269 */
  const int txw = orc_tx_w(tx_size), txh = orc_tx_h(tx_size);
  const int w = txw > 32 ? 32 : txw, h = txh > 32 ? 32 : txh;
  const int mn = txw < txh ? txw : txh, mx = txw < txh ? txh : txw;
  const int txs_ctx = (lg2i(mn) - 2 + lg2i(mx) - 2 + 1) >> 1;
  const int pt = plane > 0;
  Tr t;
  t.c = &cc->coeff_costs[txs_ctx][pt];
  t.e = &cc->eob_costs[lg2i(w * h) - 4][pt];
  t.w = w;
  t.h = h;
  t.bhl = lg2i(h);
  t.stride = h + PAD;
  t.cls = clsof(tx_type);
  t.txw = txw;
  t.txh = txh;
  t.dc_sign_ctx = dc_sign_ctx;
  t.sharpness = sharpness;
  t.shift = orc_tx_scale(tx_size);
  t.rdmult = (((int64_t)x_rdmult * (plane_rd_mult[is_inter][pt] << (2 * (bd - 8)))) + 2) >>
             (sharpness + 2);
  const int16_t *scan = orc_scan(tx_size, tx_type);
  const int skip_cost = t.c->txb_skip_cost[txb_skip_ctx][1];
  const int non_skip_cost = t.c->txb_skip_cost[txb_skip_ctx][0];
  if (eob == 0) { /* av1_optimize_b's early exit (av1_cost_skip_txb) */
    *rate_cost = skip_cost;
    *entropy_ctx = 0;
    return 0;
  }
  t.lv = calloc((size_t)(w + PAD) * t.stride + 16, 1);
  if (eob > 1)
    for (int col = 0; col < w; ++col)
      for (int row = 0; row < h; ++row) {
        const int a = abs(qcoeff[col * h + row]);
        t.lv[col * t.stride + row] = (uint8_t)(a > 127 ? 127 : a);
      }
  int accu_rate = eob_cost(&t, eob);
  int64_t accu_dist = 0;
  int si = eob - 1;
  const int ci = scan[si];
  const int32_t q = qcoeff[ci];
  const int abs_qc = abs(q);
  int nz_num = 1;
  int nz_ci[3] = {ci, 0, 0};
  if (abs_qc >= 2) {
    upd_general(&t, &accu_rate, &accu_dist, si, eob, scan, dequant, tcoeff, qcoeff, dqcoeff);
  } else {
    accu_rate += cost_eob(&t, ci, abs_qc, q < 0, eob_ctx(&t, si));
    accu_dist += cdist(tcoeff[ci], dqcoeff[ci], t.shift) - cdist(tcoeff[ci], 0, t.shift);
  }
  --si;
  for (; si >= 0 && nz_num <= 2; --si)
    upd_eob(&t, &accu_rate, &accu_dist, &eob, &nz_num, nz_ci, si, scan, dequant, tcoeff, qcoeff,
            dqcoeff);
  if (si == -1 && nz_num <= 2) { /* update_skip */
    const int64_t rd = rdcost(t.rdmult, accu_rate + non_skip_cost, accu_dist);
    const int64_t rd_skip = rdcost(t.rdmult, skip_cost, 0);
    if (rd_skip < rd && sharpness == 0) {
      for (int i = 0; i < nz_num; ++i) {
        qcoeff[nz_ci[i]] = 0;
        dqcoeff[nz_ci[i]] = 0;
      }
      accu_rate = 0;
      eob = 0;
    }
  }
  for (; si >= 1; --si) upd_simple(&t, &accu_rate, si, scan, dequant, tcoeff, qcoeff, dqcoeff);
  if (si == 0) {
    int64_t dummy = 0;
    upd_general(&t, &accu_rate, &dummy, si, eob, scan, dequant, tcoeff, qcoeff, dqcoeff);
  }
  accu_rate += eob == 0 ? skip_cost : non_skip_cost + (plane ? 0 : tx_type_cost);
  *rate_cost = accu_rate;
  /* av1_get_txb_entropy_context */
  int cul = 0;
  for (int c = 0; c < eob; ++c) {
    cul += abs(qcoeff[scan[c]]);
    if (cul > 7) break;
  }
  if (cul > 7) cul = 7;
  if (eob > 0) {
    if (qcoeff[0] < 0) cul |= 1 << 3;
    else if (qcoeff[0] > 0) cul += 2 << 3;
  }
  *entropy_ctx = (uint8_t)cul;
  free(t.lv);
  return eob;
}
