/* oracle_costcoeffs.c -- CPU restatement of the coefficient rate
 * (TEST INFRASTRUCTURE: only tests/, smoke() and bench.py's cpu_baseline use
 * it, as the checker).
 *
 * av1_cost_coeffs_txb (av1/encoder/txb_rdopt.c:599-624) and
 * av1_cost_coeffs_txb_laplacian with adjust_eob = 0 (:626-660), in the
 * reference's own order: levels (av1_txb_init_levels_c, encodetxb.c:238-254),
 * the scan-ordered context pass (av1_get_nz_map_contexts_c, :256-267), then
 * warehouse_efficients_txb (txb_rdopt.c:451-536) walking the scan from the
 * last coefficient down to DC.  Context helpers follow av1/common/
 * txb_common.h:50-272, the eob token encodetxb.c:100-131, the eob / Golomb /
 * base-range costs av1/encoder/txb_rdopt_utils.h:70-104.
 *
 * av1_nz_map_ctx_offset (av1/common/txb_common.c:18-360) is not copied: it is
 * regenerated from the algorithm its users state (txb_common.h:199-209);
 * tests/golden/fix_costcoeffs.npz (the reference function executed) pins the
 * result for every tx size.
 */
#include <stdlib.h>

#include "oracle.h"

#define PAD_HOR 4
#define COST_SHIFT 9 /* AV1_PROB_COST_SHIFT */

static const int k_eob_group_start[12] = {0, 1, 2, 3, 5, 9, 17, 33, 65, 129, 257, 513};
static const int k_eob_offset_bits[12] = {0, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9};
static const int k_cost_lut[15] = {-1143, 53, 545, 825, 1031, 1209, 1393, 1577,
                                   1763, 1947, 2132, 2317, 2501, 2686, 2871};

static int lg2(int v) {
  int r = 0;
  while ((1 << (r + 1)) <= v) ++r;
  return r;
}

/* tx_type_to_class (txb_common.h:31-48): 0 2D, 1 horizontal, 2 vertical */
static int tx_class_of(int tx_type) {
  if (tx_type < 10) return 0;
  return (tx_type & 1) ? 1 : 2;
}

/* av1_get_eob_pos_token (encodetxb.c:117-131) */
static int eob_pos_token(int eob, int *extra) {
  int t = 0;
  while (t < 11 && k_eob_group_start[t + 1] <= eob) ++t;
  *extra = eob - k_eob_group_start[t];
  return t;
}

/* the av1_nz_map_ctx_offset entry at raster coefficient (col, row) of a
 * W x H transform (txb_common.h:199-209); entry 0 is never read */
static int nz_map_offset(int w, int h, int col, int row) {
  if (w < h) {
    if (row < 2) return 11;
  } else if (w > h) {
    if (col < 2) return 16;
  }
  if (row + col < 2) return 1;
  if (row + col < 4) return 6;
  return 21;
}

static int min3(int v) { return v < 3 ? v : 3; }

typedef struct {
  int w, h, bhl, stride, cls, txw, txh;
  const uint8_t *lv;
} Txb;

/* get_nz_mag + get_nz_map_ctx_from_stats (txb_common.h:150-224) */
static int lower_levels_ctx(const Txb *t, int pos) {
  const int col = pos >> t->bhl, row = pos - (col << t->bhl);
  const uint8_t *l = t->lv + col * t->stride + row;
  const int s = t->stride;
  int mag = min3(l[s]) + min3(l[1]);
  if (t->cls == 0)
    mag += min3(l[s + 1]) + min3(l[2 * s]) + min3(l[2]);
  else if (t->cls == 2)
    mag += min3(l[2]) + min3(l[3]) + min3(l[4]);
  else
    mag += min3(l[2 * s]) + min3(l[3 * s]) + min3(l[4 * s]);
  if (t->cls == 0 && pos == 0) return 0;
  int ctx = (mag + 1) >> 1;
  if (ctx > 4) ctx = 4;
  if (t->cls == 0) return ctx + nz_map_offset(t->txw, t->txh, col, row);
  const int idx = t->cls == 1 ? col : row; /* nz_map_ctx_offset_1d */
  return ctx + 26 + (idx == 0 ? 0 : (idx == 1 ? 5 : 10));
}

/* get_br_ctx (txb_common.h:103-135) */
static int br_ctx(const Txb *t, int pos) {
  const int col = pos >> t->bhl, row = pos - (col << t->bhl);
  const uint8_t *l = t->lv + col * t->stride + row;
  const int s = t->stride;
  int mag = l[1] + l[s];
  int near;
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
  if (pos == 0) return mag;
  return near ? mag + 7 : mag + 14;
}

/* get_br_ctx_eob (txb_common.h:90-101) */
static int br_ctx_eob(const Txb *t, int pos) {
  const int col = pos >> t->bhl, row = pos - (col << t->bhl);
  if (pos == 0) return 0;
  if ((t->cls == 0 && row < 2 && col < 2) || (t->cls == 1 && col == 0) ||
      (t->cls == 2 && row == 0))
    return 7;
  return 14;
}

/* get_br_cost + get_golomb_cost (txb_rdopt_utils.h:86-104) */
static int br_cost(int level, const int32_t *lps) {
  int base_range = level - 3;
  if (base_range > 12) base_range = 12;
  int cost = lps[base_range];
  if (level >= 15) {
    const int r = level - 14;
    cost += (2 * (lg2(r) + 1) - 1) << COST_SHIFT;
  }
  return cost;
}

int orc_cost_coeffs_txb(const OrcCoeffCosts *cc, const int32_t *qcoeff, int eob, int plane,
                        int tx_size, int tx_type, int txb_skip_ctx, int dc_sign_ctx,
                        int tx_type_cost, int laplacian) {
  const int txw = orc_tx_w(tx_size), txh = orc_tx_h(tx_size);
  const int w = txw > 32 ? 32 : txw, h = txh > 32 ? 32 : txh;
  const int mn = txw < txh ? txw : txh, mx = txw < txh ? txh : txw;
  const int txs_ctx = (lg2(mn) - 2 + lg2(mx) - 2 + 1) >> 1; /* get_txsize_entropy_ctx */
  const int plane_type = plane > 0;
  const OrcCoeffCost *c = &cc->coeff_costs[txs_ctx][plane_type];
  if (eob == 0) return c->txb_skip_cost[txb_skip_ctx][1];
  const int eob_multi_size = lg2(w * h) - 4; /* txsize_log2_minus4 */
  const OrcEobCost *ec = &cc->eob_costs[eob_multi_size][plane_type];
  const int cls = tx_class_of(tx_type);
  const int16_t *scan = orc_scan(tx_size, tx_type);

  int cost = c->txb_skip_cost[txb_skip_ctx][0] + (plane ? 0 : tx_type_cost);
  /* get_eob_cost (txb_rdopt_utils.h:70-84) */
  {
    int extra;
    const int pt = eob_pos_token(eob, &extra);
    cost += ec->eob_cost[cls == 0 ? 0 : 1][pt - 1];
    const int bits = k_eob_offset_bits[pt];
    if (bits > 0) {
      const int bit = (extra >> (bits - 1)) & 1;
      cost += c->eob_extra_cost[pt - 3][bit];
      if (bits > 1) cost += (bits - 1) << COST_SHIFT;
    }
  }

  if (laplacian) { /* av1_cost_coeffs_txb_estimate (txb_rdopt.c:538-569) */
    cost += (abs(qcoeff[scan[eob - 1]]) - 1) << (COST_SHIFT + 2);
    for (int i = eob - 2; i >= 0; --i) {
      int v = abs(qcoeff[scan[i]]);
      cost += k_cost_lut[v < 14 ? v : 14];
    }
    const int loge_par = ((14427 << COST_SHIFT) + 5000) / 10000;
    return cost + ((1 << COST_SHIFT) + loge_par) * (eob - 1);
  }

  /* levels: |qcoeff| clamped to 127, padded columns (av1_txb_init_levels) */
  const int stride = h + PAD_HOR;
  uint8_t *lv = calloc((size_t)(w + PAD_HOR) * stride + 16, 1);
  for (int col = 0; col < w; ++col)
    for (int row = 0; row < h; ++row) {
      int a = abs(qcoeff[col * h + row]);
      lv[col * stride + row] = (uint8_t)(a > 127 ? 127 : a);
    }
  Txb t = {w, h, lg2(h), stride, cls, txw, txh, lv};
  int8_t ctxs[1024];
  for (int i = 0; i < eob; ++i) { /* av1_get_nz_map_contexts_c */
    const int pos = scan[i];
    if (i == eob - 1)
      ctxs[pos] = i == 0 ? 0 : (i <= (w * h) / 8 ? 1 : (i <= (w * h) / 4 ? 2 : 3));
    else
      ctxs[pos] = (int8_t)lower_levels_ctx(&t, pos);
  }
  for (int i = eob - 1; i >= 0; --i) {
    const int pos = scan[i];
    const int v = qcoeff[pos];
    const int level = abs(v);
    const int ml = level < 3 ? level : 3;
    if (i == eob - 1) {
      cost += c->base_eob_cost[ctxs[pos]][ml - 1];
      if (level > 2) cost += br_cost(level, c->lps_cost[br_ctx_eob(&t, pos)]);
    } else {
      cost += c->base_cost[ctxs[pos]][ml];
      if (level > 2) cost += br_cost(level, c->lps_cost[br_ctx(&t, pos)]);
    }
    if (level) cost += i ? 1 << COST_SHIFT : c->dc_sign_cost[dc_sign_ctx][v < 0];
  }
  free(lv);
  return cost;
}

void orc_cost_coeffs_txb_batch(const OrcCoeffCosts *cc, const int32_t *qcoeff, int n_stride,
                               const uint16_t *eob, int nblocks, int plane, int tx_size,
                               int tx_type, const int32_t *txb_ctx, int tx_type_cost,
                               int laplacian, int32_t *rate) {
  for (int b = 0; b < nblocks; ++b)
    rate[b] = orc_cost_coeffs_txb(cc, qcoeff + (size_t)b * n_stride, eob[b], plane, tx_size,
                                  tx_type, txb_ctx ? txb_ctx[2 * b] : 0,
                                  txb_ctx ? txb_ctx[2 * b + 1] : 0, tx_type_cost, laplacian);
}
