/*
 * oracle_quant.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates, from the reference:
 *   av1_quantize_fp_no_qmatrix / quantize_fp_helper_c (qm == NULL path)
 *                               av1/encoder/av1_quantize.c:36-122
 *   highbd_quantize_fp_helper_c av1/encoder/av1_quantize.c:125-198
 *   aom_quantize_b_helper_c     aom_dsp/quantize.c:108-169
 *   aom_highbd_quantize_b_helper_c aom_dsp/quantize.c:261-320
 *   invert_quant / get_qzbin_factor / av1_build_quantizer (incl. the fork's
 *   quant_sharpness)            av1/encoder/av1_quantize.c:580-686
 *   av1_dc_quant_QTX / av1_ac_quant_QTX  av1/common/quant_common.c:193-215
 *   av1_scan_orders             av1/common/scan.c (generated, see orc_scan)
 * The qlookup tables are the AV1 specification's Dc_Qlookup / Ac_Qlookup
 * (identical to quant_common.c:19-160; checked by tests/test_oracle_golden.py).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "qlookup_tables.h"

#define ROUND_POW2(v, n) (((v) + (((1 << (n)) >> 1))) >> (n))

int16_t orc_dc_quant(int qindex, int delta, int bd) {
  int q = qindex + delta;
  q = q < 0 ? 0 : (q > 255 ? 255 : q);
  return bd == 8 ? kDcQ8[q] : (bd == 10 ? kDcQ10[q] : kDcQ12[q]);
}

int16_t orc_ac_quant(int qindex, int delta, int bd) {
  int q = qindex + delta;
  q = q < 0 ? 0 : (q > 255 ? 255 : q);
  return bd == 8 ? kAcQ8[q] : (bd == 10 ? kAcQ10[q] : kAcQ12[q]);
}

static void invert_quant(int16_t *quant, int16_t *shift, int d) {
  uint32_t t = (uint32_t)d;
  int l = 0;
  while (t > 1) {
    t >>= 1;
    ++l;
  }
  const int m = 1 + (1 << (16 + l)) / d;
  *quant = (int16_t)(m - (1 << 16));
  *shift = (int16_t)(1 << (16 - l));
}

void orc_build_quant(int bd, int q, int sharpness, int y_dc_delta_q,
                     OrcQuant *o) {
  const int dc8 = orc_dc_quant(q, 0, bd);
  const int thr = bd == 8 ? 148 : (bd == 10 ? 592 : 2368);
  int zf = q == 0 ? 64 : (dc8 < thr ? 84 : 80);
  int rf = q == 0 ? 64 : 48;
  int adj = 16 * (7 - sharpness) / 7;
  if (sharpness > 0 && q > 0) {
    zf = 64 + adj;
    rf = 64 - adj;
  } else if (sharpness < 0 && q > 0) {
    adj = 16 * (7 + sharpness) / 7;
    zf = 64 + adj;
    rf = 64 - adj;
  }
  int rf_fp = 64;
  if (sharpness > 0) rf_fp = 64 - adj;
  if (sharpness < 0) rf_fp = 64 - adj;
  for (int i = 0; i < 2; ++i) {
    const int qv = i == 0 ? orc_dc_quant(q, y_dc_delta_q, bd)
                          : orc_ac_quant(q, 0, bd);
    invert_quant(&o->quant[i], &o->quant_shift[i], qv);
    o->quant_fp[i] = (int16_t)((1 << 16) / qv);
    o->round_fp[i] = (int16_t)((rf_fp * qv) >> 7);
    o->zbin[i] = (int16_t)ROUND_POW2(zf * qv, 7);
    o->round[i] = (int16_t)((rf * qv) >> 7);
    o->dequant[i] = (int16_t)qv;
  }
}

/* ---- quantizers ---- */
void orc_quantize_fp(const int32_t *coeff, intptr_t n, const int16_t *zbin,
                     const int16_t *round, const int16_t *quant,
                     const int16_t *quant_shift, int32_t *qcoeff,
                     int32_t *dqcoeff, const int16_t *dequant, uint16_t *eob,
                     const int16_t *scan, const int16_t *iscan,
                     int log_scale) {
  (void)zbin;
  (void)quant_shift;
  (void)iscan;
  memset(qcoeff, 0, n * sizeof(*qcoeff));
  memset(dqcoeff, 0, n * sizeof(*dqcoeff));
  const int rnd[2] = { ROUND_POW2(round[0], log_scale),
                       ROUND_POW2(round[1], log_scale) };
  int last = 0;
  for (intptr_t i = 0; i < n; ++i) {
    const int rc = scan[i];
    const int ac = rc != 0;
    const int c = coeff[rc];
    const int sgn = c < 0 ? -1 : 0;
    int64_t a = (c ^ sgn) - sgn;
    int q = 0;
    if ((a << (1 + log_scale)) >= (int32_t)dequant[ac]) {
      a += rnd[ac];
      if (a > INT16_MAX) a = INT16_MAX;
      if (a < INT16_MIN) a = INT16_MIN;
      q = (int)((a * quant[ac]) >> (16 - log_scale));
      if (q) {
        qcoeff[rc] = (q ^ sgn) - sgn;
        const int32_t dq = (q * dequant[ac]) >> log_scale;
        dqcoeff[rc] = (dq ^ sgn) - sgn;
      }
    }
    if (q) last = (int)i + 1;
  }
  *eob = (uint16_t)last;
}

void orc_highbd_quantize_fp(const int32_t *coeff, intptr_t n,
                            const int16_t *zbin, const int16_t *round,
                            const int16_t *quant, const int16_t *quant_shift,
                            int32_t *qcoeff, int32_t *dqcoeff,
                            const int16_t *dequant, uint16_t *eob,
                            const int16_t *scan, const int16_t *iscan,
                            int log_scale) {
  (void)zbin;
  (void)quant_shift;
  (void)iscan;
  const int shift = 16 - log_scale;
  const int rnd[2] = { ROUND_POW2(round[0], log_scale),
                       ROUND_POW2(round[1], log_scale) };
  int last = -1;
  for (intptr_t i = 0; i < n; ++i) {
    const int rc = scan[i];
    const int ac = rc != 0;
    const int c = coeff[rc];
    const int sgn = c < 0 ? -1 : 0;
    const int a = (c ^ sgn) - sgn;
    if ((a << (1 + log_scale)) >= dequant[ac]) {
      const int64_t t = (int64_t)a + rnd[ac];
      const int aq = (int)((t * quant[ac]) >> shift);
      qcoeff[rc] = (aq ^ sgn) - sgn;
      const int32_t adq = (aq * dequant[ac]) >> log_scale;
      if (aq) last = (int)i;
      dqcoeff[rc] = (adq ^ sgn) - sgn;
    } else {
      qcoeff[rc] = 0;
      dqcoeff[rc] = 0;
    }
  }
  *eob = (uint16_t)(last + 1);
}

void orc_quantize_b(const int32_t *coeff, intptr_t n, const int16_t *zbin,
                    const int16_t *round, const int16_t *quant,
                    const int16_t *quant_shift, int32_t *qcoeff,
                    int32_t *dqcoeff, const int16_t *dequant, uint16_t *eob,
                    const int16_t *scan, const int16_t *iscan, int log_scale) {
  (void)iscan;
  const int zb[2] = { ROUND_POW2(zbin[0], log_scale),
                      ROUND_POW2(zbin[1], log_scale) };
  memset(qcoeff, 0, n * sizeof(*qcoeff));
  memset(dqcoeff, 0, n * sizeof(*dqcoeff));
  /* pre-scan from the end: trailing coefficients strictly inside the zbin are
   * skipped (aom_dsp/quantize.c:126-137); qm weight is 1<<5 */
  int nzc = (int)n;
  for (int i = (int)n - 1; i >= 0; --i) {
    const int rc = scan[i];
    const int c = coeff[rc] * 32;
    if (c < zb[rc != 0] * 32 && c > -zb[rc != 0] * 32)
      --nzc;
    else
      break;
  }
  int last = -1;
  for (int i = 0; i < nzc; ++i) {
    const int rc = scan[i];
    const int ac = rc != 0;
    const int c = coeff[rc];
    const int sgn = c < 0 ? -1 : 0;
    const int a = (c ^ sgn) - sgn;
    if (a * 32 >= (zb[ac] << 5)) {
      int t = a + ROUND_POW2(round[ac], log_scale);
      t = t < INT16_MIN ? INT16_MIN : (t > INT16_MAX ? INT16_MAX : t);
      const int64_t tw = (int64_t)t * 32;
      const int q =
          (int)(((((tw * quant[ac]) >> 16) + tw) * quant_shift[ac]) >>
                (16 - log_scale + 5));
      qcoeff[rc] = (q ^ sgn) - sgn;
      const int dqv = (dequant[ac] * 32 + 16) >> 5;
      const int32_t adq = (q * dqv) >> log_scale;
      dqcoeff[rc] = (adq ^ sgn) - sgn;
      if (q) last = i;
    }
  }
  *eob = (uint16_t)(last + 1);
}

void orc_highbd_quantize_b(const int32_t *coeff, intptr_t n,
                           const int16_t *zbin, const int16_t *round,
                           const int16_t *quant, const int16_t *quant_shift,
                           int32_t *qcoeff, int32_t *dqcoeff,
                           const int16_t *dequant, uint16_t *eob,
                           const int16_t *scan, const int16_t *iscan,
                           int log_scale) {
  (void)iscan;
  const int zb[2] = { ROUND_POW2(zbin[0], log_scale),
                      ROUND_POW2(zbin[1], log_scale) };
  memset(qcoeff, 0, n * sizeof(*qcoeff));
  memset(dqcoeff, 0, n * sizeof(*dqcoeff));
  int last = -1;
  for (intptr_t i = 0; i < n; ++i) {
    const int rc = scan[i];
    const int ac = rc != 0;
    const int cw = coeff[rc] * 32;
    if (!(cw >= zb[ac] * 32 || cw <= -zb[ac] * 32)) continue;
    const int c = coeff[rc];
    const int sgn = c < 0 ? -1 : 0;
    const int a = (c ^ sgn) - sgn;
    const int64_t t1 = a + ROUND_POW2(round[ac], log_scale);
    const int64_t tw = t1 * 32;
    const int64_t t2 = ((tw * quant[ac]) >> 16) + tw;
    const int q = (int)((t2 * quant_shift[ac]) >> (16 - log_scale + 5));
    qcoeff[rc] = (q ^ sgn) - sgn;
    const int dqv = (dequant[ac] * 32 + 16) >> 5;
    const int32_t adq = (q * dqv) >> log_scale;
    dqcoeff[rc] = (adq ^ sgn) - sgn;
    if (q) last = (int)i;
  }
  *eob = (uint16_t)(last + 1);
}

/* ---- scans ----
 * The coefficient buffer is column-major (rc = col * H + row).  mcol is the
 * identity, mrow walks rows, default walks anti-diagonals: square sizes
 * zig-zag (odd diagonals from high col to low), tall sizes always high col to
 * low, wide sizes always low col to high.  64-point sizes reuse the 32-point
 * scans of their kept quadrant.  The generated orders are compared with every
 * table in av1/common/scan.c by tests/test_oracle_golden.py. */
static int16_t *g_scan[ORC_TX_SIZES_ALL][3];
static int16_t *g_iscan[ORC_TX_SIZES_ALL][3];

static void gen_scan(int W, int H, int kind, int16_t *s) {
  int k = 0;
  if (kind == 1) { /* mcol */
    for (int i = 0; i < W * H; ++i) s[i] = (int16_t)i;
    return;
  }
  if (kind == 2) { /* mrow */
    for (int i = 0; i < W * H; ++i) s[i] = (int16_t)((i % W) * H + i / W);
    return;
  }
  for (int d = 0; d < W + H - 1; ++d) {
    int hi_to_lo;
    if (W == H)
      hi_to_lo = d & 1;
    else
      hi_to_lo = W < H;
    const int cmin = d - (H - 1) > 0 ? d - (H - 1) : 0;
    const int cmax = d < W - 1 ? d : W - 1;
    if (hi_to_lo) {
      for (int c = cmax; c >= cmin; --c) s[k++] = (int16_t)(c * H + (d - c));
    } else {
      for (int c = cmin; c <= cmax; ++c) s[k++] = (int16_t)(c * H + (d - c));
    }
  }
}

static int scan_kind(int tx_type) {
  /* av1/common/scan.c av1_scan_orders: types 0-9 default; V_* use mrow,
   * H_* use mcol */
  if (tx_type < 10) return 0;
  return (tx_type & 1) ? 1 : 2; /* 10 V_DCT->mrow, 11 H_DCT->mcol, ... */
}

static void ensure_scan(int s, int kind) {
  if (g_scan[s][kind]) return;
  int W = orc_tx_w(s), H = orc_tx_h(s);
  if (W > 32) W = 32;
  if (H > 32) H = 32;
  int16_t *sc = (int16_t *)malloc(sizeof(int16_t) * W * H);
  int16_t *is = (int16_t *)malloc(sizeof(int16_t) * W * H);
  gen_scan(W, H, kind, sc);
  for (int i = 0; i < W * H; ++i) is[sc[i]] = (int16_t)i;
  g_iscan[s][kind] = is;
  g_scan[s][kind] = sc;
}

const int16_t *orc_scan(int s, int t) {
  const int k = scan_kind(t);
  ensure_scan(s, k);
  return g_scan[s][k];
}

const int16_t *orc_iscan(int s, int t) {
  const int k = scan_kind(t);
  ensure_scan(s, k);
  return g_iscan[s][k];
}
