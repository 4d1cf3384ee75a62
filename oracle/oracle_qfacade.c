/* oracle_qfacade.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of av1_quant's quantizer selection:
 *   av1_quant (av1/encoder/encodemb.c:308-341) with quant_func_list
 *   (:262-273): the fp / b / dc facades (av1/encoder/av1_quantize.c:266-420,
 *   423-563) without quantization matrices, quantize_dc (:374-405),
 *   highbd_quantize_dc (:516-545);
 *   skip_trellis_opt_based_on_satd (av1/encoder/tx_search.c:1923-1955) and
 *   the initial selection of search_tx_type (:2140-2145).
 */
#include <limits.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static const int kSqrtPx[19] = { 4, 8, 16, 32, 32, 6, 6, 12, 12, 23, 23, 32, 32, 8, 8, 16, 16, 23, 23 };
static const int kTxW[19] = { 4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64 };
static const int kTxH[19] = { 4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16 };

static int max_eob(int s) {
  if (s == 17 || s == 18) return 512;
  if (kTxW[s] == 64 || kTxH[s] == 64) return 1024;
  return kTxW[s] * kTxH[s];
}

static void quant_dc(const int32_t *c, int n, const OrcQuant *q, int ls, int hbd, int32_t *qc,
                     int32_t *dq, uint16_t *eob) {
  memset(qc, 0, sizeof(*qc) * n);
  memset(dq, 0, sizeof(*dq) * n);
  const int coeff = c[0];
  const int sign = coeff < 0 ? -1 : 0;
  const int ac = (coeff ^ sign) - sign;
  int64_t tmp = ac + ((q->round[0] + ((1 << ls) >> 1)) >> ls);
  if (!hbd) tmp = tmp < INT16_MIN ? INT16_MIN : (tmp > INT16_MAX ? INT16_MAX : tmp);
  const int32_t aq = (int32_t)((tmp * q->quant_fp[0]) >> (16 - ls));
  qc[0] = (aq ^ sign) - sign;
  const int32_t adq = (int32_t)((uint32_t)aq * (uint32_t)q->dequant[0]) >> ls;
  dq[0] = (adq ^ sign) - sign;
  *eob = aq ? 1 : 0;
}

int orc_av1_quant_block(const int32_t *coeff, int tx_size, int tx_type, int bd,
                        const OrcQuant *q, int mode, int skip_trellis, unsigned threshold,
                        int qstep, int dc_only, int32_t *qcoeff, int32_t *dqcoeff,
                        uint16_t *eob) {
  const int n = max_eob(tx_size);
  const int ls = (kTxW[tx_size] * kTxH[tx_size] > 256) + (kTxW[tx_size] * kTxH[tx_size] > 1024);
  const int hbd = bd > 8;
  int kind = mode, optb = 0;
  if (mode == 4) {
    if (skip_trellis || threshold == UINT_MAX) {
      kind = skip_trellis ? 1 : 0;
      optb = !skip_trellis;
    } else {
      int satd = 0;
      if (dc_only) {
        satd = abs(coeff[0]);
      } else {
        for (int i = 0; i < n; ++i) satd += abs(coeff[i]);
      }
      const int shift = 1 - ls; /* MAX_TX_SCALE - tx_scale */
      satd = shift < 0 ? satd << -shift : satd >> shift;
      satd >>= bd - 8;
      const int skip = (uint64_t)satd > (uint64_t)threshold * qstep * kSqrtPx[tx_size];
      kind = skip ? 1 : 0;
      optb = !skip;
    }
  }
  if (kind == 3) return optb | (kind << 1);
  const int16_t *scan = orc_scan(tx_size, tx_type), *iscan = orc_iscan(tx_size, tx_type);
  if (kind == 2) {
    quant_dc(coeff, n, q, ls, hbd, qcoeff, dqcoeff, eob);
  } else if (kind == 0) {
    (hbd ? orc_highbd_quantize_fp : orc_quantize_fp)(coeff, n, q->zbin, q->round_fp, q->quant_fp,
                                                     q->quant_shift, qcoeff, dqcoeff, q->dequant,
                                                     eob, scan, iscan, ls);
  } else {
    (hbd ? orc_highbd_quantize_b : orc_quantize_b)(coeff, n, q->zbin, q->round, q->quant,
                                                   q->quant_shift, qcoeff, dqcoeff, q->dequant,
                                                   eob, scan, iscan, ls);
  }
  return optb | (kind << 1);
}
