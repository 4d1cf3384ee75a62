/*
 * oracle_pipeline.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the C2 hot loop: the body of
 * search_tx_type's per-type loop (av1/encoder/tx_search.c:2148-2312) reduced
 * to av1_xform -> av1_quant (encodemb.c:295-341) for every full block of a
 * residual plane and every requested TX type.  Quantizer selection follows
 * av1_quantize_fp_facade / av1_quantize_b_facade (av1/encoder/av1_quantize.c:
 * 266-330): log_scale = av1_get_tx_scale(tx_size), n = av1_get_max_eob.
 * Used for parity checks and, multi-threaded, as bench.py's cpu_baseline.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  const int16_t *res;
  int stride, width, height, tx_size, bd, quant_b, row0, row1, ntypes;
  int types[16];
  const OrcQuant *q;
  int32_t *qcoeff, *dqcoeff;
  uint16_t *eob;
} Job;

static void *run_rows(void *arg) {
  Job *j = (Job *)arg;
  const int W = orc_tx_w(j->tx_size), H = orc_tx_h(j->tx_size);
  const int bw = j->width / W;
  const int n = orc_max_eob(j->tx_size);
  const int ls = orc_tx_scale(j->tx_size);
  int32_t *coeff = (int32_t *)malloc(sizeof(int32_t) * 64 * 64);
  for (int by = j->row0; by < j->row1; ++by) {
    for (int bx = 0; bx < bw; ++bx) {
      const int16_t *src = j->res + (size_t)by * H * j->stride + bx * W;
      const long blk = (long)by * bw + bx;
      for (int ti = 0; ti < j->ntypes; ++ti) {
        const int t = j->types[ti];
        const long slot = blk * j->ntypes + ti;
        orc_fwd_txfm2d(src, coeff, j->stride, t, j->tx_size, j->bd);
        int32_t *qc = j->qcoeff + slot * n;
        int32_t *dq = j->dqcoeff + slot * n;
        const int16_t *sc = orc_scan(j->tx_size, t);
        const int16_t *isc = orc_iscan(j->tx_size, t);
        if (j->bd == 8) {
          (j->quant_b ? orc_quantize_b : orc_quantize_fp)(
              coeff, n, j->q->zbin, j->quant_b ? j->q->round : j->q->round_fp,
              j->quant_b ? j->q->quant : j->q->quant_fp, j->q->quant_shift, qc,
              dq, j->q->dequant, j->eob + slot, sc, isc, ls);
        } else {
          (j->quant_b ? orc_highbd_quantize_b : orc_highbd_quantize_fp)(
              coeff, n, j->q->zbin, j->quant_b ? j->q->round : j->q->round_fp,
              j->quant_b ? j->q->quant : j->q->quant_fp, j->q->quant_shift, qc,
              dq, j->q->dequant, j->eob + slot, sc, isc, ls);
        }
      }
    }
  }
  free(coeff);
  return NULL;
}

long orc_txq_plane(const int16_t *residual, int stride, int width, int height,
                   int tx_size, unsigned type_mask, int bd, const OrcQuant *q,
                   int quant_b, int32_t *qcoeff, int32_t *dqcoeff,
                   uint16_t *eob, int threads) {
  const int W = orc_tx_w(tx_size), H = orc_tx_h(tx_size);
  const int bh = height / H, bw = width / W;
  Job base;
  memset(&base, 0, sizeof(base));
  base.res = residual;
  base.stride = stride;
  base.width = width;
  base.height = height;
  base.tx_size = tx_size;
  base.bd = bd;
  base.quant_b = quant_b;
  base.q = q;
  base.qcoeff = qcoeff;
  base.dqcoeff = dqcoeff;
  base.eob = eob;
  for (int t = 0; t < 16; ++t)
    if ((type_mask >> t) & 1) base.types[base.ntypes++] = t;
  /* warm the lazily-built tables before threads start */
  for (int t = 0; t < base.ntypes; ++t) {
    orc_scan(tx_size, base.types[t]);
    orc_iscan(tx_size, base.types[t]);
  }
  orc_cospi(10, 0);
  if (threads < 1) threads = 1;
  if (threads > bh) threads = bh > 0 ? bh : 1;
  pthread_t tid[256];
  Job jobs[256];
  if (threads > 256) threads = 256;
  for (int i = 0; i < threads; ++i) {
    jobs[i] = base;
    jobs[i].row0 = (int)((long)bh * i / threads);
    jobs[i].row1 = (int)((long)bh * (i + 1) / threads);
    if (threads == 1)
      run_rows(&jobs[i]);
    else
      pthread_create(&tid[i], NULL, run_rows, &jobs[i]);
  }
  if (threads > 1)
    for (int i = 0; i < threads; ++i) pthread_join(tid[i], NULL);
  return (long)bh * bw;
}
