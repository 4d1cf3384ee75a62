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
