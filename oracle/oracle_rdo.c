/* oracle_rdo.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the C4 per-block TX-type RDO: for
 * every full tx_size block of (src - pred) and every requested type:
 *   aom_highbd_subtract_block      aom_dsp/subtract.c:38-54
 *   av1_fwd_txfm2d_*               av1/encoder/av1_fwd_txfm2d.c:56-312
 *   av1_highbd_quantize_fp         av1/encoder/av1_quantize.c:125-198,565-577
 *   aom_satd                       aom_dsp/avg.c:509-516
 *   av1_highbd_block_error         av1/encoder/rdopt.c:664-682
 *   dist_block_tx_domain shift     av1/encoder/tx_search.c:1077-1116
 *   rate_estimator                 av1/encoder/tpl_model.c:214-226
 *   RDCOST                         av1/encoder/rd.h:31-33
 * keeping the first type with the strictly lowest cost
 * (tx_search.c:2246 `if (rd < best_rd)`).
 *
 * Pixel-domain distortion (orc_rdo_plane_px; search_tx_type with
 * use_transform_domain_distortion == 0, predict_dc_level 0,
 * tx_search.c:2060-2103, 2187-2231):
 *   block_sse = ROUND_POWER_OF_TWO(sum_squares(residual), 2 (bd-8)) * 16
 *   eob == 0        -> dist = sse = block_sse
 *   otherwise       -> is_high_energy = block_sse >= 128*128*pels;
 *     TX_64X64 or high energy: tx-domain (dist_td, sse_td) as above and
 *       sse_diff = block_sse - sse_td;
 *     if (tx_size != TX_64X64 || !high || 2*sse_diff < sse_td):
 *       dist = dist_block_px_domain (tx_search.c:969-1017): recon = pred +
 *       av1_inverse_transform_block, 16 * vf-sse(src, recon) (highbd vf
 *       rounds the sse by 2 (bd-8) bits, variance.c:321-408); a high-energy
 *       block keeps dist_td when that is larger;
 *     else dist = dist_td + sse_diff;
 *     sse = block_sse.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int get_msb(unsigned n) { return 31 - __builtin_clz(n); }

/* RDCOST (av1/encoder/rd.h:31-33): ROUND_POWER_OF_TWO(rate * rdmult,
 * AV1_PROB_COST_SHIFT) + dist * (1 << RDDIV_BITS) */
static int64_t rdcost(int rdmult, int rate, int64_t dist) {
  return ((((int64_t)rate) * rdmult + 256) >> 9) + dist * 128;
}

/* search_tx_type's best-type update (tx_search.c:2243-2256): the first
 * candidate of strictly lowest RDCOST wins; rds[i] = each candidate's cost.
 * The per-block loop below uses the same two lines; pinned by
 * tests/golden/fix_rdselect.npz. */
int orc_rd_select(int rdmult, const int *rates, const int64_t *dists, int n, int64_t *rds) {
  int64_t best_rd = INT64_MAX;
  int best = -1;
  for (int i = 0; i < n; ++i) {
    const int64_t rd = rdcost(rdmult, rates[i], dists[i]);
    rds[i] = rd;
    if (rd < best_rd) {
      best_rd = rd;
      best = i;
    }
  }
  return best;
}

/* rate_estimator (tpl_model.c:214-226): DCT_DCT scan of tx_size */
static int rate_estimator(const int32_t *qcoeff, int eob, int tx_size) {
  const int16_t *scan = orc_scan(tx_size, 0);
  int rate_cost = 1;
  for (int idx = 0; idx < eob; ++idx) {
    const unsigned abs_level = (unsigned)abs(qcoeff[scan[idx]]);
    rate_cost += get_msb(abs_level + 1) + 1 + (abs_level > 0);
  }
  return rate_cost << 9; /* AV1_PROB_COST_SHIFT */
}

typedef struct {
  const uint16_t *src, *pred;
  int stride, width, tx_size, bd, rdmult, row0, row1, ntypes, px;
  int types[16];
  const uint16_t *block_mask; /* optional allowed_tx_mask per block */
  const uint8_t *block_map;   /* optional txk_map per block ([16]) */
  const OrcQuant *q;
  OrcRdoBlock *out;
  int32_t *qcoeff, *dqcoeff;
  /* optional: the coefficient rate (av1_cost_coeffs_txb) instead of
   * rate_estimator, with per-block TXB_CTX pairs and per-type tx-type costs */
  const OrcCoeffCosts *cc;
  const int32_t *txb_ctx;
  const int32_t *tx_type_costs;
} RdoJob;

static void *rdo_rows(void *arg) {
  RdoJob *j = (RdoJob *)arg;
  const int W = orc_tx_w(j->tx_size), H = orc_tx_h(j->tx_size);
  const int bw = j->width / W;
  const int n = orc_max_eob(j->tx_size);
  const int ls = orc_tx_scale(j->tx_size);
  const int shift = (1 - ls) * 2; /* (MAX_TX_SCALE - tx_scale) * 2 */
  int16_t diff[64 * 64];
  int32_t coeff[64 * 64], qc[4096], dq[4096];
  uint16_t rec[64 * 64];
  const int rsh = 2 * (j->bd - 8);
  for (int by = j->row0; by < j->row1; ++by) {
    for (int bx = 0; bx < bw; ++bx) {
      const long blk = (long)by * bw + bx;
      const size_t off = (size_t)by * H * j->stride + (size_t)bx * W;
      orc_highbd_subtract_block(H, W, diff, W, j->src + off, j->stride, j->pred + off,
                                j->stride);
      int64_t block_sse = 0;
      if (j->px) {
        uint64_t ss = 0;
        for (int i = 0; i < W * H; ++i) ss += (uint64_t)((int64_t)diff[i] * diff[i]);
        if (rsh) ss = (ss + ((uint64_t)1 << (rsh - 1))) >> rsh;
        block_sse = (int64_t)ss * 16;
      }
      OrcRdoBlock best;
      memset(&best, 0, sizeof(best));
      best.rdcost = INT64_MAX;
      /* search_tx_type's loop (tx_search.c:2148-2157): txk_map order,
       * skipping TX_TYPE_INVALID and types outside allowed_tx_mask
       * (get_tx_mask: a zero mask becomes DCT_DCT, tx_search.c:1885-1888);
       * only types of the call's type set are evaluated */
      unsigned inset = 0;
      for (int ti = 0; ti < j->ntypes; ++ti) inset |= 1u << j->types[ti];
      unsigned allowed = j->block_mask ? j->block_mask[blk] : 0xFFFFu;
      if (!allowed) allowed = 1;
      int seq[16], nseq = 0;
      for (int idx = 0; idx < 16; ++idx) {
        const int t = j->block_map ? j->block_map[blk * 16 + idx] : idx;
        if (t >= 16 || !((allowed >> t) & 1) || !((inset >> t) & 1)) continue;
        int dup = 0;
        for (int u = 0; u < nseq; ++u) dup |= seq[u] == t;
        if (!dup) seq[nseq++] = t;
      }
      for (int ti = 0; ti < nseq; ++ti) {
        const int t = seq[ti];
        orc_fwd_txfm2d(diff, coeff, W, t, j->tx_size, j->bd);
        uint16_t eob;
        orc_highbd_quantize_fp(coeff, n, j->q->zbin, j->q->round_fp, j->q->quant_fp,
                               j->q->quant_shift, qc, dq, j->q->dequant, &eob,
                               orc_scan(j->tx_size, t), orc_iscan(j->tx_size, t), ls);
        const int satd = orc_satd(coeff, n);
        int64_t ssz;
        int64_t err = orc_highbd_block_error(coeff, dq, n, &ssz, j->bd);
        /* RIGHT_SIGNED_SHIFT (aom_ports/mem.h:69-70) */
        int64_t dist = shift < 0 ? err << -shift : err >> shift;
        int64_t sse = shift < 0 ? ssz << -shift : ssz >> shift;
        if (j->px) {
          if (eob == 0) {
            dist = block_sse;
          } else {
            const int high = block_sse >= (int64_t)128 * 128 * W * H;
            const int is64 = j->tx_size == 4; /* TX_64X64 */
            const int64_t sse_diff = block_sse - sse;
            if (!is64 || !high || sse_diff * 2 < sse) {
              for (int r = 0; r < H; ++r)
                memcpy(rec + r * W, j->pred + off + (size_t)r * j->stride, 2 * W);
              orc_inv_txfm2d_add(dq, rec, W, t, j->tx_size, j->bd);
              uint64_t ps = 0;
              for (int r = 0; r < H; ++r)
                for (int c = 0; c < W; ++c) {
                  const int64_t d = (int64_t)j->src[off + (size_t)r * j->stride + c] - rec[r * W + c];
                  ps += (uint64_t)(d * d);
                }
              if (rsh) ps = (ps + ((uint64_t)1 << (rsh - 1))) >> rsh;
              /* `16 * pixel_dist(...)` is an unsigned (32-bit) product */
              const int64_t px = (int64_t)(uint32_t)(16u * (uint32_t)ps);
              dist = (high && px < dist) ? dist : px;
            } else {
              dist += sse_diff;
            }
          }
          sse = block_sse;
        }
        /* search_tx_type's cost_coeffs (tx_search.c:2172-2176) when tables are
         * given, else the TPL rate_estimator proxy */
        const int rate =
            j->cc ? orc_cost_coeffs_txb(j->cc, qc, eob, 0, j->tx_size, t,
                                        j->txb_ctx ? j->txb_ctx[2 * blk] : 0,
                                        j->txb_ctx ? j->txb_ctx[2 * blk + 1] : 0,
                                        j->tx_type_costs ? j->tx_type_costs[t] : 0, 0)
                  : rate_estimator(qc, eob, j->tx_size);
        const int64_t rd = rdcost(j->rdmult, rate, dist);
        if (rd < best.rdcost) {
          best.best_type = t;
          best.eob = eob;
          best.rate = rate;
          best.satd = satd;
          best.dist = dist;
          best.sse = sse;
          best.rdcost = rd;
          memcpy(j->qcoeff + blk * n, qc, sizeof(int32_t) * n);
          memcpy(j->dqcoeff + blk * n, dq, sizeof(int32_t) * n);
        }
      }
      if (best.rdcost == INT64_MAX) {
        /* no allowed type in the evaluated set (caller masks only): the
         * build's defined "no candidate" result -- TX_TYPE_INVALID, eob 0,
         * zero coefficients, rdcost INT64_MAX */
        best.best_type = 255;
        memset(j->qcoeff + blk * n, 0, sizeof(int32_t) * n);
        memset(j->dqcoeff + blk * n, 0, sizeof(int32_t) * n);
      }
      j->out[blk] = best;
    }
  }
  return NULL;
}

static long rdo_plane(const uint16_t *src, const uint16_t *pred, int stride, int width,
                      int height, int tx_size, unsigned type_mask, int bd, const OrcQuant *q,
                      int rdmult, OrcRdoBlock *out, int32_t *qcoeff, int32_t *dqcoeff,
                      int threads, int px, const uint16_t *block_mask,
                      const uint8_t *block_map, const OrcCoeffCosts *cc,
                      const int32_t *txb_ctx, const int32_t *tx_type_costs) {
  const int W = orc_tx_w(tx_size), H = orc_tx_h(tx_size);
  const int bh = height / H;
  RdoJob base;
  memset(&base, 0, sizeof(base));
  base.src = src;
  base.pred = pred;
  base.stride = stride;
  base.width = width;
  base.tx_size = tx_size;
  base.bd = bd;
  base.rdmult = rdmult;
  base.q = q;
  base.out = out;
  base.qcoeff = qcoeff;
  base.dqcoeff = dqcoeff;
  base.px = px;
  base.block_mask = block_mask;
  base.block_map = block_map;
  base.cc = cc;
  base.txb_ctx = txb_ctx;
  base.tx_type_costs = tx_type_costs;
  for (int t = 0; t < 16; ++t)
    if ((type_mask >> t) & 1) base.types[base.ntypes++] = t;
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  if (threads > bh) threads = bh > 0 ? bh : 1;
  pthread_t tid[64];
  RdoJob jobs[64];
  for (int i = 0; i < threads; ++i) {
    jobs[i] = base;
    jobs[i].row0 = bh * i / threads;
    jobs[i].row1 = bh * (i + 1) / threads;
    if (threads > 1) pthread_create(&tid[i], NULL, rdo_rows, &jobs[i]);
    else rdo_rows(&jobs[i]);
  }
  if (threads > 1)
    for (int i = 0; i < threads; ++i) pthread_join(tid[i], NULL);
  return (long)bh * (width / W);
}

long orc_rdo_plane(const uint16_t *src, const uint16_t *pred, int stride, int width,
                   int height, int tx_size, unsigned type_mask, int bd, const OrcQuant *q,
                   int rdmult, OrcRdoBlock *out, int32_t *qcoeff, int32_t *dqcoeff,
                   int threads) {
  return rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bd, q, rdmult, out,
                   qcoeff, dqcoeff, threads, 0, NULL, NULL, NULL, NULL, NULL);
}

long orc_rdo_plane_px(const uint16_t *src, const uint16_t *pred, int stride, int width,
                      int height, int tx_size, unsigned type_mask, int bd, const OrcQuant *q,
                      int rdmult, OrcRdoBlock *out, int32_t *qcoeff, int32_t *dqcoeff,
                      int threads) {
  return rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bd, q, rdmult, out,
                   qcoeff, dqcoeff, threads, 1, NULL, NULL, NULL, NULL, NULL);
}

long orc_rdo_plane_masked(const uint16_t *src, const uint16_t *pred, int stride, int width,
                          int height, int tx_size, unsigned type_mask, int bd, const OrcQuant *q,
                          int rdmult, const uint16_t *block_mask, const uint8_t *block_map,
                          int px, OrcRdoBlock *out, int32_t *qcoeff, int32_t *dqcoeff,
                          int threads) {
  return rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bd, q, rdmult, out,
                   qcoeff, dqcoeff, threads, px, block_mask, block_map, NULL, NULL, NULL);
}

long orc_rdo_plane_rate(const uint16_t *src, const uint16_t *pred, int stride, int width,
                        int height, int tx_size, unsigned type_mask, int bd, const OrcQuant *q,
                        int rdmult, const OrcCoeffCosts *cc, const int32_t *txb_ctx,
                        const int32_t *tx_type_costs, const uint16_t *block_mask,
                        const uint8_t *block_map, OrcRdoBlock *out, int32_t *qcoeff,
                        int32_t *dqcoeff, int threads) {
  return rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bd, q, rdmult, out,
                   qcoeff, dqcoeff, threads, 0, block_mask, block_map, cc, txb_ctx,
                   tx_type_costs);
}

/* Per 64x64 SB: the size (of `sizes`, largest area first) whose full blocks
 * tile the SB with the lowest summed rdcost (ties: the earlier size), then
 * recon = pred + inverse transforms of the chosen blocks (eob 0: untouched).
 * recs / dqs: per size (index into `sizes`), raster block order. */
void orc_rdo_reconstruct(int nsizes, const int *sizes, const OrcRdoBlock *const *recs,
                         const int32_t *const *dqs, int width, int height,
                         const uint16_t *pred, uint16_t *recon, int stride, int bd,
                         uint8_t *sb_tx_size) {
  const int sbw = (width + 63) / 64, sbh = (height + 63) / 64;
  for (int sy = 0; sy < sbh; ++sy)
    for (int sx = 0; sx < sbw; ++sx) {
      int64_t best = INT64_MAX;
      int best_s = 255;
      for (int i = 0; i < nsizes; ++i) {
        const int s = sizes[i], W = orc_tx_w(s), H = orc_tx_h(s);
        const int y1 = height - sy * 64 < 64 ? height - sy * 64 : 64;
        const int x1 = width - sx * 64 < 64 ? width - sx * 64 : 64;
        if (y1 % H || x1 % W) continue;
        /* costs are >= 0; sums saturate at INT64_MAX (a block without a
         * candidate costs INT64_MAX) */
        int64_t sum = 0;
        for (int y = 0; y < y1; y += H)
          for (int x = 0; x < x1; x += W) {
            const int64_t c = recs[i][((sy * 64 + y) / H) * (width / W) + (sx * 64 + x) / W].rdcost;
            sum = sum > INT64_MAX - c ? INT64_MAX : sum + c;
          }
        if (sum < best) {
          best = sum;
          best_s = s;
        }
      }
      sb_tx_size[sy * sbw + sx] = (uint8_t)best_s;
    }
  for (int y = 0; y < height; ++y)
    memcpy(recon + (size_t)y * stride, pred + (size_t)y * stride, sizeof(uint16_t) * width);
  for (int i = 0; i < nsizes; ++i) {
    const int s = sizes[i], W = orc_tx_w(s), H = orc_tx_h(s), n = orc_max_eob(s);
    const int bw = width / W, bh = height / H;
    for (int by = 0; by < bh; ++by)
      for (int bx = 0; bx < bw; ++bx) {
        const int y = by * H, x = bx * W, blk = by * bw + bx;
        if (sb_tx_size[(y / 64) * sbw + x / 64] != s || recs[i][blk].eob == 0) continue;
        orc_inv_txfm2d_add(dqs[i] + (size_t)blk * n, recon + (size_t)y * stride + x, stride,
                           recs[i][blk].best_type, s, bd);
      }
  }
}
