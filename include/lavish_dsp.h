/*
 * lavish_dsp.h -- C ABI of liblavish_hip.so, the MI355X (gfx950) backend for
 * the per-block RDO hot path of aom-av1-lavish (a libaom v3.6.0 fork).
 *
 * Two layers:
 *
 *  1. Per-call RTCD shims.  Same prototypes as the reference's rtcd entries,
 *     suffixed `_hip`, so a maintainer can add `hip` as an RTCD arch
 *      and `specialize` these names.  They take the
 *     reference's caller-owned HOST buffers, stage them through a per-thread
 *     device scratch and run the same HIP kernels as the batch layer.  One
 *     block per call cannot amortise a kernel launch: these exist for drop-in
 *     parity, not speed.
 *
 *  2. Batch API (`lavish_*`).  Device pointers, asynchronous on a caller
 *     stream (hipStream_t passed as void*; NULL = default stream), a whole
 *     residual plane / candidate list per launch.  This is the performance
 *     boundary used by bench.py.
 *
 * Types follow the reference: tran_low_t == int32_t, tran_high_t == int64_t
 * (aom_dsp/aom_dsp_common.h:63-64); TX_SIZE / TX_TYPE are the uint8_t enums of
 * aom_dsp/txfm_common.h:25-71.  Highbd pixel pointers in the shims are the
 * reference's tagged pointers (CONVERT_TO_BYTEPTR, aom_ports/mem.h:79-80).
 *
 * Errors: the reference has no error channel; on a HIP failure the library
 * records a sticky status (lavish_hip_status) and, by default, prints the
 * failure and aborts.  There is no CPU fallback.
 */
#ifndef LAVISH_DSP_H_
#define LAVISH_DSP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Library state                                                            */
/* ------------------------------------------------------------------------ */
/* 0 when no HIP error has been seen, else the first hipError_t value. */
int lavish_hip_status(void);
const char *lavish_hip_status_string(void);
/* 1 (default): abort() on a HIP error; 0: record the status and continue. */
void lavish_hip_set_abort_on_error(int on);
/* Select the HIP device used by the per-call shims (default: current). */
int lavish_hip_init(int device);
/* ABI version: 0x00MMmmpp */
int lavish_hip_version(void);

/* TxfmParam of aom_dsp/txfm_common.h:89-101 (same field order / padding). */
typedef struct LavishTxfmParam {
  uint8_t tx_type;
  uint8_t tx_size;
  int lossless;
  int bd;
  int is_hbd;
  uint8_t tx_set_type;
  int eob;
} LavishTxfmParam;

/* ------------------------------------------------------------------------ */
/* Quantizer tables                                                         */
/* ------------------------------------------------------------------------ */
/* The two-entry ([0]=DC, [1]=AC) tables a quantizer reads, i.e. one row of
 * the reference's QUANTS/Dequants (av1/encoder/av1_quantize.h).  For the fp
 * quantizer `round`/`quant` hold round_fp/quant_fp. */
typedef struct LavishQuantParams {
  int16_t zbin[2];
  int16_t round[2];
  int16_t quant[2];
  int16_t quant_shift[2];
  int16_t dequant[2];
} LavishQuantParams;

enum { LAVISH_QUANT_FP = 0, LAVISH_QUANT_B = 1, LAVISH_QUANT_NONE = 2 };

/* av1_build_quantizer (av1/encoder/av1_quantize.c:590-686, including the
 * fork's quant_sharpness) for the luma plane at one qindex.
 * kind = LAVISH_QUANT_FP or LAVISH_QUANT_B selects which round/quant pair is
 * returned.  Returns 0 on success. */
int lavish_build_quant_params(int bit_depth, int qindex, int quant_sharpness,
                              int y_dc_delta_q, int kind,
                              LavishQuantParams *out);

/* av1_scan_orders[tx_size][tx_type] (av1/common/scan.c); host pointers. */
const int16_t *lavish_scan(int tx_size, int tx_type);
const int16_t *lavish_iscan(int tx_size, int tx_type);

/* ------------------------------------------------------------------------ */
/* Batch API (device pointers)                                              */
/* ------------------------------------------------------------------------ */
/* Forward transform + quantize every full tx_size block of a residual plane
 * for every TX type set in type_mask (the body of search_tx_type's per-type
 * loop, av1/encoder/tx_search.c:2148-2312: av1_xform -> av1_quant,
 * av1/encoder/encodemb.c:295-341).
 *   residual : int16 plane, `stride` elements per row, width x height.
 *   blocks   : B = (width / W) * (height / H), raster order (full blocks).
 *   tx_size  : any of the 19 sizes; the 64-point ones keep the reference's
 *              packed 32x32 (or 32x16 / 16x32) low-frequency quadrant.
 *   slots    : the set bits of type_mask in ascending TX_TYPE order; every
 *              set type must be valid for tx_size (EXT_TX_SET rules).
 *   outputs  : qcoeff/dqcoeff[slot][block][n], eob[slot][block], with
 *              n = av1_get_max_eob(tx_size); coeff (nullable) receives the
 *              unquantized transform output in the same layout.
 *   quant    : LAVISH_QUANT_FP (av1_quantize_fp*), LAVISH_QUANT_B
 *              (aom_quantize_b*), LAVISH_QUANT_NONE (transform only);
 *              log_scale = av1_get_tx_scale(tx_size); bit_depth > 8 selects
 *              the highbd quantizers.
 * Returns 0 on success, a negative value on invalid arguments. */
int lavish_txq_plane(const int16_t *residual, int stride, int width,
                     int height, int tx_size, uint32_t type_mask,
                     int bit_depth, int quant_kind,
                     const LavishQuantParams *qp, int32_t *qcoeff,
                     int32_t *dqcoeff, uint16_t *eob, int32_t *coeff,
                     void *stream);

/* Streams the per-size kernels of lavish_rdo_frame are dealt over: 1 .. 3
 * -- the caller's stream + streams - 1 internal streams, forked and joined
 * by events (default 3; 1: every size on the caller's stream, for isolated
 * per-kernel timings under a profiler).  Results are identical.  Returns -1
 * for other values.  No reference counterpart. */
int lavish_set_fan_width(int streams);

/* Frame batch: lavish_txq_plane for every TX size whose bit is set in
 * size_mask (bit = TX_SIZE), with type_masks[tx_size] and per-size output
 * pointers qcoeff[tx_size] / dqcoeff[tx_size] / eob[tx_size] (arrays of 19
 * entries, unused entries ignored).  The independent per-size kernels run
 * concurrently on internal streams forked from and joined back to `stream`;
 * the call is asynchronous with respect to the host like the others. */
int lavish_txq_frame(const int16_t *residual, int stride, int width,
                     int height, uint32_t size_mask,
                     const uint32_t *type_masks, int bit_depth,
                     int quant_kind, const LavishQuantParams *qp,
                     int32_t *const *qcoeff, int32_t *const *dqcoeff,
                     uint16_t *const *eob, void *stream);

/* Quantize `nblocks` coefficient blocks of n words each (contiguous) with one
 * scan order (device pointers to scan / iscan of n entries). */
int lavish_quantize_batch(const int32_t *coeff, int n, int nblocks,
                          const int16_t *scan, const int16_t *iscan,
                          int log_scale, int bit_depth, int quant_kind,
                          const LavishQuantParams *qp, int32_t *qcoeff,
                          int32_t *dqcoeff, uint16_t *eob, void *stream);

/* ---- av1_quant: quantizer selection ------------------
 * The tables av1_quant reads from MACROBLOCK_PLANE (*_QTX, [0] DC, [1] AC;
 * av1/encoder/block.h), as av1_build_quantizer fills them. */
typedef struct LavishPlaneQuant {
  int16_t zbin[2], round_fp[2], quant_fp[2], round[2], quant[2], quant_shift[2],
      dequant[2];
} LavishPlaneQuant;
int lavish_build_plane_quant(int bit_depth, int qindex, int quant_sharpness,
                             int y_dc_delta_q, LavishPlaneQuant *out);

/* xform_quant_idx (AV1_XFORM_QUANT, av1/encoder/encodemb.h) plus the
 * search_tx_type selection */
enum {
  LAVISH_AV1_QUANT_FP = 0,   /* av1_quantize_fp_facade / highbd */
  LAVISH_AV1_QUANT_B = 1,    /* av1_quantize_b_facade / highbd */
  LAVISH_AV1_QUANT_DC = 2,   /* av1_quantize_dc_facade / highbd */
  LAVISH_AV1_QUANT_SKIP = 3, /* AV1_XFORM_QUANT_SKIP_QUANT: outputs untouched */
  /* search_tx_type (tx_search.c:2140-2169): skip_trellis ? B : FP, then per
   * block skip_trellis_opt_based_on_satd (:1923-1955) -> B without trellis
   * when the satd gate fires, else FP with trellis */
  LAVISH_AV1_QUANT_SATD_GATE = 4
};

/* av1_quant (av1/encoder/encodemb.c:308-341) over nblocks contiguous blocks
 * of n = av1_get_max_eob(tx_size) coefficients (device): the facade of `mode`
 * (is_hbd = bit_depth > 8, log_scale of tx_size, scan of (tx_size, tx_type),
 * no quantization matrix) -> qcoeff / dqcoeff [nblocks][n], eob[nblocks].
 * SATD_GATE mode: skip_trellis, coeff_opt_satd_threshold
 * (coeff_opt_thresholds[1], UINT_MAX = off), qstep (dequant_QTX[1] >>
 * (hbd ? bd - 5 : 3)) and the optional per-block dc_only flags as the
 * reference passes them.  flags (device, nullable) [nblocks]: bit 0 =
 * use_optimize_b (the caller's trellis, av1_optimize_b, is still due for
 * these), bits 1-2 = the quantizer used.  Returns 0 or negative on bad
 * arguments. */
int lavish_av1_quant_batch(const int32_t *coeff, int nblocks, int tx_size,
                           int tx_type, int bit_depth, const LavishPlaneQuant *pq,
                           int mode, int skip_trellis,
                           unsigned coeff_opt_satd_threshold, int qstep,
                           const uint8_t *dc_only, int32_t *qcoeff, int32_t *dqcoeff,
                           uint16_t *eob, uint8_t *flags, void *stream);

/* ---- coefficient rate ---------------------------- */
/* MACROBLOCK::coeff_costs, field for field (CoeffCosts, av1/encoder/block.h:
 * 172-211): LV_MAP_COEFF_COST per [txs_ctx][plane_type] and LV_MAP_EOB_COST
 * per [eob_multi_size][plane_type], as av1_fill_coeff_costs leaves them (the
 * caller copies x->coeff_costs to the device once per frame / cdf update). */
typedef struct LavishCoeffCost {
  int32_t txb_skip_cost[13][2];  /* TXB_SKIP_CONTEXTS */
  int32_t base_eob_cost[4][3];   /* SIG_COEF_CONTEXTS_EOB */
  int32_t base_cost[42][8];      /* SIG_COEF_CONTEXTS */
  int32_t eob_extra_cost[9][2];  /* EOB_COEF_CONTEXTS */
  int32_t dc_sign_cost[3][2];    /* DC_SIGN_CONTEXTS */
  int32_t lps_cost[21][26];      /* LEVEL_CONTEXTS x (COEFF_BASE_RANGE + 1) * 2 */
} LavishCoeffCost;
typedef struct LavishEobCost {
  int32_t eob_cost[2][11];
} LavishEobCost;
typedef struct LavishCoeffCosts {
  LavishCoeffCost coeff_costs[5][2]; /* [TX_SIZES][PLANE_TYPES] */
  LavishEobCost eob_costs[7][2];
} LavishCoeffCosts;
/* TXB_CTX (av1/common/txb_common.h:22-25) */
typedef struct LavishTxbCtx {
  int32_t txb_skip_ctx; /* 0..12 */
  int32_t dc_sign_ctx;  /* 0..2 */
} LavishTxbCtx;

enum {
  LAVISH_COEFF_RATE_EXACT = 0,    /* av1_cost_coeffs_txb (txb_rdopt.c:599-624) */
  LAVISH_COEFF_RATE_LAPLACIAN = 1 /* av1_cost_coeffs_txb_laplacian, adjust_eob 0 */
};

/* Replaces av1_cost_coeffs_txb / av1_cost_coeffs_txb_laplacian (av1/encoder/
 * txb_rdopt.c:599-660; cost_coeffs, tx_search.c:1903-1921, is the caller) for
 * nblocks blocks of one (tx_size, tx_type, plane): qcoeff [nblocks][n], n =
 * av1_get_max_eob(tx_size), raster order as the quantizer writes it (the kept
 * 32x32 quadrant for 64-point sizes); eob [nblocks] = p->eobs (the scan
 * position after the last nonzero coefficient, as the quantizers return it);
 * costs / txb_ctx (nullable: all {0, 0}) / rate [nblocks] on the device;
 * tx_type_cost = get_tx_type_cost's value (txb_rdopt.c:263-294; a
 * MACROBLOCK-level table lookup the caller owns), added for plane 0 when
 * eob > 0.  Returns 0 or negative on bad arguments. */
int lavish_cost_coeffs_txb_batch(const LavishCoeffCosts *costs, const int32_t *qcoeff,
                                 const uint16_t *eob, int nblocks, int plane, int tx_size,
                                 int tx_type, const LavishTxbCtx *txb_ctx, int tx_type_cost,
                                 int mode, int32_t *rate, void *stream);

/* Replaces av1_optimize_b (av1/encoder/encodemb.c:87-103) -> av1_optimize_txb
 * (txb_rdopt.c:326-449), the trellis search_tx_type runs on FP-quantized
 * blocks flagged use_optimize_b, for nblocks blocks of one (tx_size,
 * tx_type, plane), no quantization matrix.  Device arrays [nblocks][n] (n =
 * av1_get_max_eob): tcoeff (p->coeff) in; qcoeff / dqcoeff updated in place;
 * eob [nblocks] in / out; txb_ctx nullable ({0, 0}); rate [nblocks] out
 * (rate_cost, incl. the skip / non-skip and tx-type cost); entropy_ctx
 * [nblocks] out, nullable (p->txb_entropy_ctx = av1_get_txb_entropy_context).
 * rdmult = x->rdmult, is_inter = is_inter_block, sharpness =
 * oxcf.algo_cfg.sharpness, dequant = p->dequant_QTX[0..1] (host).  eob 0:
 * rate = txb_skip_cost[ctx][1] (the early exit; segments with
 * optimize_seg_arr 0 or lossless are the caller's to skip).  Returns 0 or
 * negative on bad arguments. */
int lavish_optimize_b_batch(const LavishCoeffCosts *costs, const int32_t *tcoeff,
                            int32_t *qcoeff, int32_t *dqcoeff, uint16_t *eob, int nblocks,
                            int plane, int tx_size, int tx_type, int bit_depth, int is_inter,
                            int rdmult, int sharpness, const int16_t *dequant,
                            const LavishTxbCtx *txb_ctx, int tx_type_cost, int32_t *rate,
                            uint8_t *entropy_ctx, void *stream);

/* ---- pixel-domain batch kernels ----------------------------------------- */
/* One job = one block.  Offsets are in ELEMENTS (u8 or u16 samples / int16
 * residual words) from the plane base pointers passed to the call.  Which
 * fields a kernel reads is stated per call. */
typedef struct LavishPixJob {
  int64_t src_off;    /* first operand (src) */
  int64_t ref_off[4]; /* second operand(s): ref / candidate positions */
  int64_t aux_off;    /* second_pred / diff / coefficient offset */
  int32_t xoff, yoff; /* sub-pixel offsets (1/8 pel, 0..7) */
} LavishPixJob;

/* SAD of a w x h block against nrefs (1..4) reference positions
 * (aom_dsp/sad.c:22-129, highbd :240-330).
 *   mode 0: aom_sad, 1: aom_sad_skip (2 x SAD of even rows),
 *        2: aom_sad_avg against ROUND_POWER_OF_TWO(ref + second_pred, 1)
 *           with second_pred at second_pred + job.aux_off, stride w.
 *   highbd: 0 = u8 planes, 1 = u16 planes (plain device pointers).
 *   sad_out[job * nrefs + k]. */
int lavish_sad_batch(const void *src, int src_stride, const void *ref,
                     int ref_stride, int w, int h, const LavishPixJob *jobs,
                     int njobs, int nrefs, int mode, const void *second_pred,
                     int highbd, uint32_t *sad_out, void *stream);

/* Variance family, d = a[src_off] - b[ref_off[0]]
 * (aom_dsp/variance.c:38-145,321-408,454-670).
 *   kind 0: variance (var_out, sse_out), 1: mse (var_out = sse),
 *        2: get_var (sse_out, sum_out), 3: sub-pixel variance of the
 *        bilinear-filtered a (job.xoff/yoff; reads (h+1) x (w+1) of a),
 *        4: sse as int64 (aom_sse / aom_highbd_sse; sse64_out),
 *        5: sub-pixel avg variance (second_pred + job.aux_off, stride w).
 *   bit_depth 8/10/12 selects the highbd rounding (highbd = 1 only).
 * Unused output pointers may be NULL. */
int lavish_variance_batch(const void *a, int a_stride, const void *b,
                          int b_stride, int w, int h, const LavishPixJob *jobs,
                          int njobs, int kind, int bit_depth, int highbd,
                          const void *second_pred, uint32_t *var_out,
                          uint32_t *sse_out, int32_t *sum_out,
                          int64_t *sse64_out, void *stream);

/* diff[aux_off + r*diff_stride + c] = src[src_off..] - pred[ref_off[0]..]
 * (aom_subtract_block / aom_highbd_subtract_block, aom_dsp/subtract.c). */
int lavish_subtract_batch(int rows, int cols, int16_t *diff, int diff_stride,
                          const void *src, int src_stride, const void *pred,
                          int pred_stride, const LavishPixJob *jobs,
                          int njobs, int highbd, void *stream);

/* aom_sum_squares_2d_i16 (aom_dsp/sum_squares.c:16-30) at src + src_off. */
int lavish_sum_squares_batch(const int16_t *src, int stride, int w, int h,
                             const LavishPixJob *jobs, int njobs,
                             uint64_t *out, void *stream);

/* aom_hadamard_{4x4,8x8,16x16,32x32} (highbd = 0) and
 * aom_highbd_hadamard_{8x8,16x16,32x32} (highbd = 1), aom_dsp/avg.c:102-507:
 * src_diff + job.src_off (stride) -> coeff + job.aux_off (n*n words). */
int lavish_hadamard_batch(int n, int highbd, const int16_t *src_diff,
                          int stride, const LavishPixJob *jobs, int njobs,
                          int32_t *coeff, void *stream);

/* aom_satd (aom_dsp/avg.c:509-516) of nblocks contiguous blocks. */
int lavish_satd_batch(const int32_t *coeff, int length, int nblocks, int *out,
                      void *stream);

/* av1_block_error (bit_depth 0) / av1_highbd_block_error (bit_depth 8/10/12)
 * (av1/encoder/rdopt.c:635-682) of nblocks contiguous blocks of n words. */
int lavish_block_error_batch(const int32_t *coeff, const int32_t *dqcoeff,
                             int n, int nblocks, int bit_depth, int64_t *err,
                             int64_t *ssz, void *stream);

/* aom_hadamard_lp_{8x8,16x16} (aom_dsp/avg.c:207-316): int16 coefficients
 * (n = 8 or 16, else -1). */
int lavish_hadamard_lp_batch(int n, const int16_t *src_diff, int stride,
                             const LavishPixJob *jobs, int njobs,
                             int16_t *coeff, void *stream);
/* aom_satd_lp (aom_dsp/avg.c:518-524) of nblocks contiguous int16 blocks. */
int lavish_satd_lp_batch(const int16_t *coeff, int length, int nblocks,
                         int *out, void *stream);
/* av1_block_error_lp (av1/encoder/rdopt.c:650-660). */
int lavish_block_error_lp_batch(const int16_t *coeff, const int16_t *dqcoeff,
                                int n, int nblocks, int64_t *err,
                                void *stream);
/* (sum, sum of squares) of a w x h int16 block at src + job.src_off:
 * aom_sum_sse_2d_i16 (aom_dsp/sum_squares.c:75-90) and aom_get_blk_sse_sum
 * (aom_dsp/blk_sse_sum.c:14-27).  Either output may be NULL. */
int lavish_sum_sse_batch(const int16_t *src, int stride, int w, int h,
                         const LavishPixJob *jobs, int njobs, int32_t *sum,
                         int64_t *sse, void *stream);

/* ---- lossless 4x4 Walsh-Hadamard ----------------------------------------
 * av1_fwht4x4 (hybrid_fwd_txfm.c:24-76): src_diff + job.src_off (stride) ->
 * 16 words at coeff + job.aux_off. */
int lavish_fwht4x4_batch(const int16_t *src_diff, int stride,
                         const LavishPixJob *jobs, int njobs, int32_t *coeff,
                         void *stream);

/* ---- inverse transform + reconstruction (a17) ---------------------------
 * av1_inverse_transform_block (av1/common/idct.c:304-322) for a list of
 * blocks of one tx_size: dst (u8 when highbd = 0, then bit_depth must be 8;
 * u16 otherwise) += inverse 2-D transform of the block's dqcoeff, clipped to
 * the bit depth.  Blocks with eob == 0 are left untouched (the reference
 * returns early).  coeff_off addresses av1_get_max_eob(tx_size) words in the
 * reference's layout (64-point sizes: the packed 32-column quadrant).  Jobs of
 * one call must not overlap in dst. */
typedef struct LavishInvJob {
  int64_t dst_off;   /* element offset of the block's top-left pixel */
  int64_t coeff_off; /* word offset of the block's dqcoeff */
  int32_t tx_type;
  int32_t eob;
} LavishInvJob;

int lavish_inv_txfm_add_batch(const int32_t *dqcoeff, int tx_size,
                              const LavishInvJob *jobs, int njobs, void *dst,
                              int dst_stride, int bit_depth, int highbd,
                              void *stream);
/* The lossless TX_4X4 inverse (av1_highbd_iwht4x4_add, idct.c:34-40): per
 * job the 16-coefficient WHT when eob > 1, the DC-only form when eob == 1,
 * nothing when eob == 0; same job / destination conventions. */
int lavish_iwht4x4_add_batch(const int32_t *dqcoeff, const LavishInvJob *jobs,
                             int njobs, void *dst, int dst_stride,
                             int bit_depth, int highbd, void *stream);

/* ---- C4: fused TX-type RDO ----------------------------------------------
 * For every full tx_size block of (src - pred) (u16 planes, bit_depth 8/10/12)
 * and every TX type in type_mask: forward transform -> av1_highbd_quantize_fp
 * -> aom_satd(coeff) -> av1_highbd_block_error -> TX-domain distortion shift
 * (tx_search.c:1077-1116) -> rate_estimator (tpl_model.c:214-226) ->
 * RDCOST(rdmult, rate, dist) (rd.h:31-33); the block keeps the first type
 * with the strictly lowest cost.  Outputs per block (raster order): the
 * decision record and the winner's qcoeff / dqcoeff (n words each,
 * n = av1_get_max_eob). */
typedef struct LavishRdoBlock {
  int32_t best_type;
  int32_t eob;
  int32_t rate;   /* rate_estimator (<< AV1_PROB_COST_SHIFT) */
  int32_t satd;   /* aom_satd of the winner's coefficients */
  int64_t dist;   /* TX-domain distortion after the tx-scale shift */
  int64_t sse;
  int64_t rdcost;
} LavishRdoBlock;

int lavish_rdo_plane(const uint16_t *src, const uint16_t *pred, int stride,
                     int width, int height, int tx_size, uint32_t type_mask,
                     int bit_depth, const LavishQuantParams *qp, int rdmult,
                     LavishRdoBlock *out, int32_t *qcoeff, int32_t *dqcoeff,
                     void *stream);
/* The same with the per-block allowed_tx_mask / search order that
 * lavish_prune_tx_2d_batch produces (device arrays, either may be NULL):
 * block b only considers types set in block_mask[b] (0 = DCT_DCT only,
 * get_tx_mask's rule) that appear in block_map[b][0..15], and equal costs go
 * to the type earlier in block_map[b] (search_tx_type's txk_map loop,
 * tx_search.c:2148-2246).  type_mask is the evaluated superset.
 * pixel_domain: 0 TX-domain distortion, 1 pixel-domain (sizes <= 32). */
int lavish_rdo_plane_masked(const uint16_t *src, const uint16_t *pred, int stride,
                            int width, int height, int tx_size, uint32_t type_mask,
                            int bit_depth, const LavishQuantParams *qp, int rdmult,
                            const uint16_t *block_mask, const uint8_t *block_map,
                            int pixel_domain, LavishRdoBlock *out, int32_t *qcoeff,
                            int32_t *dqcoeff, void *stream);
/* The TX-domain decision ranked by the coefficient rate: per type, rate =
 * av1_cost_coeffs_txb (txb_rdopt.c:599-624, the cost_coeffs of
 * search_tx_type, tx_search.c:1903-1921,2172-2176) on the FP-quantized block
 * instead of rate_estimator, with the luma tables of the device CoeffCosts
 * `costs`, per-block TXB_CTX txb_ctx (device, nullable: {0, 0}) and
 * tx_type_costs[16] = get_tx_type_cost per tx type for this tx_size (host,
 * nullable: 0).  Records' rate is that rate.  Masks as above. */
int lavish_rdo_plane_rate(const uint16_t *src, const uint16_t *pred, int stride,
                          int width, int height, int tx_size, uint32_t type_mask,
                          int bit_depth, const LavishQuantParams *qp, int rdmult,
                          const LavishCoeffCosts *costs, const LavishTxbCtx *txb_ctx,
                          const int32_t *tx_type_costs, const uint16_t *block_mask,
                          const uint8_t *block_map, LavishRdoBlock *out,
                          int32_t *qcoeff, int32_t *dqcoeff, void *stream);

/* Frame level: lavish_rdo_plane for every size set in size_mask (bit =
 * TX_SIZE) with type_masks[tx_size] and per-size outputs (arrays of 19
 * pointers), the sizes running concurrently on internal streams. */
int lavish_rdo_frame(const uint16_t *src, const uint16_t *pred, int stride,
                     int width, int height, uint32_t size_mask,
                     const uint32_t *type_masks, int bit_depth,
                     const LavishQuantParams *qp, int rdmult,
                     LavishRdoBlock *const *records, int32_t *const *qcoeff,
                     int32_t *const *dqcoeff, void *stream);

/* Pixel-domain distortion: search_tx_type with
 * use_transform_domain_distortion == 0 and predict_dc_level 0
 * (tx_search.c:2060-2103, 2187-2231).  Same outputs; per block
 * block_sse = ROUND_POWER_OF_TWO(sum of squared residual, 2 (bd-8)) * 16 and,
 * per type: eob 0 -> dist = block_sse; otherwise dist = dist_block_px_domain
 * (tx_search.c:969-1017: recon = pred + av1_inverse_transform_block,
 * 16 * the highbd-rounded sse of src - recon), a high-energy block
 * (block_sse >= 128*128*pels) keeping the TX-domain distortion when that is
 * larger, and TX_64X64 with high energy using TX-domain + the energy outside
 * the kept quadrant unless that energy is small; sse = block_sse.  The 64-point
 * sizes take exactly one type (DCT_DCT); -6 otherwise.
 * Replaces the search_tx_type distortion step (tx_search.c:2187-2231). */
int lavish_rdo_plane_px(const uint16_t *src, const uint16_t *pred, int stride,
                        int width, int height, int tx_size, uint32_t type_mask,
                        int bit_depth, const LavishQuantParams *qp, int rdmult,
                        LavishRdoBlock *out, int32_t *qcoeff, int32_t *dqcoeff,
                        void *stream);
int lavish_rdo_frame_px(const uint16_t *src, const uint16_t *pred, int stride,
                        int width, int height, uint32_t size_mask,
                        const uint32_t *type_masks, int bit_depth,
                        const LavishQuantParams *qp, int rdmult,
                        LavishRdoBlock *const *records, int32_t *const *qcoeff,
                        int32_t *const *dqcoeff, void *stream);

/* Per 64x64 superblock: the candidate size (of size_mask) whose blocks tile
 * the SB with the lowest summed rd cost (ties: the larger size) -> sb_tx_size
 * (255 when none tiles it); then recon = pred + the chosen blocks' inverse
 * transforms with their best types (lavish_inv_txfm_add_batch semantics:
 * eob 0 leaves the prediction).  u16 planes, `stride` elements. */
int lavish_rdo_reconstruct(uint32_t size_mask,
                           const LavishRdoBlock *const *records,
                           const int32_t *const *dqcoeff, int width,
                           int height, const uint16_t *pred, uint16_t *recon,
                           int stride, int bit_depth, uint8_t *sb_tx_size,
                           void *stream);

/* The C4 step captured once for fixed buffers: lavish_rdo_frame (all sizes
 * of size_mask) + lavish_rdo_reconstruct recorded into a HIP graph that
 * lavish_rdo_graph_launch replays with one launch on any stream (device
 * pointers and parameters are the capture's; replays of one graph must not
 * overlap).  No reference counterpart: a launch-count aid for callers that
 * run the step on many small rectangles.  Creation runs the step once
 * (uncaptured) after the work already queued on `stream` and waits for it:
 * it WRITES records, qcoeff, dqcoeff, recon and sb_tx_size.  The graph owns
 * its reconstruction scratch and the internal streams / fork-join events its
 * capture forked over (none shared with uncaptured calls on the thread).
 * -8: capture / instantiation failed. */
typedef struct LavishRdoGraph LavishRdoGraph;
int lavish_rdo_graph_create(const uint16_t *src, const uint16_t *pred, int stride,
                            int width, int height, uint32_t size_mask,
                            const uint32_t *type_masks, int bit_depth,
                            const LavishQuantParams *qp, int rdmult,
                            LavishRdoBlock *const *records, int32_t *const *qcoeff,
                            int32_t *const *dqcoeff, uint16_t *recon, uint8_t *sb_tx_size,
                            void *stream, LavishRdoGraph **graph);
int lavish_rdo_graph_launch(LavishRdoGraph *graph, void *stream);
void lavish_rdo_graph_destroy(LavishRdoGraph *graph);

/* ---- C3: DIAMOND full-pixel motion search ------------------------------
 * av1_full_pixel_search with search_method DIAMOND (av1/encoder/mcomp.c:
 * 1755-1895 -> full_pixel_diamond :1479-1526 -> diamond_search_sad
 * :1318-1477), one (block, reference) per job, 8-bit planes.
 * Offsets in bytes from src / ref; ref_off is the block origin at mv (0,0);
 * both planes must be padded so that every mv inside the limits (as
 * av1_set_mv_limits computes them) addresses memory, plus 3 bytes of slack
 * after each row end. */
typedef struct LavishDiamondJob {
  int64_t src_off;
  int64_t ref_off;
  int16_t start_row, start_col;   /* FULLPEL_MV start */
  int16_t ref_mv_row, ref_mv_col; /* MV (1/8 pel) the mv cost refers to */
  int16_t col_min, col_max, row_min, row_max; /* FullMvLimits */
} LavishDiamondJob;

typedef struct LavishDiamondResult {
  int16_t best_row, best_col; /* FULLPEL_MV */
  int32_t bestsme;  /* returned var cost: aom_variance + mv_err_cost */
  int32_t steps;    /* DIAMOND: 8-site steps; pattern methods: candidate rounds */
  int32_t searches; /* DIAMOND: diamond_search_sad runs; pattern methods
                       (lavish_full_pixel_search_batch, BIGDIA family): the
                       SAD blocks read (start, in-range candidates, cost list) */
} LavishDiamondResult;

/* mv_cost_type: MV_COST_TYPE (av1/encoder/mcomp.h:31-38) 1 L1_LOWRES,
 * 2 L1_MIDRES, 3 L1_HDRES, 4 NONE (ENTROPY needs the entropy context's cost
 * tables: -2).  use_downsampled_sad: sdf/sdx4df = aom_sad_skip_* for blocks
 * >= 16 high with the reference's quality recheck.  w x h: any
 * @encoder_block_sizes entry (else -3). */
int lavish_diamond_search_batch(const uint8_t *src, int src_stride,
                                const uint8_t *ref, int ref_stride, int w,
                                int h, const LavishDiamondJob *jobs, int njobs,
                                int step_param, int mv_cost_type,
                                int use_downsampled_sad,
                                LavishDiamondResult *out, void *stream);

/* FAST_BIGDIA (search_method of the TPL model at speed >= 5 and of
 * bsize-dependent full-pel searches): fast_bigdia_search -> bigdia_search ->
 * pattern_search (av1/encoder/mcomp.c:498-550, 1017-1316) with
 * do_init_search 0, then get_mvpred_var_cost; the downsampled-SAD recheck of
 * av1_full_pixel_search (:1840-1873) as for DIAMOND.  Same jobs / results as
 * lavish_diamond_search_batch (steps = candidate rounds, searches = passes). */
int lavish_fast_bigdia_search_batch(const uint8_t *src, int src_stride,
                                    const uint8_t *ref, int ref_stride, int w,
                                    int h, const LavishDiamondJob *jobs,
                                    int njobs, int step_param,
                                    int mv_cost_type, int use_downsampled_sad,
                                    LavishDiamondResult *out, void *stream);

/* MV_COST_PARAMS (av1/encoder/mcomp.h:69-85) for any mv_cost_type.  The
 * tables are DEVICE pointers: mvjcost[MV_JOINTS] and mvcost[0] / [1] at the
 * centre (index MV_MAX = 16383) of 2 * MV_MAX + 1 entries each, as
 * x->mv_costs->mv_cost_stack is addressed (av1/encoder/block.h); needed for
 * MV_COST_ENTROPY only.  sad_per_bit / error_per_bit: x->sadperbit /
 * x->errorperbit (av1_set_error_per_bit / av1_set_sad_per_bit). */
typedef struct LavishMvCostParams {
  int32_t mv_cost_type; /* MV_COST_TYPE: 0 ENTROPY, 1..3 L1_{LOW,MID,HD}RES, 4 NONE */
  int32_t sad_per_bit;
  int32_t error_per_bit;
  int32_t reserved;
  const int32_t *mvjcost;
  const int32_t *mvcost[2];
} LavishMvCostParams;

/* av1_full_pixel_search (av1/encoder/mcomp.c:1755-1873, no mesh refinement)
 * for search_method (SEARCH_METHODS, mcomp_structs.h:56-86) DIAMOND 0,
 * BIGDIA 5 (pattern_search with do_init_search), FAST_DIAMOND 8,
 * FAST_BIGDIA 9, VFAST_DIAMOND 10 (BIGDIA sites, do_init_search 0, start
 * scale clamps of :1291-1316), any mv cost (cost: HOST pointer to the
 * parameters), the downsampled-SAD recheck, and -- when cost_lists (device,
 * int32 [njobs][5]) is not NULL -- the cost list the reference returns for
 * the sub-pel search (calc_int_sad_list: centre, left, bottom, right, top;
 * INT_MAX where out of range); passing a cost list changes the BIGDIA-family
 * walk exactly as in the reference (last_s).  Returns 0, -1 bad step_param,
 * -2 bad cost parameters, -3 unsupported w x h, -4 unsupported method. */
int lavish_full_pixel_search_batch(const uint8_t *src, int src_stride,
                                   const uint8_t *ref, int ref_stride, int w,
                                   int h, const LavishDiamondJob *jobs,
                                   int njobs, int search_method, int step_param,
                                   const LavishMvCostParams *cost,
                                   int use_downsampled_sad,
                                   LavishDiamondResult *out, int32_t *cost_lists,
                                   void *stream);

/* Candidate-row layout of the reference buffer for the full-pel searches
 * (the build's own addition, no reference counterpart; results are
 * identical with or without it).  The searches read, per candidate, rows
 * y, y + 2, ... (downsampled SAD) of a w <= 16 byte segment at any column:
 * in the linear plane every such row is a separate cache line.  The tiled
 * copy splits the buffer's rows by parity (two fields) and each field into
 * 32-byte-wide column strips starting every 16 bytes (strip k holds bytes
 * [16k, 16k + 32) of every field row, consecutive field rows 32 bytes
 * apart), so a 16-byte segment lies in one strip and a downsampled 16-row
 * candidate in 2-3 cache lines instead of 8.  2x the buffer's bytes.
 *   rows: rows of the whole buffer (all reference planes stacked, stride
 *   `ref_stride`); the tiled copy must be rebuilt when the buffer changes. */
typedef struct LavishRefTiles {
  const uint8_t *data; /* device; lavish_ref_tiles_bytes(stride, rows) bytes */
  int64_t field_bytes; /* bytes of one field (the odd field follows the even) */
  int32_t field_rows;  /* (rows + 1) / 2 */
  int32_t stride;      /* the linear buffer's stride (= ref_stride) */
} LavishRefTiles;
int64_t lavish_ref_tiles_bytes(int stride, int rows);
/* Fills tiles->data (caller-allocated, device) from the linear buffer and
 * sets the other fields; asynchronous on `stream`.  -1 on bad arguments or
 * a copy of 2 GiB or more. */
int lavish_ref_tiles_build(const uint8_t *ref, int stride, int rows, uint8_t *data,
                           LavishRefTiles *tiles, void *stream);
/* lavish_full_pixel_search_batch reading candidate rows from the tiled copy
 * of the same `ref` buffer (w <= 16; other sizes, or tiles == NULL, run the
 * linear form).  Same results. */
int lavish_full_pixel_search_batch_tiled(const uint8_t *src, int src_stride,
                                         const uint8_t *ref, int ref_stride,
                                         const LavishRefTiles *tiles, int w, int h,
                                         const LavishDiamondJob *jobs, int njobs,
                                         int search_method, int step_param,
                                         const LavishMvCostParams *cost,
                                         int use_downsampled_sad,
                                         LavishDiamondResult *out,
                                         int32_t *cost_lists, void *stream);

/* The mesh fields of FULLPEL_MOTION_SEARCH_PARAMS (av1/encoder/mcomp.h:
 * 114-123), with the pattern set the search reads
 * (mesh_patterns[is_intra_mode]: sf->mv_sf.mesh_patterns or
 * intrabc_mesh_patterns, speed_features.c:25-44,2292-2308). */
typedef struct LavishMeshParams {
  int32_t run_mesh_search;
  int32_t force_mesh_thresh;
  int32_t prune_mesh_search;
  int32_t mesh_search_mv_diff_threshold;
  int32_t fine_search_interval;
  int32_t is_intra_mode;
  int32_t range[4]; /* MESH_PATTERN range / interval per step (MAX_MESH_STEP 4) */
  int32_t interval[4];
} LavishMeshParams;
/* lavish_full_pixel_search_batch[_tiled] followed by the exhaustive mesh
 * refinement of av1_full_pixel_search (mcomp.c:1818-1838, 1875-1893 ->
 * full_pixel_exhaustive :1603-1680 -> exhaustive_mesh_search :1529-1601):
 * per job, when run_mesh_search or (NSTEP / NSTEP_8PT) the variance exceeds
 * force_mesh_thresh >> (10 - mi_size_wide_log2 - mi_size_high_log2), unless
 * pruned (not intra, the search moved <= mesh_search_mv_diff_threshold),
 * the mesh passes around the search's best with the search's sdf; its var
 * cost replaces the result when smaller, and the cost list (when
 * cost_lists) is the one around the mesh's best either way, as the reference
 * writes it.  An illegal first pattern (range outside [7, 256], interval
 * outside [1, range]) makes the mesh a no-op, as in the reference.  mesh:
 * HOST pointer (NULL: no mesh); tiles may be NULL.  Same returns as
 * lavish_full_pixel_search_batch, and -6 when a later pass the walk can
 * reach has an interval < 1. */
int lavish_full_pixel_search_batch_mesh(const uint8_t *src, int src_stride,
                                        const uint8_t *ref, int ref_stride,
                                        const LavishRefTiles *tiles, int w, int h,
                                        const LavishDiamondJob *jobs, int njobs,
                                        int search_method, int step_param,
                                        const LavishMvCostParams *cost,
                                        int use_downsampled_sad,
                                        const LavishMeshParams *mesh,
                                        LavishDiamondResult *out, int32_t *cost_lists,
                                        void *stream);

/* C2 and the C3 search in one launch: lavish_txq_frame(residual, ...) and
 * lavish_full_pixel_search_batch_tiled(src, ..., 16, 16, jobs, njobs,
 * DIAMOND, ...) with the same results, run as one grid (the 64-point sizes
 * and the 32-point class of the transform first, as lavish_txq_frame runs
 * them; then the <= 16-point class's workgroups and the search's job groups
 * interleaved in the dispatch order, a search unit of 8 workgroups every
 * `every` units from the start).  The search must be the 16x16 DIAMOND with
 * a tiled reference copy.  -6: every < 1.  No reference counterpart: the
 * reference runs the two on the encoder's threads. */
int lavish_txq_frame_search(const int16_t *residual, int stride, int width, int height,
                            uint32_t size_mask, const uint32_t *type_masks, int bit_depth,
                            int quant_kind, const LavishQuantParams *qp,
                            int32_t *const *qcoeff, int32_t *const *dqcoeff,
                            uint16_t *const *eob, const uint8_t *src, int src_stride,
                            const uint8_t *ref, int ref_stride, const LavishRefTiles *tiles,
                            const LavishDiamondJob *jobs, int njobs, int step_param,
                            const LavishMvCostParams *cost, int use_downsampled_sad,
                            LavishDiamondResult *out, int32_t *cost_lists, int every,
                            void *stream);

/* Process-wide cap on the workgroups of the 16x16 DIAMOND search of
 * lavish_full_pixel_search_batch[_tiled] (rounded up to 8; 0 = no cap, one
 * workgroup per 32 jobs).  A scheduling knob for running the search beside
 * another stream's work (the search holds fewer CU slots and runs longer);
 * results do not depend on it.  Default 0; -1 for a
 * negative value.  No reference counterpart (the reference's search runs on
 * the encoder's threads). */
int lavish_set_search_workgroup_cap(int workgroups);

/* How a capped 16x16 DIAMOND search deals its 8-job wave units: 1 (default)
 * every wave pulls its next unit from one of 8 queues (one per XCD label
 * blockIdx % 8, the label's units a contiguous range of blocks); 0 the
 * static grid-stride over virtual workgroups.  Results do not depend on it;
 * -1 for another value.  No reference counterpart. */
int lavish_set_search_schedule(int queued);

/* ---- sub-pixel refinement ------------------------
 * av1_find_best_sub_pixel_tree_pruned_more (av1/encoder/mcomp.c:2907-2981;
 * subpel_search_method SUBPEL_TREE_PRUNED_MORE, speed >= 4) without a cost
 * list or a repeated-mv list, unscaled reference: setup_center_error at the
 * start, then two_level_checks_fast at half, quarter (forced_stop <
 * HALF_PEL) and eighth pel (allow_hp && forced_stop == EIGHTH_PEL), every
 * check check_better_fast with svf = aom_sub_pixel_variance (bilinear) +
 * mv_err_cost_.  8-bit planes.  One job per (block, reference): offsets as
 * LavishDiamondJob, start / ref mv and the SubpelMvLimits
 * (av1_set_subpel_mv_search_range, mcomp.h:357-373) in 1/8 pel.  The
 * search reads up to H+1 rows and W+5 bytes per row from the floor of every
 * in-range candidate.  forced_stop: 0 EIGHTH_PEL .. 3 FULL_PEL;
 * iters_per_step 1 or 2; mv_cost_type as lavish_diamond_search_batch. */
typedef struct LavishSubpelJob {
  int64_t src_off, ref_off;
  int16_t start_row, start_col;    /* full-pel best x 8 */
  int16_t ref_mv_row, ref_mv_col;
  int16_t col_min, col_max, row_min, row_max;
} LavishSubpelJob;

typedef struct LavishSubpelResult {
  int16_t best_row, best_col;      /* 1/8 pel */
  uint32_t besterr;                /* variance + mv cost of the best mv */
  int32_t distortion;              /* its variance */
  uint32_t sse;
} LavishSubpelResult;

int lavish_subpel_search_batch(const uint8_t *src, int src_stride,
                               const uint8_t *ref, int ref_stride, int w, int h,
                               const LavishSubpelJob *jobs, int njobs,
                               int forced_stop, int allow_hp,
                               int iters_per_step, int mv_cost_type,
                               LavishSubpelResult *out, void *stream);

/* The same, chained on the device after lavish_diamond_search_batch: job j
 * starts at fullpel[j].best_{row,col} x 8 (the jobs' start fields are
 * ignored), so the full-pel and sub-pel searches of a frame need no host
 * round trip. */
int lavish_subpel_search_after_diamond(const uint8_t *src, int src_stride,
                                       const uint8_t *ref, int ref_stride, int w,
                                       int h, const LavishSubpelJob *jobs,
                                       const LavishDiamondResult *fullpel,
                                       int njobs, int forced_stop, int allow_hp,
                                       int iters_per_step, int mv_cost_type,
                                       LavishSubpelResult *out, void *stream);

/* The general form: subpel_search_method (SUBPEL_SEARCH_METHODS,
 * mcomp_structs.h) 0 SUBPEL_TREE (av1_find_best_sub_pixel_tree,
 * mcomp.c:3128-3200, with subpel_search_type USE_2_TAPS_ORIG: the svf error,
 * first_level_check_fast + second_level_check_v2 per level; no cost list),
 * 1 SUBPEL_TREE_PRUNED (av1_find_best_sub_pixel_tree_pruned,
 * mcomp.c:2992-3126) or 2 SUBPEL_TREE_PRUNED_MORE (:2907-2990); any mv cost
 * (cost: HOST pointer, tables on the device, as for
 * lavish_full_pixel_search_batch -- the hp tables when allow_hp); cost_lists
 * (device int32 [njobs][5] or NULL): the full-pel search's cost lists, which
 * steer the first (half-pel) step exactly as in the reference.  fullpel
 * (device, or NULL to use the jobs' start fields): start = its best x 8.
 * Returns 0, -1 bad forced_stop, -2 bad cost parameters, -3 unsupported
 * w x h, -4 bad iters_per_step, -6 unsupported method. */
int lavish_find_best_sub_pixel_tree_batch(
    const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, int w,
    int h, const LavishSubpelJob *jobs, const LavishDiamondResult *fullpel,
    int njobs, int subpel_search_method, int forced_stop, int allow_hp,
    int iters_per_step, const LavishMvCostParams *cost, const int32_t *cost_lists,
    LavishSubpelResult *out, void *stream);
/* The same with var_params.subpel_search_type (SUBPEL_SEARCH_TYPE,
 * av1/common/filter.h:45-50: 0 USE_2_TAPS_ORIG, 1 USE_2_TAPS, 2 USE_4_TAPS,
 * 3 USE_8_TAPS; else -7).  SUBPEL_TREE with a type other than
 * USE_2_TAPS_ORIG ranks by upsampled_pref_error (av1/encoder/mcomp.c:
 * 2402-2491, check_better / first_level_check / second_level_check_v2's
 * check_better branch) -- aom_upsampled_pred_c's prediction
 * (av1/encoder/reconinter_enc.c:424-496, unscaled reference) -- which for
 * USE_2_TAPS equals the bilinear svf.  The pruned methods take the svf for
 * every type (check_better_fast on an unscaled reference), as in the
 * reference.  The speed-0..3 default is SUBPEL_TREE with USE_8_TAPS
 * (speed_features.c:1929-1931). */
int lavish_find_best_sub_pixel_tree_batch_ex(
    const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, int w,
    int h, const LavishSubpelJob *jobs, const LavishDiamondResult *fullpel,
    int njobs, int subpel_search_method, int subpel_search_type, int forced_stop,
    int allow_hp, int iters_per_step, const LavishMvCostParams *cost,
    const int32_t *cost_lists, LavishSubpelResult *out, void *stream);

/* ---- Inter prediction -----------------------------
 * av1_enc_build_one_inter_predictor (av1/encoder/reconinter_enc.c:47-51) for
 * a batch of single-reference translational blocks: init_subpel_params
 * (av1/common/reconinter.h:131-165, unscaled, border clamp), the block-size
 * filter choice (filter.h:253-259) and convolve_2d_facade_single
 * (av1/common/convolve.c:614-634 / highbd :1106-1128).
 *   ref: plane origin (buf0) of the reference, with the reference's
 *        AOM_BORDER_IN_PIXELS >> ss border around it (per direction; 12-tap
 *        MULTITAP_SHARP2 reads one more row / column at the clamp extremes,
 *        as the C does); ref_width / height: the plane's size (the clamp
 *        window).
 *   w, h: 2..128 (powers of two); ss_x / ss_y: the plane's subsampling.
 *   highbd 0: u8 planes (bit_depth 8); 1: u16 planes, bit_depth 8/10/12.
 * dst[job.dst_off + y * dst_stride + x] receives the prediction. */
typedef struct LavishInterPredJob {
  int64_t ref_off;             /* element offset of this job's reference plane origin */
  int64_t dst_off;             /* element offset of the block's first output pixel */
  int32_t pix_row, pix_col;    /* block position in the plane (pixels) */
  int16_t mv_row, mv_col;      /* MV, 1/8 luma pel */
  uint8_t filter_x, filter_y;  /* InterpFilter: 0 REGULAR 1 SMOOTH 2 SHARP 3 BILINEAR 4 SHARP2 */
  uint8_t pad[2];
} LavishInterPredJob;

int lavish_build_inter_pred_batch(const void *ref, int ref_stride, int ref_width,
                                  int ref_height, int ss_x, int ss_y, int w, int h,
                                  const LavishInterPredJob *jobs, int njobs,
                                  void *dst, int dst_stride, int bit_depth,
                                  int highbd, void *stream);
/* The interpolation kernels the library itself uses, as data:
 * av1_get_interp_filter_params_with_block_size(interp_filter, size)
 * (av1/common/filter.h:253-259) -> out[16][taps] (one row per 1/16 phase),
 * returns taps (8, or 12 for MULTITAP_SHARP2), -1 on bad arguments.  For
 * callers that build LavishInterpFilterParams (the RTCD convolve shims, the
 * compound batch) without the reference's tables at hand.  Host only. */
int lavish_interp_kernels(int interp_filter, int size, int16_t *out);
/* The same with job j's mv taken from a sub-pel search result (chained on
 * the device after lavish_subpel_search_batch / _after_diamond). */
int lavish_build_inter_pred_after_subpel(const void *ref, int ref_stride,
                                         int ref_width, int ref_height, int ss_x,
                                         int ss_y, int w, int h,
                                         const LavishInterPredJob *jobs,
                                         const LavishSubpelResult *mvs, int njobs,
                                         void *dst, int dst_stride, int bit_depth,
                                         int highbd, void *stream);

/* ---- TPL block transform leg ----------------------
 * For every full bsize x bsize block of a width x height frame (raster
 * order; bsize 8 / 16 / 32 with TX = the block, tpl_model.c uses 16): the
 * inter cost of each of nrefs predictions (tpl_get_satd_cost,
 * av1/encoder/tpl_model.c:199-210: subtract, av1_quick_txfm DCT_DCT,
 * aom_satd), the cheapest reference (lowest cost, earlier reference on
 * ties), and on its prediction txfm_quant_rdcost (:225-247):
 * get_quantize_error (:98-135, quantize_fp with qp built for
 * LAVISH_QUANT_FP, block error and sse >> (TX_32X32 ? 0 : 2), each >= 1),
 * rate_estimator (:212-223) and recon = prediction + the inverse transform.
 *   src: plane origin, src_stride elements; preds: reference k's
 *   prediction plane at preds + k * pred_plane elements (same geometry);
 *   recon: output plane.  8-bit: uint8_t planes; 10 / 12-bit: uint16_t.
 *   ref_costs (device, optional): int32 [nblocks][nrefs] inter costs.
 * Returns 0, or -1 bad bsize, -2 bad bit_depth, -3 NULL argument, -4 bad
 * nrefs / preds, -5 bad geometry. */
typedef struct LavishTplBlock {
  int32_t best_ref;    /* index of the cheapest prediction */
  int32_t inter_cost;  /* its satd cost */
  int32_t rate_cost;   /* rate_estimator, << AV1_PROB_COST_SHIFT */
  int32_t eob;
  int64_t recon_error; /* get_quantize_error's recon_error */
  int64_t sse;         /* and sse */
} LavishTplBlock;

int lavish_tpl_block_batch(const void *src, int src_stride, const void *preds,
                           int64_t pred_plane, int pred_stride, int nrefs,
                           int width, int height, int bsize, int bit_depth,
                           const LavishQuantParams *qp, LavishTplBlock *out,
                           void *recon, int recon_stride, int32_t *ref_costs,
                           void *stream);

/* ---- TPL motion search with start-mv candidates --
 * Replaces the per-reference loop of mode_estimation
 * (av1/encoder/tpl_model.c:632-743) for a frame of 16x16 TPL blocks
 * (set_tpl_stats_block_size, :136-144): centre mvs = zero, then the above,
 * left and above-right blocks' tpl mvs of the same reference unless
 * is_alike_mv (:319-333, threshold by skip_alike_starting_mv), the optional
 * third-pass mv in slot 0 (:687-703); with prune_starting_mv the full-SAD
 * ranking at the clamped full-pel centres and the cut (:705-728); then
 * motion_estimation (:249-303) per centre -- av1_full_pixel_search with
 * ref_mv = the centre, tpl_sf.search_method, step_param =
 * AOMMIN(reduce_first_step_size, 9), the caller's mv costs and
 * use_downsampled_sad, a cost list when cost_lists != NULL -- keeping the
 * lowest sub-pel error (strict <).  subpel_force_stop must be FULL_PEL
 * (speed >= 5, speed_features.c:1212-1216; else -6): the tpl mv is the
 * full-pel best x 8.  Blocks depend on their finished neighbours: the call
 * runs as a device wavefront (one wave per reference x block row).
 *   jobs: [nrefs][rows * cols] LavishDiamondJob in raster order (offsets;
 *     limits = x->mv_limits of av1_set_mv_limits with tpl border_in_pixels;
 *     start / ref_mv fields ignored); the src / ref planes as for
 *     lavish_full_pixel_search_batch.
 *   third_pass_mvs: NULL or int_mv [nrefs][rows * cols] (INVALID_MV =
 *     0x80008000 for none).
 *   out (device): mvs int_mv [nrefs][rows * cols] = tpl_stats->mv[rf_idx]
 *     (row in the low 16 bits); out: the winning full-pel search's
 *     LavishDiamondResult; cost_lists (or NULL) its cost list; centers (or
 *     NULL) its centre mv (int_mv).
 *   sync: device int32 scratch of lavish_tpl_motion_sync_ints(nrefs, rows)
 *     entries (zeroed by the call); after the stream drains, sync[1] != 0
 *     means a wait timed out (results invalid).  mvs is filled with
 *     INVALID_MV first and each entry published once, when final.
 * Returns 0, -1 bad geometry / parameters, -2 bad costs, -4 bad method,
 * -6 subpel_force_stop != FULL_PEL. */
typedef struct LavishTplMvParams {
  int search_method;          /* tpl_sf.search_method (SEARCH_METHODS value) */
  int step_param;             /* tpl_sf.reduce_first_step_size */
  int use_downsampled_sad;    /* mv_sf.use_downsampled_sad */
  int prune_starting_mv;      /* tpl_sf.prune_starting_mv, 0..3 */
  int skip_alike_starting_mv; /* tpl_sf.skip_alike_starting_mv, 0..2 */
  int subpel_force_stop;      /* tpl_sf.subpel_force_stop: FULL_PEL (3) */
} LavishTplMvParams;

int64_t lavish_tpl_motion_sync_ints(int nrefs, int rows);
int lavish_tpl_motion_search(const uint8_t *src, int src_stride,
                             const uint8_t *ref, int ref_stride,
                             const LavishDiamondJob *jobs, int cols, int rows,
                             int nrefs, const LavishTplMvParams *p,
                             const LavishMvCostParams *cost,
                             const int32_t *third_pass_mvs, int32_t *mvs,
                             LavishDiamondResult *out, int32_t *cost_lists,
                             int32_t *centers, int32_t *sync, void *stream);

/* ---- TX-type pruning features ---------------------
 * Every full bw x bh block of an int16 residual plane (raster order):
 * av1_get_horver_correlation_full (av1/encoder/rdopt.c:514-609) -> hcorr /
 * vcorr[block] (bw, bh in 2..128). */
int lavish_horver_correlation_batch(const int16_t *residual, int stride,
                                    int width, int height, int bw, int bh,
                                    float *hcorr, float *vcorr, void *stream);
/* prune_tx_2D's two neural-net inputs (av1/encoder/tx_search.c:1516-1529)
 * per tx_size block: hfeatures[block][16] = get_energy_distribution_finer's
 * column projection (tx_search.c:1411-1473) in [0, n-1) and hcorr at n-1
 * (n = w <= 8 ? w : w / 2); vfeatures likewise for rows; unused entries 0.
 * tx sizes up to 32x32 (else -2).  Bit-exact single precision. */
int lavish_tx_prune_features_batch(const int16_t *residual, int stride,
                                   int width, int height, int tx_size,
                                   float *hfeatures, float *vfeatures,
                                   void *stream);

/* Layout of NN_CONFIG (av1/encoder/ml.h:24-34): a caller passes the
 * reference's own models (e.g. av1_tx_type_nnconfig_map_hor[tx_size]).
 * Models are uploaded once per distinct content. */
typedef struct LavishNNConfig {
  int num_inputs;
  int num_outputs;
  int num_hidden_layers;
  int num_hidden_nodes[10];
  const float *weights[11];
  const float *bias[11];
} LavishNNConfig;

/* prune_tx_2D (av1/encoder/tx_search.c:1487-1641) for every full tx_size
 * block of an int16 residual plane (raster order): features, the two nets
 * (av1_nn_predict_c with reduce_prec), av1_nn_fast_softmax_16_c, the
 * adaptive threshold of (tx_set_type, prune_2d_txfm_mode), the sorting
 * network and the TX_TYPE_PRUNE_4/5 cumulative cut.
 *   allowed_in[block] (or allowed_default for every block when NULL): the
 *   incoming allowed_tx_mask; allowed_out[block]: the pruned mask;
 *   txk_map[block][16]: the search order (TX_TYPE values, 255 unused),
 *   identity where prune_tx_2D leaves it untouched (tx set other than
 *   ALL16 / DTT9_IDTX_1DDCT, mode 0, or nn_hor / nn_ver NULL).
 * Float results follow the C functions bit for bit.  -2: tx size or
 * threshold outside the reference's tables; -3: model shape unsupported
 * (outputs != 4, > 16 inputs, differing depths, > 128 nodes). */
int lavish_prune_tx_2d_batch(const int16_t *residual, int stride, int width,
                             int height, int tx_size, int tx_set_type,
                             int prune_2d_txfm_mode, const LavishNNConfig *nn_hor,
                             const LavishNNConfig *nn_ver,
                             const uint16_t *allowed_in, uint16_t allowed_default,
                             uint16_t *allowed_out, uint8_t *txk_map,
                             void *stream);
/* av1_nn_predict_c (av1/encoder/ml.c:31-70) for n input vectors
 * (inputs[n][num_inputs] -> outputs[n][num_outputs], device memory). */
int lavish_nn_predict_batch(const float *inputs, const LavishNNConfig *nn_config,
                            int reduce_prec, float *outputs, int n, void *stream);

/* ------------------------------------------------------------------------ */
/* Per-call RTCD shims (host pointers)                                      */
/* ------------------------------------------------------------------------ */
/* av1_fwd_txfm2d_WxH (av1/common/av1_rtcd_defs.pl:358-399); the 64-point
 * sizes reproduce the reference's in-place zero + re-pack of the whole W*H
 * output buffer (av1/encoder/av1_fwd_txfm2d.c:240-311). */
#define LAVISH_FWD2D(w, h)                                                   \
  void av1_fwd_txfm2d_##w##x##h##_hip(const int16_t *input, int32_t *output, \
                                      int stride, uint8_t tx_type, int bd);
LAVISH_FWD2D(4, 4)
LAVISH_FWD2D(64, 64)
LAVISH_FWD2D(32, 64)
LAVISH_FWD2D(64, 32)
LAVISH_FWD2D(16, 64)
LAVISH_FWD2D(64, 16)
LAVISH_FWD2D(8, 8)
LAVISH_FWD2D(16, 16)
LAVISH_FWD2D(32, 32)
LAVISH_FWD2D(4, 8)
LAVISH_FWD2D(8, 4)
LAVISH_FWD2D(8, 16)
LAVISH_FWD2D(16, 8)
LAVISH_FWD2D(16, 32)
LAVISH_FWD2D(32, 16)
LAVISH_FWD2D(4, 16)
LAVISH_FWD2D(16, 4)
LAVISH_FWD2D(8, 32)
LAVISH_FWD2D(32, 8)
#undef LAVISH_FWD2D

/* av1_lowbd_fwd_txfm (av1/common/av1_rtcd_defs.pl:355,
 * av1/encoder/hybrid_fwd_txfm.c:244); a lossless TX_4X4 takes av1_fwht4x4 */
void av1_lowbd_fwd_txfm_hip(const int16_t *src_diff, int32_t *coeff,
                            int diff_stride, LavishTxfmParam *txfm_param);
/* lossless Walsh-Hadamard (av1/common/av1_rtcd_defs.pl:351,217-218;
 * hybrid_fwd_txfm.c:24-76, av1_inv_txfm2d.c:20-107); tagged u16 dest */
void av1_fwht4x4_hip(const int16_t *input, int32_t *output, int stride);
void av1_highbd_iwht4x4_16_add_hip(const int32_t *input, uint8_t *dest,
                                   int dest_stride, int bd);
void av1_highbd_iwht4x4_1_add_hip(const int32_t *input, uint8_t *dest,
                                  int dest_stride, int bd);
/* BitDepthInfo of av1/common/blockd.h:952-960 */
typedef struct LavishBitDepthInfo {
  int bit_depth;
  int use_highbitdepth_buf;
} LavishBitDepthInfo;
/* av1_quick_txfm (av1/encoder/hybrid_fwd_txfm.c:315-336, the TPL model's
 * transform): aom_hadamard_{4x4..32x32} when use_hadamard, else the DCT_DCT
 * forward transform of tx_size. */
void av1_quick_txfm_hip(int use_hadamard, uint8_t tx_size,
                        LavishBitDepthInfo bd_info, const int16_t *src_diff,
                        int src_stride, int32_t *coeff);

/* quantizers (aom_dsp/aom_dsp_rtcd_defs.pl:655-694,
 * av1/common/av1_rtcd_defs.pl:334-344,428) */
#define LAVISH_QUANT_PROTO(name)                                              \
  void name(const int32_t *coeff_ptr, intptr_t n_coeffs,                      \
            const int16_t *zbin_ptr, const int16_t *round_ptr,                \
            const int16_t *quant_ptr, const int16_t *quant_shift_ptr,         \
            int32_t *qcoeff_ptr, int32_t *dqcoeff_ptr,                        \
            const int16_t *dequant_ptr, uint16_t *eob_ptr,                    \
            const int16_t *scan, const int16_t *iscan);
LAVISH_QUANT_PROTO(av1_quantize_fp_hip)
LAVISH_QUANT_PROTO(av1_quantize_fp_32x32_hip)
LAVISH_QUANT_PROTO(av1_quantize_fp_64x64_hip)
LAVISH_QUANT_PROTO(aom_quantize_b_hip)
LAVISH_QUANT_PROTO(aom_quantize_b_32x32_hip)
LAVISH_QUANT_PROTO(aom_quantize_b_64x64_hip)
LAVISH_QUANT_PROTO(aom_highbd_quantize_b_hip)
LAVISH_QUANT_PROTO(aom_highbd_quantize_b_32x32_hip)
LAVISH_QUANT_PROTO(aom_highbd_quantize_b_64x64_hip)
#undef LAVISH_QUANT_PROTO
void av1_highbd_quantize_fp_hip(const int32_t *coeff_ptr, intptr_t count,
                                const int16_t *zbin_ptr,
                                const int16_t *round_ptr,
                                const int16_t *quant_ptr,
                                const int16_t *quant_shift_ptr,
                                int32_t *qcoeff_ptr, int32_t *dqcoeff_ptr,
                                const int16_t *dequant_ptr, uint16_t *eob_ptr,
                                const int16_t *scan, const int16_t *iscan,
                                int log_scale);

/* ---- inverse transform shims (av1/common/av1_rtcd_defs.pl:137-243) ---- */
#define LAVISH_TX_SIZES_ALL(X)                                               \
  X(4, 4) X(8, 8) X(16, 16) X(32, 32) X(64, 64) X(4, 8) X(8, 4) X(8, 16)    \
  X(16, 8) X(16, 32) X(32, 16) X(32, 64) X(64, 32) X(4, 16) X(16, 4)        \
  X(8, 32) X(32, 8) X(16, 64) X(64, 16)
#define LAVISH_INV2D(w, h)                                                   \
  void av1_inv_txfm2d_add_##w##x##h##_hip(const int32_t *input,             \
                                          uint16_t *output, int stride,     \
                                          uint8_t tx_type, int bd);
LAVISH_TX_SIZES_ALL(LAVISH_INV2D)
#undef LAVISH_INV2D
void av1_inv_txfm_add_hip(const int32_t *dqcoeff, uint8_t *dst, int stride,
                          const LavishTxfmParam *txfm_param);
void av1_highbd_inv_txfm_add_hip(const int32_t *input, uint8_t *dest,
                                 int stride,
                                 const LavishTxfmParam *txfm_param);
#define LAVISH_HBD_INV(w, h)                                                 \
  void av1_highbd_inv_txfm_add_##w##x##h##_hip(                             \
      const int32_t *input, uint8_t *dest, int stride,                      \
      const LavishTxfmParam *txfm_param);
LAVISH_HBD_INV(4, 4) LAVISH_HBD_INV(8, 8) LAVISH_HBD_INV(4, 8)
LAVISH_HBD_INV(8, 4) LAVISH_HBD_INV(4, 16) LAVISH_HBD_INV(16, 4)
LAVISH_HBD_INV(8, 16) LAVISH_HBD_INV(16, 8) LAVISH_HBD_INV(16, 32)
LAVISH_HBD_INV(32, 16) LAVISH_HBD_INV(32, 32) LAVISH_HBD_INV(32, 64)
LAVISH_HBD_INV(64, 32) LAVISH_HBD_INV(64, 64) LAVISH_HBD_INV(8, 32)
LAVISH_HBD_INV(32, 8) LAVISH_HBD_INV(16, 64) LAVISH_HBD_INV(64, 16)
#undef LAVISH_HBD_INV

/* ---- pixel shims ---------------------------------------------------------
 * @encoder_block_sizes of aom_dsp/aom_dsp_rtcd_defs.pl:42-58. */
#define LAVISH_ENCODER_BLOCK_SIZES(X)                                     \
  X(128, 128) X(128, 64) X(64, 128) X(64, 64) X(64, 32) X(32, 64)         \
  X(32, 32) X(32, 16) X(16, 32) X(16, 16) X(16, 8) X(8, 16) X(8, 8)       \
  X(8, 4) X(4, 8) X(4, 4) X(4, 16) X(16, 4) X(8, 32) X(32, 8) X(16, 64)   \
  X(64, 16)

/* aom_dsp_rtcd_defs.pl:764-766,1003-1006 (lowbd) and :882-884,1139-1141
 * (highbd) */
#define LAVISH_SAD_PROTOS(w, h)                                               \
  unsigned int aom_sad##w##x##h##_hip(const uint8_t *src_ptr, int src_stride, \
                                      const uint8_t *ref_ptr, int ref_stride); \
  unsigned int aom_sad_skip_##w##x##h##_hip(const uint8_t *src_ptr,           \
                                            int src_stride,                   \
                                            const uint8_t *ref_ptr,           \
                                            int ref_stride);                  \
  unsigned int aom_sad##w##x##h##_avg_hip(                                    \
      const uint8_t *src_ptr, int src_stride, const uint8_t *ref_ptr,         \
      int ref_stride, const uint8_t *second_pred);                            \
  void aom_sad##w##x##h##x4d_hip(const uint8_t *src_ptr, int src_stride,      \
                                 const uint8_t *const ref_ptr[4],             \
                                 int ref_stride, uint32_t sad_array[4]);      \
  void aom_sad##w##x##h##x3d_hip(const uint8_t *src_ptr, int src_stride,      \
                                 const uint8_t *const ref_ptr[4],             \
                                 int ref_stride, uint32_t sad_array[4]);      \
  void aom_sad##w##x##h##x4d_avg_hip(                                         \
      const uint8_t *src_ptr, int src_stride,                                 \
      const uint8_t *const ref_ptr[4], int ref_stride,                        \
      const uint8_t *second_pred, uint32_t sad_array[4]);                     \
  void aom_sad_skip_##w##x##h##x4d_hip(const uint8_t *src_ptr,                \
                                       int src_stride,                        \
                                       const uint8_t *const ref_ptr[4],       \
                                       int ref_stride, uint32_t sad_array[4]); \
  unsigned int aom_highbd_sad##w##x##h##_hip(                                 \
      const uint8_t *src_ptr, int src_stride, const uint8_t *ref_ptr,         \
      int ref_stride);                                                        \
  unsigned int aom_highbd_sad_skip_##w##x##h##_hip(                           \
      const uint8_t *src_ptr, int src_stride, const uint8_t *ref_ptr,         \
      int ref_stride);                                                        \
  unsigned int aom_highbd_sad##w##x##h##_avg_hip(                             \
      const uint8_t *src_ptr, int src_stride, const uint8_t *ref_ptr,         \
      int ref_stride, const uint8_t *second_pred);                            \
  void aom_highbd_sad##w##x##h##x4d_hip(const uint8_t *src_ptr,               \
                                        int src_stride,                       \
                                        const uint8_t *const ref_ptr[],       \
                                        int ref_stride, uint32_t *sad_array); \
  void aom_highbd_sad##w##x##h##x3d_hip(const uint8_t *src_ptr,               \
                                        int src_stride,                       \
                                        const uint8_t *const ref_ptr[],       \
                                        int ref_stride, uint32_t *sad_array); \
  void aom_highbd_sad_skip_##w##x##h##x4d_hip(                                \
      const uint8_t *src_ptr, int src_stride,                                 \
      const uint8_t *const ref_ptr[], int ref_stride, uint32_t *sad_array);

/* aom_dsp_rtcd_defs.pl:1363-1365 (lowbd) and :1476-1478 (highbd 8/10/12) */
#define LAVISH_VAR_PROTOS_BD(pre, w, h)                                       \
  unsigned int pre##variance##w##x##h##_hip(const uint8_t *src_ptr,           \
                                            int source_stride,                \
                                            const uint8_t *ref_ptr,           \
                                            int ref_stride, uint32_t *sse);   \
  uint32_t pre##sub_pixel_variance##w##x##h##_hip(                            \
      const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset,    \
      const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);                 \
  uint32_t pre##sub_pixel_avg_variance##w##x##h##_hip(                        \
      const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset,    \
      const uint8_t *ref_ptr, int ref_stride, uint32_t *sse,                  \
      const uint8_t *second_pred);
#define LAVISH_VAR_PROTOS(w, h)                  \
  LAVISH_VAR_PROTOS_BD(aom_, w, h)               \
  LAVISH_VAR_PROTOS_BD(aom_highbd_8_, w, h)      \
  LAVISH_VAR_PROTOS_BD(aom_highbd_10_, w, h)     \
  LAVISH_VAR_PROTOS_BD(aom_highbd_12_, w, h)

LAVISH_ENCODER_BLOCK_SIZES(LAVISH_SAD_PROTOS)
LAVISH_ENCODER_BLOCK_SIZES(LAVISH_VAR_PROTOS)

/* aom_dsp_rtcd_defs.pl:1303-1318,1326-1333 */
#define LAVISH_MSE_PROTOS(pre)                                                 \
  void pre##get16x16var_hip(const uint8_t *src_ptr, int source_stride,        \
                            const uint8_t *ref_ptr, int ref_stride,           \
                            unsigned int *sse, int *sum);                     \
  void pre##get8x8var_hip(const uint8_t *src_ptr, int source_stride,          \
                          const uint8_t *ref_ptr, int ref_stride,             \
                          unsigned int *sse, int *sum);                       \
  unsigned int pre##mse16x16_hip(const uint8_t *src_ptr, int source_stride,   \
                                 const uint8_t *ref_ptr, int recon_stride,    \
                                 unsigned int *sse);                          \
  unsigned int pre##mse16x8_hip(const uint8_t *src_ptr, int source_stride,    \
                                const uint8_t *ref_ptr, int recon_stride,     \
                                unsigned int *sse);                           \
  unsigned int pre##mse8x16_hip(const uint8_t *src_ptr, int source_stride,    \
                                const uint8_t *ref_ptr, int recon_stride,     \
                                unsigned int *sse);                           \
  unsigned int pre##mse8x8_hip(const uint8_t *src_ptr, int source_stride,     \
                               const uint8_t *ref_ptr, int recon_stride,      \
                               unsigned int *sse);
LAVISH_MSE_PROTOS(aom_)
LAVISH_MSE_PROTOS(aom_highbd_8_)
LAVISH_MSE_PROTOS(aom_highbd_10_)
LAVISH_MSE_PROTOS(aom_highbd_12_)

/* aom_dsp_rtcd_defs.pl:725-746 */
void aom_subtract_block_hip(int rows, int cols, int16_t *diff_ptr,
                            ptrdiff_t diff_stride, const uint8_t *src_ptr,
                            ptrdiff_t src_stride, const uint8_t *pred_ptr,
                            ptrdiff_t pred_stride);
void aom_highbd_subtract_block_hip(int rows, int cols, int16_t *diff_ptr,
                                   ptrdiff_t diff_stride,
                                   const uint8_t *src_ptr,
                                   ptrdiff_t src_stride,
                                   const uint8_t *pred_ptr,
                                   ptrdiff_t pred_stride);
int64_t aom_sse_hip(const uint8_t *a, int a_stride, const uint8_t *b,
                    int b_stride, int width, int height);
int64_t aom_highbd_sse_hip(const uint8_t *a8, int a_stride, const uint8_t *b8,
                           int b_stride, int width, int height);
uint64_t aom_sum_squares_2d_i16_hip(const int16_t *src, int stride, int width,
                                    int height);

/* aom_dsp_rtcd_defs.pl:1244-1278 */
void aom_hadamard_4x4_hip(const int16_t *src_diff, ptrdiff_t src_stride,
                          int32_t *coeff);
void aom_hadamard_8x8_hip(const int16_t *src_diff, ptrdiff_t src_stride,
                          int32_t *coeff);
void aom_hadamard_16x16_hip(const int16_t *src_diff, ptrdiff_t src_stride,
                            int32_t *coeff);
void aom_hadamard_32x32_hip(const int16_t *src_diff, ptrdiff_t src_stride,
                            int32_t *coeff);
void aom_highbd_hadamard_8x8_hip(const int16_t *src_diff,
                                 ptrdiff_t src_stride, int32_t *coeff);
void aom_highbd_hadamard_16x16_hip(const int16_t *src_diff,
                                   ptrdiff_t src_stride, int32_t *coeff);
void aom_highbd_hadamard_32x32_hip(const int16_t *src_diff,
                                   ptrdiff_t src_stride, int32_t *coeff);
int aom_satd_hip(const int32_t *coeff, int length);

/* aom_dsp_rtcd_defs.pl:1256-1263,1278 (int16 "low precision" forms) */
void aom_hadamard_lp_8x8_hip(const int16_t *src_diff, ptrdiff_t src_stride,
                             int16_t *coeff);
void aom_hadamard_lp_16x16_hip(const int16_t *src_diff, ptrdiff_t src_stride,
                               int16_t *coeff);
void aom_hadamard_lp_8x8_dual_hip(const int16_t *src_diff, ptrdiff_t src_stride,
                                  int16_t *coeff);
int aom_satd_lp_hip(const int16_t *coeff, int length);
/* aom_dsp_rtcd_defs.pl:770,731 */
uint64_t aom_sum_sse_2d_i16_hip(const int16_t *src, int src_stride, int width,
                                int height, int *sum);
void aom_get_blk_sse_sum_hip(const int16_t *data, int stride, int bw, int bh,
                             int *x_sum, int64_t *x2_sum);

/* av1/common/av1_rtcd_defs.pl:331 */
int64_t av1_block_error_lp_hip(const int16_t *coeff, const int16_t *dqcoeff,
                               intptr_t block_size);
/* av1/common/av1_rtcd_defs.pl:328,423 */
int64_t av1_block_error_hip(const int32_t *coeff, const int32_t *dqcoeff,
                            intptr_t block_size, int64_t *ssz);
int64_t av1_highbd_block_error_hip(const int32_t *coeff,
                                   const int32_t *dqcoeff,
                                   intptr_t block_size, int64_t *ssz, int bd);
/* av1_get_horver_correlation_full (av1/common/av1_rtcd_defs.pl:469) */
void av1_get_horver_correlation_full_hip(const int16_t *diff, int stride, int w,
                                         int h, float *hcorr, float *vcorr);

/* av1_nn_predict (av1/common/av1_rtcd_defs.pl:472) */
void av1_nn_predict_hip(const float *input_nodes, const LavishNNConfig *nn_config,
                        int reduce_prec, float *output);

/* Convolution (av1/common/av1_rtcd_defs.pl:565-575, aom_dsp_rtcd_defs.pl:449,461).
 * Layout mirrors of InterpFilterParams (av1/common/filter.h:105-109) and
 * ConvolveParams (av1/common/convolve.h:21-32). */
typedef struct LavishInterpFilterParams {
  const int16_t *filter_ptr;
  uint16_t taps;
  uint8_t interp_filter;
} LavishInterpFilterParams;
typedef struct LavishConvolveParams {
  int do_average;
  uint16_t *dst;
  int dst_stride;
  int round_0;
  int round_1;
  int plane;
  int is_compound;
  int use_dist_wtd_comp_avg;
  int fwd_offset;
  int bck_offset;
} LavishConvolveParams;
void av1_convolve_2d_sr_hip(const uint8_t *src, int src_stride, uint8_t *dst,
                            int dst_stride, int w, int h,
                            const LavishInterpFilterParams *filter_params_x,
                            const LavishInterpFilterParams *filter_params_y,
                            const int subpel_x_qn, const int subpel_y_qn,
                            LavishConvolveParams *conv_params);
void av1_convolve_x_sr_hip(const uint8_t *src, int src_stride, uint8_t *dst,
                           int dst_stride, int w, int h,
                           const LavishInterpFilterParams *filter_params_x,
                           const int subpel_x_qn, LavishConvolveParams *conv_params);
void av1_convolve_y_sr_hip(const uint8_t *src, int src_stride, uint8_t *dst,
                           int dst_stride, int w, int h,
                           const LavishInterpFilterParams *filter_params_y,
                           const int subpel_y_qn);
void av1_highbd_convolve_2d_sr_hip(const uint16_t *src, int src_stride,
                                   uint16_t *dst, int dst_stride, int w, int h,
                                   const LavishInterpFilterParams *filter_params_x,
                                   const LavishInterpFilterParams *filter_params_y,
                                   const int subpel_x_qn, const int subpel_y_qn,
                                   LavishConvolveParams *conv_params, int bd);
void av1_highbd_convolve_x_sr_hip(const uint16_t *src, int src_stride,
                                  uint16_t *dst, int dst_stride, int w, int h,
                                  const LavishInterpFilterParams *filter_params_x,
                                  const int subpel_x_qn,
                                  LavishConvolveParams *conv_params, int bd);
void av1_highbd_convolve_y_sr_hip(const uint16_t *src, int src_stride,
                                  uint16_t *dst, int dst_stride, int w, int h,
                                  const LavishInterpFilterParams *filter_params_y,
                                  const int subpel_y_qn, int bd);
void aom_convolve_copy_hip(const uint8_t *src, ptrdiff_t src_stride, uint8_t *dst,
                           ptrdiff_t dst_stride, int w, int h);
void aom_highbd_convolve_copy_hip(const uint16_t *src, ptrdiff_t src_stride,
                                  uint16_t *dst, ptrdiff_t dst_stride, int w, int h);


/* ---- affine warp --------------------------------
 * Replaces av1_warp_affine_c (av1/common/warped_motion.c:538-666) and
 * av1_highbd_warp_affine_c (:264-388) for a batch of prediction blocks of
 * one reference plane.  A job is one block: its warp matrix (wmmat[0..5])
 * and shear parameters (av1_get_shear_params), the block position p_col /
 * p_row / p_width / p_height in the predicted plane, the element offset of
 * the reference plane origin (ref_off: several planes may be stacked) and of
 * the block's top-left in pred / conv_dst.  conv_params: round_0, round_1,
 * is_compound, do_average, use_dist_wtd_comp_avg, fwd_offset, bck_offset as
 * the reference reads them (its dst / dst_stride are replaced by conv_dst /
 * dst_stride).  Device pointers; asynchronous on `stream`.  highbd: u16
 * samples (bit_depth 8/10/12), else u8 (bit_depth 8).  Returns 0, or < 0 on
 * rejected arguments. */
typedef struct LavishWarpJob {
  int32_t mat[6];
  int16_t alpha, beta, gamma, delta;
  int32_t p_col, p_row, p_width, p_height;
  int64_t ref_off;
  int64_t pred_off;
  int64_t dst_off;
} LavishWarpJob;
int lavish_warp_affine_batch(const void *ref, int width, int height, int stride, void *pred,
                             int p_stride, uint16_t *conv_dst, int dst_stride,
                             const LavishWarpJob *jobs, int njobs, int subsampling_x,
                             int subsampling_y, int bit_depth, int highbd,
                             const LavishConvolveParams *conv_params, void *stream);
/* av1_get_shear_params (warped_motion.c:218-247) on a host matrix: out =
 * alpha, beta, gamma, delta; returns 1 when the model is usable by the warp
 * filter, else 0. */
int lavish_get_shear_params(const int32_t *mat, int16_t *out);
/* av1/common/av1_rtcd_defs.pl:548,544 (per-call shims, host buffers) */
void av1_warp_affine_hip(const int32_t *mat, const uint8_t *ref, int width, int height,
                         int stride, uint8_t *pred, int p_col, int p_row, int p_width,
                         int p_height, int p_stride, int subsampling_x, int subsampling_y,
                         LavishConvolveParams *conv_params, int16_t alpha, int16_t beta,
                         int16_t gamma, int16_t delta);
void av1_highbd_warp_affine_hip(const int32_t *mat, const uint16_t *ref, int width,
                                int height, int stride, uint16_t *pred, int p_col, int p_row,
                                int p_width, int p_height, int p_stride, int subsampling_x,
                                int subsampling_y, int bd, LavishConvolveParams *conv_params,
                                int16_t alpha, int16_t beta, int16_t gamma, int16_t delta);


/* ---- compound (CONV_BUF) convolutions -----------
 * Replaces av1_dist_wtd_convolve_{2d_copy,x,y,2d}_c and the highbd forms
 * (av1/common/convolve.c:291-489,790-988) for a batch of w x h blocks
 * sharing the x / y filters (InterpFilterParams as the caller holds them:
 * host filter_ptr, taps <= 12) and the conv params (round_0, round_1,
 * do_average, use_dist_wtd_comp_avg, fwd_offset, bck_offset; its dst /
 * dst_stride are replaced by conv_dst / conv_stride).  Per block: the source
 * position (element offset of the block's integer position), the prediction
 * and CONV_BUF offsets and the sub-pel phases (1/16 pel), which choose the
 * path as convolve_2d_facade_compound does.  w, h <= 128.  Device pointers;
 * asynchronous on `stream`. */
typedef struct LavishCompoundJob {
  int64_t src_off;
  int64_t dst_off;
  int64_t conv_off;
  int32_t subpel_x_qn, subpel_y_qn;
} LavishCompoundJob;
int lavish_dist_wtd_convolve_batch(const void *src, int src_stride, void *dst, int dst_stride,
                                   uint16_t *conv_dst, int conv_stride, int w, int h,
                                   const LavishCompoundJob *jobs, int njobs,
                                   const LavishInterpFilterParams *filter_params_x,
                                   const LavishInterpFilterParams *filter_params_y,
                                   const LavishConvolveParams *conv_params, int bit_depth,
                                   int highbd, void *stream);
/* av1/common/av1_rtcd_defs.pl:568-579 (per-call shims, host buffers) */
void av1_dist_wtd_convolve_2d_hip(const uint8_t *src, int src_stride, uint8_t *dst,
                                  int dst_stride, int w, int h,
                                  const LavishInterpFilterParams *filter_params_x,
                                  const LavishInterpFilterParams *filter_params_y,
                                  const int subpel_x_qn, const int subpel_y_qn,
                                  LavishConvolveParams *conv_params);
void av1_dist_wtd_convolve_2d_copy_hip(const uint8_t *src, int src_stride, uint8_t *dst,
                                       int dst_stride, int w, int h,
                                       LavishConvolveParams *conv_params);
void av1_dist_wtd_convolve_x_hip(const uint8_t *src, int src_stride, uint8_t *dst,
                                 int dst_stride, int w, int h,
                                 const LavishInterpFilterParams *filter_params_x,
                                 const int subpel_x_qn, LavishConvolveParams *conv_params);
void av1_dist_wtd_convolve_y_hip(const uint8_t *src, int src_stride, uint8_t *dst,
                                 int dst_stride, int w, int h,
                                 const LavishInterpFilterParams *filter_params_y,
                                 const int subpel_y_qn, LavishConvolveParams *conv_params);
void av1_highbd_dist_wtd_convolve_2d_hip(const uint16_t *src, int src_stride, uint16_t *dst,
                                         int dst_stride, int w, int h,
                                         const LavishInterpFilterParams *filter_params_x,
                                         const LavishInterpFilterParams *filter_params_y,
                                         const int subpel_x_qn, const int subpel_y_qn,
                                         LavishConvolveParams *conv_params, int bd);
void av1_highbd_dist_wtd_convolve_x_hip(const uint16_t *src, int src_stride, uint16_t *dst,
                                        int dst_stride, int w, int h,
                                        const LavishInterpFilterParams *filter_params_x,
                                        const int subpel_x_qn,
                                        LavishConvolveParams *conv_params, int bd);
void av1_highbd_dist_wtd_convolve_y_hip(const uint16_t *src, int src_stride, uint16_t *dst,
                                        int dst_stride, int w, int h,
                                        const LavishInterpFilterParams *filter_params_y,
                                        const int subpel_y_qn,
                                        LavishConvolveParams *conv_params, int bd);
void av1_highbd_dist_wtd_convolve_2d_copy_hip(const uint16_t *src, int src_stride,
                                              uint16_t *dst, int dst_stride, int w, int h,
                                              LavishConvolveParams *conv_params, int bd);

/* ---- scaled convolution --------------------------
 * Replaces av1_convolve_2d_scale_c / av1_highbd_convolve_2d_scale_c
 * (av1/common/convolve.c:488-574,992-1078) -- the inter predictor of a
 * reference of another resolution (convolve_2d_scale_wrapper :576-588) --
 * for a batch of w x h blocks sharing the x / y filters (host
 * InterpFilterParams, taps <= 12) and the conv params (round_0, round_1,
 * is_compound, do_average, use_dist_wtd_comp_avg, fwd_offset, bck_offset;
 * its dst / dst_stride are replaced by conv_dst / conv_stride).  Per block:
 * the element offset of the block's integer source position, the
 * prediction and CONV_BUF offsets, and the scaled start positions and steps
 * in 1/1024 pel (SCALE_SUBPEL_BITS): subpel_*_qn in [0, 1023], *_step_qn in
 * [1, 2048] (a block outside them is left untouched).  w a power of two in
 * [2, 128], h in [1, 128].  Device pointers; asynchronous on `stream`.
 * highbd: u16 samples (bit_depth 8/10/12), else u8.  Returns 0, or < 0 on
 * rejected arguments. */
typedef struct LavishScaleJob {
  int64_t src_off;
  int64_t dst_off;
  int64_t conv_off;
  int32_t subpel_x_qn, x_step_qn, subpel_y_qn, y_step_qn;
} LavishScaleJob;
int lavish_convolve_2d_scale_batch(const void *src, int src_stride, void *dst, int dst_stride,
                                   uint16_t *conv_dst, int conv_stride, int w, int h,
                                   const LavishScaleJob *jobs, int njobs,
                                   const LavishInterpFilterParams *filter_params_x,
                                   const LavishInterpFilterParams *filter_params_y,
                                   const LavishConvolveParams *conv_params, int bit_depth,
                                   int highbd, void *stream);
/* av1/common/av1_rtcd_defs.pl:580,583 (per-call shims, host buffers) */
void av1_convolve_2d_scale_hip(const uint8_t *src, int src_stride, uint8_t *dst,
                               int dst_stride, int w, int h,
                               const LavishInterpFilterParams *filter_params_x,
                               const LavishInterpFilterParams *filter_params_y,
                               const int subpel_x_qn, const int x_step_qn,
                               const int subpel_y_qn, const int y_step_qn,
                               LavishConvolveParams *conv_params);
void av1_highbd_convolve_2d_scale_hip(const uint16_t *src, int src_stride, uint16_t *dst,
                                      int dst_stride, int w, int h,
                                      const LavishInterpFilterParams *filter_params_x,
                                      const LavishInterpFilterParams *filter_params_y,
                                      const int subpel_x_qn, const int x_step_qn,
                                      const int subpel_y_qn, const int y_step_qn,
                                      LavishConvolveParams *conv_params, int bd);

#ifdef __cplusplus
}
#endif
#endif /* LAVISH_DSP_H_ */
