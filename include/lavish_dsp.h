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

/* ------------------------------------------------------------------------ */
/* Per-call RTCD shims (host pointers)                                      */
/* ------------------------------------------------------------------------ */
/* av1_fwd_txfm2d_WxH (av1/common/av1_rtcd_defs.pl:358-399) */
#define LAVISH_FWD2D(w, h)                                                   \
  void av1_fwd_txfm2d_##w##x##h##_hip(const int16_t *input, int32_t *output, \
                                      int stride, uint8_t tx_type, int bd);
LAVISH_FWD2D(4, 4)
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
 * av1/encoder/hybrid_fwd_txfm.c:244) */
void av1_lowbd_fwd_txfm_hip(const int16_t *src_diff, int32_t *coeff,
                            int diff_stride, LavishTxfmParam *txfm_param);

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

#ifdef __cplusplus
}
#endif
#endif /* LAVISH_DSP_H_ */
