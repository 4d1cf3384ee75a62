/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference (YIVEK/aom-av1-lavish,
 * a libaom v3.6.0 fork) hot-path arithmetic, used only as the *checker* by
 * tests/, __graft_entry__.smoke() and the cpu_baseline leg of bench.py.  The
 * product (aom-av1-lavish_amd/, liblavish_hip.so) never links, loads or calls
 * anything in oracle/.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - 1-D transforms: bit-exact against tests/golden/txfm1d_golden.npz, whose
 *     outputs were produced by executing the reference's own statement lists
 *     (tests/golden/gen_golden.py).
 *   - tables (cospi/sinpi, shifts, cos_bit, scans, quant lookups): equal to the
 *     values parsed from the reference source (tests/golden/ref_tables.json).
 *   - SATD: the reference's known answers (test/avg_test.cc:972-977).
 *   - 2-D transforms: the reference's own accuracy bound vs a double-precision
 *     DCT/ADST (test/av1_fwd_txfm2d_test.cc:71-187).
 *   Everything else (quantizers, SAD/variance, ...) is a careful restatement
 *   citing file:line; bit-exact pinning of those against executed reference
 *   code is not possible here (the reference is unbuildable in this image).
 */
#ifndef LAVISH_ORACLE_H_
#define LAVISH_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* TX_SIZE / TX_TYPE numbering follows aom_dsp/txfm_common.h:25-71. */
enum {
  ORC_TX_4X4, ORC_TX_8X8, ORC_TX_16X16, ORC_TX_32X32, ORC_TX_64X64,
  ORC_TX_4X8, ORC_TX_8X4, ORC_TX_8X16, ORC_TX_16X8, ORC_TX_16X32,
  ORC_TX_32X16, ORC_TX_32X64, ORC_TX_64X32, ORC_TX_4X16, ORC_TX_16X4,
  ORC_TX_8X32, ORC_TX_32X8, ORC_TX_16X64, ORC_TX_64X16, ORC_TX_SIZES_ALL
};

int orc_tx_w(int tx_size);
int orc_tx_h(int tx_size);
int orc_max_eob(int tx_size);     /* av1_get_max_eob, av1/common/blockd.h:1596 */
int orc_tx_scale(int tx_size);    /* av1_get_tx_scale, av1/common/idct.c:24 */
int orc_tx_type_valid(int tx_size, int tx_type); /* test/av1_txfm_test.h:89 */

/* tables */
int32_t orc_cospi(int cos_bit, int idx);
int32_t orc_sinpi(int cos_bit, int idx);
const int32_t *orc_cospi_table(int cos_bit);
void orc_fwd_shift(int tx_size, int8_t out[3]);
int orc_fwd_cos_bit_col(int tx_size);
int orc_fwd_cos_bit_row(int tx_size);

/* 1-D kernels: kind 0=DCT 1=ADST 2=IDENTITY (av1/encoder/av1_fwd_txfm1d.c) */
void orc_fwd_txfm1d(int kind, int n, const int32_t *in, int32_t *out,
                    int cos_bit);
/* inverse 1-D (av1/common/av1_inv_txfm1d.c); stage_range[] as the reference */
void orc_inv_txfm1d(int kind, int n, const int32_t *in, int32_t *out,
                    int cos_bit, const int8_t *stage_range);

/* 2-D forward: av1_fwd_txfm2d_WxH_c (av1/encoder/av1_fwd_txfm2d.c:56-312) */
void orc_fwd_txfm2d(const int16_t *input, int32_t *output, int stride,
                    int tx_type, int tx_size, int bd);
/* av1_fwht4x4_c (av1/encoder/hybrid_fwd_txfm.c:24-76) */
void orc_fwht4x4(const int16_t *input, int32_t *output, int stride);

/* 2-D inverse add: av1_inv_txfm2d_add_WxH_c (av1/common/av1_inv_txfm2d.c) */
void orc_inv_txfm2d_add(const int32_t *input, uint16_t *output, int stride,
                        int tx_type, int tx_size, int bd);

/* scans: av1_scan_orders[tx_size][tx_type] (av1/common/scan.c) */
const int16_t *orc_scan(int tx_size, int tx_type);
const int16_t *orc_iscan(int tx_size, int tx_type);

/* quantizer tables: av1_build_quantizer (av1/encoder/av1_quantize.c:590-686) */
typedef struct {
  int16_t quant[2], quant_shift[2], zbin[2], round[2];
  int16_t quant_fp[2], round_fp[2], dequant[2];
} OrcQuant;
void orc_build_quant(int bd, int qindex, int sharpness, int y_dc_delta_q,
                     OrcQuant *q);
int16_t orc_dc_quant(int qindex, int delta, int bd);
int16_t orc_ac_quant(int qindex, int delta, int bd);

/* quantizers (args as the reference; zbin/round/... point at [2] arrays) */
void orc_quantize_fp(const int32_t *coeff, intptr_t n, const int16_t *zbin,
                     const int16_t *round, const int16_t *quant,
                     const int16_t *quant_shift, int32_t *qcoeff,
                     int32_t *dqcoeff, const int16_t *dequant, uint16_t *eob,
                     const int16_t *scan, const int16_t *iscan, int log_scale);
void orc_quantize_b(const int32_t *coeff, intptr_t n, const int16_t *zbin,
                    const int16_t *round, const int16_t *quant,
                    const int16_t *quant_shift, int32_t *qcoeff,
                    int32_t *dqcoeff, const int16_t *dequant, uint16_t *eob,
                    const int16_t *scan, const int16_t *iscan, int log_scale);
void orc_highbd_quantize_fp(const int32_t *coeff, intptr_t n,
                            const int16_t *zbin, const int16_t *round,
                            const int16_t *quant, const int16_t *quant_shift,
                            int32_t *qcoeff, int32_t *dqcoeff,
                            const int16_t *dequant, uint16_t *eob,
                            const int16_t *scan, const int16_t *iscan,
                            int log_scale);
void orc_highbd_quantize_b(const int32_t *coeff, intptr_t n,
                           const int16_t *zbin, const int16_t *round,
                           const int16_t *quant, const int16_t *quant_shift,
                           int32_t *qcoeff, int32_t *dqcoeff,
                           const int16_t *dequant, uint16_t *eob,
                           const int16_t *scan, const int16_t *iscan,
                           int log_scale);

/* ---- pixel kernels (aom_dsp/ sad, variance, avg, sse, ...) ---- */
unsigned int orc_sad(const uint8_t *a, int a_stride, const uint8_t *b,
                     int b_stride, int w, int h);
unsigned int orc_sad_skip(const uint8_t *a, int a_stride, const uint8_t *b,
                          int b_stride, int w, int h);
unsigned int orc_sad_avg(const uint8_t *src, int src_stride,
                         const uint8_t *ref, int ref_stride, int w, int h,
                         const uint8_t *second_pred);
unsigned int orc_highbd_sad(const uint16_t *a, int a_stride, const uint16_t *b,
                            int b_stride, int w, int h);
unsigned int orc_variance(const uint8_t *a, int a_stride, const uint8_t *b,
                          int b_stride, int w, int h, unsigned int *sse);
unsigned int orc_highbd_variance(const uint16_t *a, int a_stride,
                                 const uint16_t *b, int b_stride, int w, int h,
                                 int bd, unsigned int *sse);
unsigned int orc_sub_pixel_variance(const uint8_t *a, int a_stride,
                                    int xoffset, int yoffset, const uint8_t *b,
                                    int b_stride, int w, int h,
                                    unsigned int *sse);
unsigned int orc_sub_pixel_avg_variance(const uint8_t *a, int a_stride,
                                        int xoffset, int yoffset,
                                        const uint8_t *b, int b_stride, int w,
                                        int h, unsigned int *sse,
                                        const uint8_t *second_pred);
unsigned int orc_highbd_sub_pixel_variance(const uint16_t *a, int a_stride,
                                           int xoffset, int yoffset,
                                           const uint16_t *b, int b_stride,
                                           int w, int h, int bd,
                                           unsigned int *sse,
                                           const uint16_t *second_pred);
unsigned int orc_highbd_sad_avg(const uint16_t *src, int src_stride,
                                const uint16_t *ref, int ref_stride, int w,
                                int h, const uint16_t *second_pred);
void orc_highbd_hadamard(int n, const int16_t *src_diff, ptrdiff_t src_stride,
                         int32_t *coeff);
unsigned int orc_mse(const uint8_t *a, int a_stride, const uint8_t *b,
                     int b_stride, int w, int h, unsigned int *sse);
int64_t orc_sse(const uint8_t *a, int a_stride, const uint8_t *b, int b_stride,
                int w, int h);
int64_t orc_highbd_sse(const uint16_t *a, int a_stride, const uint16_t *b,
                       int b_stride, int w, int h);
void orc_subtract_block(int rows, int cols, int16_t *diff, ptrdiff_t ds,
                        const uint8_t *src, ptrdiff_t ss, const uint8_t *pred,
                        ptrdiff_t ps);
void orc_highbd_subtract_block(int rows, int cols, int16_t *diff,
                               ptrdiff_t ds, const uint16_t *src,
                               ptrdiff_t ss, const uint16_t *pred,
                               ptrdiff_t ps);
uint64_t orc_sum_squares_2d_i16(const int16_t *src, int stride, int w, int h);
void orc_hadamard(int n, const int16_t *src_diff, ptrdiff_t src_stride,
                  int32_t *coeff);
int orc_satd(const int32_t *coeff, int length);
/* oracle_lp.c: int16 forms, (sum, sse), lossless WHT */
void orc_hadamard_lp(int n, const int16_t *src, ptrdiff_t st, int16_t *coeff);
int orc_satd_lp(const int16_t *coeff, int length);
int64_t orc_block_error_lp(const int16_t *coeff, const int16_t *dqcoeff, intptr_t n);
void orc_sum_sse(const int16_t *src, int stride, int w, int h, int *sum, int64_t *sse);
void orc_iwht4x4_add(const int32_t *in, uint16_t *dst, int stride, int eob, int bd);
int64_t orc_block_error(const int32_t *coeff, const int32_t *dqcoeff,
                        intptr_t block_size, int64_t *ssz);
int64_t orc_highbd_block_error(const int32_t *coeff, const int32_t *dqcoeff,
                               intptr_t block_size, int64_t *ssz, int bd);

/* ---- C3: full-pixel motion search (oracle_mcomp.c) ---- */
/* MV_COST_PARAMS (av1/encoder/mcomp.h:40-50): mvcost[k] point at the centre
 * entry of MV_VALS-entry tables (indices -MV_MAX..MV_MAX). */
typedef struct OrcMvCost {
  int mv_cost_type; /* MV_COST_TYPE: 0 ENTROPY 1 L1_LOWRES 2 L1_MIDRES 3 L1_HDRES 4 NONE */
  int sad_per_bit, error_per_bit;
  const int32_t *mvjcost;
  const int32_t *mvcost[2];
} OrcMvCost;
typedef struct OrcMsParams {
  const uint8_t *src; /* block origin */
  int src_stride;
  const uint8_t *ref; /* reference block origin at mv (0,0) */
  int ref_stride;
  int w, h;
  int col_min, col_max, row_min, row_max; /* FullMvLimits */
  int ref_mv_row, ref_mv_col;             /* MV (1/8 pel) for the mv cost */
  int mv_cost_type; /* MV_COST_TYPE */
  int skip_sad;     /* use_downsampled_sad: sdf = aom_sad_skip */
  const OrcMvCost *cost; /* tables for MV_COST_ENTROPY (NULL otherwise) */
} OrcMsParams;
/* search methods (SEARCH_METHODS, av1/encoder/mcomp_structs.h) */
/* SEARCH_METHODS values (av1/encoder/mcomp_structs.h:56-86) */
/* SEARCH_METHODS (av1/encoder/mcomp_structs.h:56-86) */
enum { ORC_DIAMOND = 0, ORC_NSTEP = 1, ORC_NSTEP_8PT = 2, ORC_HEX = 4, ORC_BIGDIA = 5,
       ORC_SQUARE = 6, ORC_FAST_HEX = 7, ORC_FAST_DIAMOND = 8, ORC_FAST_BIGDIA = 9,
       ORC_VFAST_DIAMOND = 10 };
/* the mesh fields of FULLPEL_MOTION_SEARCH_PARAMS (av1/encoder/mcomp.h:
 * 114-123) with the pattern set mesh_patterns[is_intra_mode] */
typedef struct OrcMeshParams {
  int run_mesh_search, force_mesh_thresh, prune_mesh_search, mesh_search_mv_diff_threshold;
  int fine_search_interval, is_intra_mode;
  int range[4], interval[4];
} OrcMeshParams;
/* av1_full_pixel_search (no mesh) with DIAMOND / FAST_BIGDIA / BIGDIA:
 * returns the var cost, writes the best FULLPEL_MV, the step count and,
 * when cost_list != NULL, the reference's 5-entry cost list. */
int orc_full_pixel_search(const OrcMsParams *p, int method, int start_row, int start_col,
                          int step_param, int *cost_list, int *best_row, int *best_col,
                          int *steps);
/* with the mesh refinement (mesh NULL: none) */
int orc_full_pixel_search_ex(const OrcMsParams *p, int method, int start_row, int start_col,
                             int step_param, int *cost_list, int *best_row, int *best_col,
                             int *steps, const OrcMeshParams *mesh);
int orc_full_pixel_search_diamond(const OrcMsParams *p, int start_row,
                                  int start_col, int step_param, int *best_row,
                                  int *best_col, int *steps);

/* batch over jobs laid out like LavishDiamondJob / LavishDiamondResult
 * (include/lavish_dsp.h); threads > 1 uses pthreads. */
typedef struct OrcDiamondJob {
  int64_t src_off, ref_off;
  int16_t start_row, start_col, ref_mv_row, ref_mv_col;
  int16_t col_min, col_max, row_min, row_max;
} OrcDiamondJob;
typedef struct OrcDiamondResult {
  int16_t best_row, best_col;
  int32_t bestsme, steps, reserved;
} OrcDiamondResult;
void orc_diamond_batch(const uint8_t *src, int src_stride, const uint8_t *ref,
                       int ref_stride, int w, int h, const OrcDiamondJob *jobs,
                       long njobs, int step_param, int mv_cost_type,
                       int skip_sad, OrcDiamondResult *out, int threads);

/* FAST_BIGDIA full-pel search (oracle_mcomp.c), same jobs / results */
void orc_bigdia_batch(const uint8_t *src, int src_stride, const uint8_t *ref,
                      int ref_stride, int w, int h, const OrcDiamondJob *jobs,
                      long njobs, int step_param, int mv_cost_type,
                      int skip_sad, OrcDiamondResult *out, int threads);

/* any method, any mv cost (cost->mv_cost_type), optional cost lists
 * (cost_lists[job][5]) */
void orc_full_pixel_search_batch(const uint8_t *src, int src_stride, const uint8_t *ref,
                                 int ref_stride, int w, int h, const OrcDiamondJob *jobs,
                                 long njobs, int method, int step_param, const OrcMvCost *cost,
                                 int skip_sad, int32_t *cost_lists, OrcDiamondResult *out,
                                 int threads);
void orc_full_pixel_search_batch_ex(const uint8_t *src, int src_stride, const uint8_t *ref,
                                    int ref_stride, int w, int h, const OrcDiamondJob *jobs,
                                    long njobs, int method, int step_param,
                                    const OrcMvCost *cost, int skip_sad, int32_t *cost_lists,
                                    OrcDiamondResult *out, int threads,
                                    const OrcMeshParams *mesh);

/* ---- sub-pixel refinement (oracle_subpel.c); layouts = LavishSubpelJob /
 * LavishSubpelResult.  MVs and limits in 1/8 pel. */
typedef struct OrcSubpelJob {
  int64_t src_off, ref_off;
  int16_t start_row, start_col, ref_mv_row, ref_mv_col;
  int16_t col_min, col_max, row_min, row_max;
} OrcSubpelJob;
typedef struct OrcSubpelResult {
  int16_t best_row, best_col;
  uint32_t besterr;
  int32_t distortion;
  uint32_t sse;
} OrcSubpelResult;
void orc_subpel_batch(const uint8_t *src, int src_stride, const uint8_t *ref,
                      int ref_stride, int w, int h, const OrcSubpelJob *jobs,
                      long njobs, int forced_stop, int allow_hp,
                      int iters_per_step, int mv_cost_type,
                      OrcSubpelResult *out, int threads);
/* any subpel method (1 SUBPEL_TREE_PRUNED, 2 SUBPEL_TREE_PRUNED_MORE), any
 * mv cost, optional full-pel cost lists (cost_lists[job][5], the full-pel
 * search's) */
void orc_subpel_search_batch(const uint8_t *src, int src_stride, const uint8_t *ref,
                             int ref_stride, int w, int h, const OrcSubpelJob *jobs, long njobs,
                             int subpel_method, int forced_stop, int allow_hp,
                             int iters_per_step, const OrcMvCost *cost,
                             const int32_t *cost_lists, OrcSubpelResult *out, int threads);
/* the same with SUBPEL_SEARCH_TYPE (0 USE_2_TAPS_ORIG, 1 USE_2_TAPS, 2
 * USE_4_TAPS, 3 USE_8_TAPS): SUBPEL_TREE's error is then the upsampled
 * prediction's (upsampled_pref_error) */
void orc_subpel_search_batch_ex(const uint8_t *src, int src_stride, const uint8_t *ref,
                                int ref_stride, int w, int h, const OrcSubpelJob *jobs,
                                long njobs, int subpel_method, int subpel_search_type,
                                int forced_stop, int allow_hp, int iters_per_step,
                                const OrcMvCost *cost, const int32_t *cost_lists,
                                OrcSubpelResult *out, int threads);

/* ---- TX-type pruning features (oracle_txfeat.c) ---- */
void orc_horver_correlation_full(const int16_t *diff, int stride, int width,
                                 int height, float *hcorr, float *vcorr);
void orc_energy_distribution_finer(const int16_t *diff, int stride, int bw,
                                   int bh, float *hordist, float *verdist);
long orc_tx_prune_features(const int16_t *residual, int stride, int width,
                           int height, int bw, int bh, float *hfeatures,
                           float *vfeatures);

/* ---- C4: per-block TX-type RDO (oracle_rdo.c); layout = LavishRdoBlock */
typedef struct OrcRdoBlock {
  int32_t best_type, eob, rate, satd;
  int64_t dist, sse, rdcost;
} OrcRdoBlock;
long orc_rdo_plane(const uint16_t *src, const uint16_t *pred, int stride,
                   int width, int height, int tx_size, unsigned type_mask,
                   int bd, const OrcQuant *q, int rdmult, OrcRdoBlock *out,
                   int32_t *qcoeff, int32_t *dqcoeff, int threads);
/* the same with pixel-domain distortion (see oracle_rdo.c) */
long orc_rdo_plane_px(const uint16_t *src, const uint16_t *pred, int stride,
                      int width, int height, int tx_size, unsigned type_mask,
                      int bd, const OrcQuant *q, int rdmult, OrcRdoBlock *out,
                      int32_t *qcoeff, int32_t *dqcoeff, int threads);
/* the same with search_tx_type's per-block allowed_tx_mask / txk_map */
long orc_rdo_plane_masked(const uint16_t *src, const uint16_t *pred, int stride, int width,
                          int height, int tx_size, unsigned type_mask, int bd, const OrcQuant *q,
                          int rdmult, const uint16_t *block_mask, const uint8_t *block_map,
                          int px, OrcRdoBlock *out, int32_t *qcoeff, int32_t *dqcoeff,
                          int threads);
void orc_rdo_reconstruct(int nsizes, const int *sizes,
                         const OrcRdoBlock *const *recs,
                         const int32_t *const *dqs, int width, int height,
                         const uint16_t *pred, uint16_t *recon, int stride,
                         int bd, uint8_t *sb_tx_size);

/* ---- C2 pipeline: fwd_txfm + quantize_fp over a residual plane ----
 * For one tx_size, tile the plane with full blocks (row-major block order),
 * evaluate each tx_type whose bit is set in type_mask (ascending type order),
 * write qcoeff/dqcoeff [block][type_slot][n] and eob [block][type_slot].
 * threads > 1 uses pthreads over block rows.  Returns the number of blocks. */
long orc_txq_plane(const int16_t *residual, int stride, int width, int height,
                   int tx_size, unsigned type_mask, int bd,
                   const OrcQuant *q, int quant_b, int32_t *qcoeff,
                   int32_t *dqcoeff, uint16_t *eob, int threads);

/* ---- inter prediction (8(f) rank 2): oracle_convolve.c ---- */
#define FILTER_BITS_ORC 7
typedef struct OrcInterPredJob {
  int64_t ref_off, dst_off;
  int32_t pix_row, pix_col;
  int16_t mv_row, mv_col;
  uint8_t filter_x, filter_y, pad[2];
} OrcInterPredJob;
int orc_interp_kernel(int interp_filter, int size, int subpel, int16_t *out);
void orc_conv_rounds(int bd, int *round_0, int *round_1);
void orc_convolve_block(const void *src, ptrdiff_t ss, void *dst, ptrdiff_t ds, int w, int h,
                        int path, const int16_t *fx, int tx, const int16_t *fy, int ty,
                        int round_0, int round_1, int bd, int hbd);
long orc_build_inter_pred_batch(const void *ref, int ref_stride, int ref_width, int ref_height,
                                int ss_x, int ss_y, int w, int h, const OrcInterPredJob *jobs,
                                long njobs, const OrcSubpelResult *mvs, void *dst,
                                int dst_stride, int bd, int hbd);

/* ---- TX-type pruning (8(f) rank 4): oracle_txfeat.c ---- */
typedef struct OrcNNConfig { /* layout of NN_CONFIG (av1/encoder/ml.h:24-34) */
  int num_inputs, num_outputs, num_hidden_layers;
  int num_hidden_nodes[10];
  const float *weights[11];
  const float *bias[11];
} OrcNNConfig;
void orc_nn_predict(const float *input_nodes, const OrcNNConfig *c, int reduce_prec,
                    float *output);
void orc_sort_fi32(float *k, int *v, int n);
int orc_prune_aggressiveness(int tx_set_type, int prune_mode);
long orc_prune_tx_2d(const int16_t *residual, int stride, int width, int height, int bw, int bh,
                     int tx_set_type, int prune_mode, const float *thresholds,
                     const OrcNNConfig *hor, const OrcNNConfig *ver, const uint16_t *allowed_in,
                     uint16_t allowed_default, uint16_t *allowed_out, uint8_t *txk_map);

/* ---- TPL block transform leg (oracle_tpl.c); layout = LavishTplBlock ---- */
typedef struct OrcTplBlock {
  int32_t best_ref, inter_cost, rate_cost, eob;
  int64_t recon_error, sse;
} OrcTplBlock;
void orc_tpl_block_batch(const void *src, int src_stride, const void *preds, long pred_plane,
                         int pred_stride, int nrefs, int width, int height, int bsize, int bd,
                         const OrcQuant *q, OrcTplBlock *out, void *recon, int recon_stride,
                         int32_t *ref_costs, int threads);
/* mode_estimation's per-reference motion search with start-mv candidates
 * (oracle_tpl.c; 16x16 blocks, subpel_force_stop FULL_PEL); layouts as
 * lavish_tpl_motion_search (include/lavish_dsp.h); one thread per reference */
void orc_tpl_motion_search(const uint8_t *src, int src_stride, const uint8_t *ref,
                           int ref_stride, const OrcDiamondJob *jobs, int cols, int rows,
                           int nrefs, int method, int step_param, int skip_sad,
                           int prune_starting_mv, int skip_alike_starting_mv,
                           const OrcMvCost *cost, const int32_t *third, int32_t *mvs,
                           OrcDiamondResult *out, int32_t *cost_lists, int32_t *centers);

/* ---- av1_quant selection (oracle_qfacade.c): mode 0 FP, 1 B, 2 DC, 3 skip
 * quant, 4 search_tx_type's satd gate; returns use_optimize_b | kind << 1 -- */
int orc_av1_quant_block(const int32_t *coeff, int tx_size, int tx_type, int bd,
                        const OrcQuant *q, int mode, int skip_trellis, unsigned threshold,
                        int qstep, int dc_only, int32_t *qcoeff, int32_t *dqcoeff,
                        uint16_t *eob);

/* ---- coefficient rate (oracle_costcoeffs.c): av1_cost_coeffs_txb and
 * av1_cost_coeffs_txb_laplacian(adjust_eob 0); the cost tables are
 * MACROBLOCK::coeff_costs (CoeffCosts, av1/encoder/block.h:172-211) ---- */
typedef struct {
  int32_t txb_skip_cost[13][2];
  int32_t base_eob_cost[4][3];
  int32_t base_cost[42][8];
  int32_t eob_extra_cost[9][2];
  int32_t dc_sign_cost[3][2];
  int32_t lps_cost[21][26];
} OrcCoeffCost;
typedef struct {
  int32_t eob_cost[2][11];
} OrcEobCost;
typedef struct {
  OrcCoeffCost coeff_costs[5][2];
  OrcEobCost eob_costs[7][2];
} OrcCoeffCosts;
int orc_cost_coeffs_txb(const OrcCoeffCosts *cc, const int32_t *qcoeff, int eob, int plane,
                        int tx_size, int tx_type, int txb_skip_ctx, int dc_sign_ctx,
                        int tx_type_cost, int laplacian);
void orc_cost_coeffs_txb_batch(const OrcCoeffCosts *cc, const int32_t *qcoeff, int n_stride,
                               const uint16_t *eob, int nblocks, int plane, int tx_size,
                               int tx_type, const int32_t *txb_ctx, int tx_type_cost,
                               int laplacian, int32_t *rate);
/* C4 ranked by the coefficient rate (oracle_rdo.c): orc_rdo_plane_masked's
 * TX-domain decision with rate = orc_cost_coeffs_txb; txb_ctx [nblocks][2]
 * and tx_type_costs[16] nullable */
long orc_rdo_plane_rate(const uint16_t *src, const uint16_t *pred, int stride, int width,
                        int height, int tx_size, unsigned type_mask, int bd, const OrcQuant *q,
                        int rdmult, const OrcCoeffCosts *cc, const int32_t *txb_ctx,
                        const int32_t *tx_type_costs, const uint16_t *block_mask,
                        const uint8_t *block_map, OrcRdoBlock *out, int32_t *qcoeff,
                        int32_t *dqcoeff, int threads);

/* ---- coefficient trellis (oracle_trellis.c): av1_optimize_b without a
 * quantization matrix; qcoeff / dqcoeff updated in place; returns the new eob */
int orc_optimize_b(const OrcCoeffCosts *cc, const int32_t *tcoeff, int32_t *qcoeff,
                   int32_t *dqcoeff, int eob, int plane, int tx_size, int tx_type, int bd,
                   int is_inter, int x_rdmult, int sharpness, const int16_t dequant[2],
                   int txb_skip_ctx, int dc_sign_ctx, int tx_type_cost, int *rate_cost,
                   uint8_t *entropy_ctx);

/* oracle_pixbatch.c: 4-candidate SAD + variance (candidate 0) per job
 * (LavishPixJob layout), 8-bit, over `threads` pthreads */
void orc_pixel_batch(const uint8_t *src, int ss, const uint8_t *ref, int rs, int w, int h,
                     const void *jobs, long njobs, uint32_t *sad, uint32_t *var, uint32_t *sse,
                     int threads);

/* oracle_warp.c: av1_get_shear_params (out: alpha, beta, gamma, delta;
 * returns validity) and av1_warp_affine_c / av1_highbd_warp_affine_c */
typedef struct {
  int do_average, round_0, round_1, is_compound, use_dist_wtd_comp_avg, fwd_offset, bck_offset;
} OrcConvParams;
int orc_get_shear_params(const int32_t mat[6], int16_t out[4]);
void orc_warp_affine(const int32_t mat[6], const void *ref, int width, int height, int stride,
                     void *pred, int p_col, int p_row, int p_width, int p_height, int p_stride,
                     int ss_x, int ss_y, int bd, int hbd, const OrcConvParams *cp,
                     uint16_t *conv_dst, int dst_stride, int alpha, int beta, int gamma,
                     int delta);
/* oracle_compound.c: the av1_dist_wtd_convolve_* family (path 0 copy, 1 x,
 * 2 y, 3 2d), lowbd / highbd */
void orc_dist_wtd_convolve(int path, const void *src, int src_stride, void *dst, int dst_stride,
                           int w, int h, const int16_t *fx, int tx, const int16_t *fy, int ty,
                           const OrcConvParams *cp, uint16_t *conv, int conv_stride, int bd,
                           int hbd);
void orc_dist_wtd_batch(const void *src, int src_stride, void *dst, int dst_stride,
                        uint16_t *conv, int conv_stride, int w, int h, const void *jobs,
                        long njobs, const int16_t *fx, int tx, const int16_t *fy, int ty,
                        const OrcConvParams *cp, int bd, int hbd, int threads);
void orc_warp_batch(const void *ref, int width, int height, int stride, void *pred,
                    int p_stride, uint16_t *dst, int dst_stride, const void *jobs, long njobs,
                    int ss_x, int ss_y, int bd, int hbd, const OrcConvParams *cp, int threads);

/* oracle_scale.c: av1_convolve_2d_scale_c / av1_highbd_convolve_2d_scale_c;
 * fx / fy: 16 kernel rows of tx / ty taps */
void orc_convolve_2d_scale(const void *src, int src_stride, void *dst, int dst_stride, int w,
                           int h, const int16_t *fx, int tx, const int16_t *fy, int ty,
                           int subpel_x_qn, int x_step_qn, int subpel_y_qn, int y_step_qn,
                           const OrcConvParams *cp, uint16_t *conv, int conv_stride, int bd,
                           int hbd);
/* the same over a batch of blocks (LavishScaleJob layout), over pthreads */
void orc_convolve_2d_scale_batch(const void *src, int src_stride, void *dst, int dst_stride,
                                 uint16_t *conv, int conv_stride, int w, int h, const void *jobs,
                                 long njobs, const int16_t *fx, int tx, const int16_t *fy, int ty,
                                 const OrcConvParams *cp, int bd, int hbd, int threads);

/* search_tx_type's RDCOST + first-strictly-lowest type choice (oracle_rdo.c) */
int orc_rd_select(int rdmult, const int *rates, const int64_t *dists, int n, int64_t *rds);

#ifdef __cplusplus
}
#endif

#endif  // LAVISH_ORACLE_H_
