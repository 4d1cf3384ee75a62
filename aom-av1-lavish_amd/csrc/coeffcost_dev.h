// coeffcost_dev.h -- device pieces of the coefficient rate shared by
// costcoeffs.hip (lavish_cost_coeffs_txb_batch) and rdo.hip (the C4 decision
// with the coefficient rate).
//
// Reference: warehouse_efficients_txb / av1_cost_coeffs_txb
// (av1/encoder/txb_rdopt.c:451-536, 599-624), the context helpers of
// av1/common/txb_common.h:90-257 and the cost helpers of
// av1/encoder/txb_rdopt_utils.h:70-104.  `lv` is the padded |level| map of
// av1_txb_init_levels_c (encodetxb.c:238-254): column-major, `stride` = h +
// TX_PAD_HOR bytes per column, zero pad rows / columns.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lavish {
namespace cc {

// int32 cells of LV_MAP_COEFF_COST (av1/encoder/block.h:172-195) and its
// field offsets; LV_MAP_EOB_COST follows it in the staged table
constexpr int kCostCells = 944, kEobCells = 22;
constexpr int kSkip = 0, kBaseEob = 26, kBase = 38, kEobExtra = 374, kDcSign = 392, kLps = 398;
constexpr int kTabCells = kCostCells + kEobCells;
static_assert(kLps + 21 * 26 == kCostCells, "LV_MAP_COEFF_COST layout");

// tx_type_to_class (txb_common.h:31-48): 0 2D, 1 horizontal, 2 vertical
__host__ __device__ __forceinline__ int tx_class(int tx_type) {
  return tx_type < 10 ? 0 : ((tx_type & 1) ? 1 : 2);
}

__device__ __forceinline__ int min3(int v) { return v < 3 ? v : 3; }

// get_nz_map_ctx_from_stats (txb_common.h:189-224) on the get_nz_mag sum;
// wlt / wgt = tx_size_wide < / > tx_size_high of the (unadjusted) size, the
// rule that generates av1_nz_map_ctx_offset (txb_common.h:199-209)
__device__ __forceinline__ int nz_ctx(int cls, int wlt, int wgt, int stats, int pos, int col,
                                      int row) {
  const int ctx = min((stats + 1) >> 1, 4);
  if (cls == 0) {
    if (pos == 0) return 0;
    int off;
    if (wlt && row < 2) off = 11;
    else if (wgt && col < 2) off = 16;
    else if (row + col < 2) off = 1;
    else if (row + col < 4) off = 6;
    else off = 21;
    return ctx + off;
  }
  const int idx = cls == 1 ? col : row;  // nz_map_ctx_offset_1d
  return ctx + 26 + (idx == 0 ? 0 : (idx == 1 ? 5 : 10));
}

// get_br_ctx's context from its neighbour sum (txb_common.h:103-135)
__device__ __forceinline__ int br_ctx_mag(int cls, int mag, int pos, int col, int row) {
  mag = min((mag + 1) >> 1, 6);
  const bool near = cls == 0 ? (row < 2 && col < 2) : (cls == 1 ? col == 0 : row == 0);
  return pos == 0 ? mag : mag + (near ? 7 : 14);
}

// get_nz_mag (txb_common.h:150-173) / get_br_ctx (:103-135) over the map.
// The neighbour offsets of one tx class are fixed per block, and
// lower_ctx_off / br_ctx_off read through them with no per-coefficient class
// branch.  The class-branching form (third = cls == 0 ? l[stride + 1] :
// cls == 1 ? l[2 * stride] : l[2]) is miscompiled by ROCm 7.2 for gfx950
// once inlined into the trellis walk: on the vertical-class path the
// ds_read_u8 address VGPR is never written (`implicit-def`), see
// profiles/r03_trellis_miscompile_isa.txt and the A/B reproducer
// tools/dbg/build_trellis_cb.sh.  Both kernels (trellis, coefficient cost)
// use this one form.
struct NbrOff {
  int nz0, nz1, nz2;  // get_nz_mag's three class-dependent neighbours
  int br;             // get_br_ctx's third neighbour
};
__host__ __device__ __forceinline__ NbrOff nbr_off(int cls, int stride) {
  NbrOff o;
  if (cls == 0) {
    o.nz0 = stride + 1; o.nz1 = 2 * stride; o.nz2 = 2; o.br = stride + 1;
  } else if (cls == 2) {
    o.nz0 = 2; o.nz1 = 3; o.nz2 = 4; o.br = 2;
  } else {
    o.nz0 = 2 * stride; o.nz1 = 3 * stride; o.nz2 = 4 * stride; o.br = 2 * stride;
  }
  return o;
}
__device__ __forceinline__ int lower_ctx_off(const NbrOff& o, int cls, int wlt, int wgt,
                                             const uint8_t* lv, int stride, int pos, int col,
                                             int row) {
  const uint8_t* l = lv + col * stride + row;
  const int mag = min3(l[stride]) + min3(l[1]) + min3(l[o.nz0]) + min3(l[o.nz1]) + min3(l[o.nz2]);
  return nz_ctx(cls, wlt, wgt, mag, pos, col, row);
}
__device__ __forceinline__ int br_ctx_off(const NbrOff& o, int cls, const uint8_t* lv, int stride,
                                          int pos, int col, int row) {
  const uint8_t* l = lv + col * stride + row;
  return br_ctx_mag(cls, l[1] + l[stride] + l[o.br], pos, col, row);
}

// get_br_ctx_eob (txb_common.h:90-101)
__device__ __forceinline__ int br_ctx_eob(int cls, int pos, int col, int row) {
  if (pos == 0) return 0;
  const bool near = cls == 0 ? (row < 2 && col < 2) : (cls == 1 ? col == 0 : row == 0);
  return near ? 7 : 14;
}

// get_br_cost + get_golomb_cost (txb_rdopt_utils.h:86-104)
__device__ __forceinline__ int br_cost(const int32_t* tab, int ctx, int level) {
  int c = tab[kLps + ctx * 26 + min(level - 3, 12)];
  if (level >= 15) {
    const int len = 32 - __clz(level - 14);  // get_msb(r) + 1
    c += (2 * len - 1) << 9;
  }
  return c;
}

// warehouse_efficients_txb's term of the coefficient v at raster pos (col,
// row) with scan index i < eob, n = coefficients of the adjusted size
__device__ __forceinline__ int coeff_term(const int32_t* tab, const NbrOff& nb, int cls, int wlt,
                                          int wgt, const uint8_t* lv, int stride, int n, int pos,
                                          int col, int row, int i, int eob, int v,
                                          int dc_sign_ctx) {
  const int level = abs(v);
  int cost;
  if (i == eob - 1) {
    const int ctx = i == 0 ? 0 : (i <= (n >> 3) ? 1 : (i <= (n >> 2) ? 2 : 3));
    cost = tab[kBaseEob + ctx * 3 + min3(level) - 1];
    if (level > 2) cost += br_cost(tab, br_ctx_eob(cls, pos, col, row), level);
  } else {
    cost = tab[kBase + lower_ctx_off(nb, cls, wlt, wgt, lv, stride, pos, col, row) * 8 +
               min3(level)];
    if (level > 2) cost += br_cost(tab, br_ctx_off(nb, cls, lv, stride, pos, col, row), level);
  }
  if (level) cost += i ? 512 : tab[kDcSign + dc_sign_ctx * 2 + (v < 0)];
  return cost;
}

// coeff_term with the neighbour sums already formed (no level map): nzmag =
// get_nz_mag's clipped sum, brmag = get_br_ctx's raw sum.  Levels clipped to
// 15 (MAX_BASE_BR_RANGE) give the same contexts: get_nz_mag clips each to 3
// and get_br_ctx saturates once its sum reaches 11.
__device__ __forceinline__ int coeff_term_mag(const int32_t* tab, int cls, int wlt, int wgt,
                                              int n, int pos, int col, int row, int i, int eob,
                                              int v, int dc_sign_ctx, int nzmag, int brmag) {
  const int level = abs(v);
  int cost;
  if (i == eob - 1) {
    const int ctx = i == 0 ? 0 : (i <= (n >> 3) ? 1 : (i <= (n >> 2) ? 2 : 3));
    cost = tab[kBaseEob + ctx * 3 + min3(level) - 1];
    if (level > 2) cost += br_cost(tab, br_ctx_eob(cls, pos, col, row), level);
  } else {
    cost = tab[kBase + nz_ctx(cls, wlt, wgt, nzmag, pos, col, row) * 8 + min3(level)];
    if (level > 2) cost += br_cost(tab, br_ctx_mag(cls, brmag, pos, col, row), level);
  }
  if (level) cost += i ? 512 : tab[kDcSign + dc_sign_ctx * 2 + (v < 0)];
  return cost;
}

// av1_cost_coeffs_txb's total from the summed coefficient terms: eob 0 ->
// txb_skip_cost[ctx][1]; else txb_skip_cost[ctx][0] + the tx-type cost +
// get_eob_cost (txb_rdopt_utils.h:70-84; av1_get_eob_pos_token,
// encodetxb.c:117-131, as a bit length; av1_eob_group_start /
// av1_eob_offset_bits in closed form) + the terms
__device__ __forceinline__ int txb_rate(const int32_t* tab, int cls, int skip_ctx, int eob,
                                        int tx_type_cost, int terms) {
  if (eob == 0) return tab[kSkip + skip_ctx * 2 + 1];
  const int t = eob < 3 ? eob : 33 - __clz(eob - 1);
  const int bits = t >= 3 ? t - 2 : 0;
  int r = tab[kSkip + skip_ctx * 2] + tx_type_cost + terms +
          tab[kCostCells + (cls ? 11 : 0) + t - 1];
  if (bits > 0) {
    const int extra = eob - ((1 << (t - 2)) + 1);
    r += tab[kEobExtra + (t - 3) * 2 + ((extra >> (bits - 1)) & 1)] + (bits - 1) * 512;
  }
  return r;
}

}  // namespace cc
}  // namespace lavish
