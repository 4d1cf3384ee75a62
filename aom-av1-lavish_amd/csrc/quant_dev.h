// quant_dev.h -- device-side quantizers and helpers shared by the
// transform + quantize kernels (txq.hip: C2 planes, rdo.hip: C4 decisions).
#pragma once
#include "txfm_dev.h"

namespace lavish {

// vtx_tab / htx_tab (av1/common/common_data.h:149-159): 0 DCT 1 ADST 2 FLIPADST 3 IDTX
// packed 2 bits per type (a runtime-indexed array would live in scratch)
constexpr uint32_t pack2(const uint8_t (&v)[16]) {
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r |= (uint32_t)v[i] << (2 * i);
  return r;
}
constexpr uint8_t kVtxTab[16] = {0, 1, 0, 1, 2, 0, 2, 1, 2, 3, 0, 3, 1, 3, 2, 3};
constexpr uint8_t kHtxTab[16] = {0, 0, 1, 1, 0, 2, 2, 2, 1, 3, 3, 0, 3, 1, 3, 2};
constexpr uint32_t kVtxPacked = pack2(kVtxTab);
constexpr uint32_t kHtxPacked = pack2(kHtxTab);

struct QP {
  int16_t zbin[2], round[2], quant[2], quant_shift[2], dequant[2];
};

// One coefficient through av1_quantize_fp* / aom_quantize_b* (qm off),
// branch-free.  QK: LAVISH_QUANT_FP or LAVISH_QUANT_B; HBD: highbd variant
// (no int16 clamp of the rounded magnitude).  `ac` selects the [1] entries.
// Exactness of the 32-bit forms:
//  * fp lowbd: t <= 32767, quant_fp < 2^15 -> t*quant < 2^30;
//  * b: ((t*32)*quant) >> 16 == (t*quant) >> 11 exactly (32 t q / 2^16);
//    t*quant < 2^30 in lowbd, 64-bit in highbd; the final multiply by
//    quant_shift is 64-bit (quant_shift may be any int16 in the per-call API).
// F24: the caller's FAST range (tools/range_analysis.py: |coefficient| <
// 2^21 for residuals <= kFastResidualMax) -- the highbd fp product and the
// pass test of fp then fit 24-bit multiplies (v_mul_i32_i24 /
// v_mul_hi_i32_i24, full rate) and 32-bit compares instead of the
// quarter-rate 64-bit multiply; same bits.
template <int LS, int QK, bool HBD, bool F24 = false>
__device__ __forceinline__ int32_t quant_one(int32_t c, bool ac, const QP& qp) {
  const int32_t sgn = c >> 31;
  const int32_t a = (c ^ sgn) - sgn;
  const int32_t rnd = ((ac ? qp.round[1] : qp.round[0]) + ((1 << LS) >> 1)) >> LS;
  const int32_t qt = ac ? qp.quant[1] : qp.quant[0];
  int32_t q;
  if constexpr (QK == LAVISH_QUANT_FP) {
    const int32_t deq = ac ? qp.dequant[1] : qp.dequant[0];
    const bool pass = F24 ? (a << (1 + LS)) >= deq : ((int64_t)a << (1 + LS)) >= deq;
    if constexpr (!HBD) {
      const int32_t t = min(a + rnd, 32767);
      q = (sext24(t) * qt) >> (16 - LS);
    } else if constexpr (F24) {
      q = (int32_t)(((int64_t)sext24(a + rnd) * (int64_t)sext24(qt)) >> (16 - LS));
    } else {
      q = (int32_t)(((int64_t)(a + rnd) * qt) >> (16 - LS));
    }
    q = pass ? q : 0;
  } else {
    const int32_t zb = ((ac ? qp.zbin[1] : qp.zbin[0]) + ((1 << LS) >> 1)) >> LS;
    const int32_t qs = ac ? qp.quant_shift[1] : qp.quant_shift[0];
    const bool pass = a >= zb;
    int64_t u;
    if constexpr (!HBD) {
      const int32_t t = min(a + rnd, 32767);
      u = (int64_t)(((sext24(t) * qt) >> 11) + (t << 5));
    } else {
      const int64_t t = (int64_t)a + rnd;
      u = ((t * qt) >> 11) + (t << 5);
    }
    q = (int32_t)((u * qs) >> (16 - LS + 5));
    q = pass ? q : 0;
  }
  return (q ^ sgn) - sgn;
}

// F24: |q| < 2^23 -- the FAST range bounds |coeff| < 2^21, and quant_b's
// worst case with the largest per-call quant_shift (2^16) reaches about
// 2^22.6, still inside 24 bits -- so the product's low 32 bits (the
// reference's int multiply, wrap included) come from one 24-bit multiply,
// mul_i24 (txfm_dev.h: v_mul_i32_i24, no C++ overflow).
template <int LS, bool F24 = false>
__device__ __forceinline__ int32_t dequant_one(int32_t q, bool ac, const QP& qp) {
  const int32_t sgn = q >> 31;
  const int32_t aq = (q ^ sgn) - sgn;
  const int32_t d = ac ? qp.dequant[1] : qp.dequant[0];
  // (abs_q * dequant) >> log_scale as an int multiply (wraps like the reference)
  const int32_t adq =
      F24 ? mul_i24(aq, d) >> LS : (int32_t)((uint32_t)aq * (uint32_t)d) >> LS;
  return (adq ^ sgn) - sgn;
}

// Largest residual magnitude for which the FAST (24-bit multiply, 32-bit sum)
// transform arithmetic is certified exact for every size <= 32x32 by
// tools/range_analysis.py (worst case 16x4: sums < 2^30.8).  Covers all 8-
// and 10-bit residuals; larger inputs take the exact 64-bit-sum path.
constexpr int kFastResidualMax = 1023;

typedef int32_t v4i __attribute__((ext_vector_type(4)));

}  // namespace lavish
