// quant_facade.hip -- av1_quant's quantizer selection for a batch of blocks
// on gfx950.
//
// Reference, per block:
//   av1_quant (av1/encoder/encodemb.c:308-341): quant_func_list
//     [xform_quant_idx][is_hbd] (:262-273) = av1_quantize_fp_facade /
//     _b_facade / _dc_facade or their highbd forms (av1/encoder/
//     av1_quantize.c:266-420, 423-563), n = av1_get_max_eob(tx_size), the
//     scan of (tx_size, tx_type), log_scale = av1_get_tx_scale (av1_setup_quant
//     :357-373), no quantization matrix;
//   the xform_quant_idx search_tx_type hands it (tx_search.c:2140-2169):
//     skip_trellis ? AV1_XFORM_QUANT_B : AV1_XFORM_QUANT_FP, then
//     skip_trellis_opt_based_on_satd (:1923-1955) per block: unless trellis is
//     already skipped or the threshold is UINT_MAX, satd = aom_satd of the
//     coefficients (|coeff[0]| for a DC-only block), RIGHT_SIGNED_SHIFT by
//     MAX_TX_SCALE - tx_scale, >> (bd - 8); satd > threshold * qstep *
//     sqrt_tx_pixels_2d[tx_size] selects B without trellis, else FP with it.
// One wave64 per block: the satd reduction, the decision (wave-uniform), the
// n coefficients lane-strided through quant_dev.h's quantizers (the C2 / C4
// kernels' code, pinned against the reference) and the eob as a max-reduce
// of the inverse scan.
#include <climits>

#include "lavish_internal.h"
#include "quant_dev.h"

namespace lavish {
namespace {

// sqrt_tx_pixels_2d (av1/encoder/tx_search.c:76-78)
__constant__ int kSqrtPx[19] = {4, 8, 16, 32, 32, 6, 6, 12, 12, 23, 23, 32, 32, 8, 8, 16, 16, 23, 23};

struct QfArgs {
  const int32_t* coeff;
  const int16_t* iscan;
  const uint8_t* dc_only;
  int32_t* qcoeff;
  int32_t* dqcoeff;
  uint16_t* eob;
  uint8_t* flags;
  int n, nblocks, tx_size, bd, mode, skip_trellis, qstep;
  unsigned threshold;
  QP fp, b;  // FP: round_fp / quant_fp in round / quant; B: the b tables
};

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v = max(v, __shfl_xor(v, m));
  return v;
}

template <int LS, bool HBD>
__global__ __launch_bounds__(64) void av1_quant_kernel(QfArgs a) {
  const int blk = blockIdx.x, lane = threadIdx.x;
  const int32_t* c = a.coeff + (int64_t)blk * a.n;
  int kind = a.mode;
  int optb = 0;
  if (a.mode == LAVISH_AV1_QUANT_SATD_GATE) {
    if (a.skip_trellis || a.threshold == UINT_MAX) {
      kind = a.skip_trellis ? LAVISH_AV1_QUANT_B : LAVISH_AV1_QUANT_FP;  // USE_B_QUANT_NO_TRELLIS
      optb = !a.skip_trellis;
    } else {
      const bool dc = a.dc_only != nullptr && a.dc_only[blk] != 0;
      int s = 0;
      if (dc) {
        s = abs(c[0]);
      } else {
        for (int i = lane; i < a.n; i += 64) s += abs(c[i]);
        s = wave_sum(s);
      }
      const int shift = 1 - LS;  // MAX_TX_SCALE - av1_get_tx_scale
      s = shift < 0 ? s << -shift : s >> shift;
      s >>= a.bd - 8;
      const bool skip = (uint64_t)(int64_t)s >
                        (uint64_t)a.threshold * (uint64_t)(int64_t)a.qstep *
                            (uint64_t)kSqrtPx[a.tx_size];
      kind = skip ? LAVISH_AV1_QUANT_B : LAVISH_AV1_QUANT_FP;
      optb = !skip;
    }
  }
  if (lane == 0 && a.flags) a.flags[blk] = (uint8_t)(optb | (kind << 1));
  if (kind == LAVISH_AV1_QUANT_SKIP) return;  // AV1_XFORM_QUANT_SKIP_QUANT: outputs untouched
  int32_t* q = a.qcoeff + (int64_t)blk * a.n;
  int32_t* dq = a.dqcoeff + (int64_t)blk * a.n;
  int last = 0;
  if (kind == LAVISH_AV1_QUANT_DC) {
    // quantize_dc / highbd_quantize_dc: round_QTX[0], quant_fp_QTX[0], dequant_QTX[0]
    for (int i = lane; i < a.n; i += 64) {
      int32_t qv = 0, dv = 0;
      if (i == 0) {
        const int32_t x = c[0];
        const int32_t sgn = x >> 31;
        const int32_t ax = (x ^ sgn) - sgn;
        const int32_t rnd = (a.b.round[0] + ((1 << LS) >> 1)) >> LS;
        int64_t t = (int64_t)ax + rnd;
        if (!HBD) t = t > 32767 ? 32767 : (t < -32768 ? -32768 : t);
        const int32_t aq = (int32_t)((t * a.fp.quant[0]) >> (16 - LS));
        const int32_t adq = (int32_t)((uint32_t)aq * (uint32_t)a.fp.dequant[0]) >> LS;
        qv = (aq ^ sgn) - sgn;
        dv = (adq ^ sgn) - sgn;
        last = aq != 0 ? 1 : 0;
      }
      q[i] = qv;
      dq[i] = dv;
    }
  } else {
    const bool fp = kind == LAVISH_AV1_QUANT_FP;
    for (int i = lane; i < a.n; i += 64) {
      const bool ac = i != 0;
      const int32_t qv = fp ? quant_one<LS, LAVISH_QUANT_FP, HBD>(c[i], ac, a.fp)
                            : quant_one<LS, LAVISH_QUANT_B, HBD>(c[i], ac, a.b);
      q[i] = qv;
      dq[i] = dequant_one<LS>(qv, ac, fp ? a.fp : a.b);
      last = qv != 0 ? max(last, a.iscan[i] + 1) : last;
    }
  }
  last = wave_max(last);
  if (lane == 0) a.eob[blk] = (uint16_t)last;
}

QP qp_fp(const LavishPlaneQuant& p) {
  QP q{};
  for (int i = 0; i < 2; ++i) {
    q.zbin[i] = p.zbin[i];
    q.round[i] = p.round_fp[i];
    q.quant[i] = p.quant_fp[i];
    q.quant_shift[i] = p.quant_shift[i];
    q.dequant[i] = p.dequant[i];
  }
  return q;
}
QP qp_b(const LavishPlaneQuant& p) {
  QP q{};
  for (int i = 0; i < 2; ++i) {
    q.zbin[i] = p.zbin[i];
    q.round[i] = p.round[i];
    q.quant[i] = p.quant[i];
    q.quant_shift[i] = p.quant_shift[i];
    q.dequant[i] = p.dequant[i];
  }
  return q;
}

}  // namespace
}  // namespace lavish

using namespace lavish;

extern "C" int lavish_build_plane_quant(int bit_depth, int qindex, int quant_sharpness,
                                        int y_dc_delta_q, LavishPlaneQuant* out) {
  if (out == nullptr) return -1;
  LavishQuantParams f, b;
  int rc = lavish_build_quant_params(bit_depth, qindex, quant_sharpness, y_dc_delta_q,
                                     LAVISH_QUANT_FP, &f);
  if (rc == 0)
    rc = lavish_build_quant_params(bit_depth, qindex, quant_sharpness, y_dc_delta_q,
                                   LAVISH_QUANT_B, &b);
  if (rc != 0) return rc;
  for (int i = 0; i < 2; ++i) {
    out->zbin[i] = b.zbin[i];
    out->round_fp[i] = f.round[i];
    out->quant_fp[i] = f.quant[i];
    out->round[i] = b.round[i];
    out->quant[i] = b.quant[i];
    out->quant_shift[i] = b.quant_shift[i];
    out->dequant[i] = b.dequant[i];
  }
  return 0;
}

extern "C" int lavish_av1_quant_batch(const int32_t* coeff, int nblocks, int tx_size,
                                      int tx_type, int bit_depth, const LavishPlaneQuant* pq,
                                      int mode, int skip_trellis,
                                      unsigned coeff_opt_satd_threshold, int qstep,
                                      const uint8_t* dc_only, int32_t* qcoeff,
                                      int32_t* dqcoeff, uint16_t* eob, uint8_t* flags,
                                      void* stream) {
  if (tx_size < 0 || tx_size >= 19 || tx_type < 0 || tx_type >= 16) return -1;
  if (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) return -2;
  if (mode < LAVISH_AV1_QUANT_FP || mode > LAVISH_AV1_QUANT_SATD_GATE) return -3;
  if (pq == nullptr || coeff == nullptr || qcoeff == nullptr || dqcoeff == nullptr ||
      eob == nullptr)
    return -4;
  if (nblocks <= 0) return 0;
  QfArgs a{};
  a.coeff = coeff;
  a.iscan = dev_iscan(tx_size, tx_type);
  a.dc_only = dc_only;
  a.qcoeff = qcoeff;
  a.dqcoeff = dqcoeff;
  a.eob = eob;
  a.flags = flags;
  a.n = max_eob(tx_size);
  a.nblocks = nblocks;
  a.tx_size = tx_size;
  a.bd = bit_depth;
  a.mode = mode;
  a.skip_trellis = skip_trellis;
  a.qstep = qstep;
  a.threshold = coeff_opt_satd_threshold;
  a.fp = qp_fp(*pq);
  a.b = qp_b(*pq);
  const int ls = tx_scale(tx_size);
  hipStream_t s = (hipStream_t)stream;
  const bool hbd = bit_depth > 8;
#define LAVISH_QF(LS)                                                                        \
  if (ls == LS) {                                                                            \
    if (hbd) hipLaunchKernelGGL((av1_quant_kernel<LS, true>), dim3(nblocks), dim3(64), 0, s, a); \
    else hipLaunchKernelGGL((av1_quant_kernel<LS, false>), dim3(nblocks), dim3(64), 0, s, a);    \
  }
  LAVISH_QF(0)
  LAVISH_QF(1)
  LAVISH_QF(2)
#undef LAVISH_QF
  LAVISH_CHECK(hipGetLastError());
  return 0;
}
