// tpl.hip -- the TPL model's per-block transform leg for gfx950 (SURVEY.md
// 8(f) rank 1).
//
// Reference, per tpl block (16x16 at every speed of this tree,
// set_tpl_stats_block_size, av1/encoder/tpl_model.c:137-145) and per
// reference frame of mode_estimation, after its motion search:
//   tpl_get_satd_cost (tpl_model.c:199-210): av1_subtract_block ->
//     av1_quick_txfm(use_hadamard 0: DCT_DCT fwd 2-D, hybrid_fwd_txfm.c:
//     315-336) -> aom_satd  => inter cost of that reference;
// the cheapest reference (strictly lower cost wins, in reference order),
// then on its prediction txfm_quant_rdcost (:225-247):
//   subtract -> quick_txfm -> get_quantize_error (:98-135: av1_setup_quant FP,
//   log_scale of the size, av1_quantize_fp_facade / highbd, block error >>
//   (TX_32X32 ? 0 : 2), both clamped to >= 1) -> rate_estimator (:212-223,
//   DCT_DCT scan up to eob, << AV1_PROB_COST_SHIFT) -> av1_inverse_transform_
//   block into the prediction (recon).
//
// Here one wave64 owns P = 64 / N blocks, N lanes per block: lane i holds
// source column i, runs column i's 1-D DCT for every reference, then row i's
// (through an LDS transpose), reduces the satd over its N lanes; the
// cheapest reference's row coefficients stay in registers for the
// quantization, error, rate and the inverse (row pass in registers, column
// pass after a second transpose), and the reconstruction is written out.
// The 1-D transforms are txfm_dev.h's (the C2 / C4 kernels' code).
#include "lane_red.h"
#include "lavish_internal.h"
#include "quant_dev.h"

namespace lavish {
namespace {

struct TplArgs {
  const void* src;
  const void* preds;
  void* recon;
  LavishTplBlock* out;
  int32_t* ref_costs;
  const int16_t* iscan;  // DCT_DCT inverse scan of the size
  int64_t pred_plane;    // elements between reference planes
  int src_stride, pred_stride, recon_stride;
  int nbx, nblocks, nrefs;
  QP qp;
};

template <int N>
struct TplCfg {
  using C = TxCfg<N, N>;
  static constexpr int P = 64 / N;  // blocks per wave
  static constexpr int TS = N + 1;  // transpose row stride (bank spread)
  static constexpr int SHIFT = N == 32 ? 0 : 2;  // get_quantize_error
};

template <int N>
__device__ __forceinline__ int seg_sum(int v) {
  return lane_sum<N>(v);
}
template <int N>
__device__ __forceinline__ int64_t seg_sum64(int64_t v) {
  return lane_sum64<N>(v);
}
template <int N>
__device__ __forceinline__ int seg_max(int v) {
  return lane_max<N>(v);
}

__device__ __forceinline__ int msb(unsigned v) { return 31 - __clz(v); }  // get_msb

template <int N, int BDI, typename PIX>
__global__ __launch_bounds__(64) void tpl_kernel(TplArgs a) {
  using T = TplCfg<N>;
  using C = typename T::C;
  using B = Bd<BDI>;
  constexpr bool FAST = BDI < 2;  // |residual| <= 1023 (quant_dev.h)
  constexpr bool HBD = BDI > 0;
  constexpr int LS = C::log_scale;
  __shared__ int32_t t1[T::P * N * T::TS];

  const int lane = threadIdx.x;
  const int b = lane / N, i = lane % N;
  const int blk = blockIdx.x * T::P + b;
  const bool live = blk < a.nblocks;
  const int bb = live ? blk : a.nblocks - 1;  // idle lanes redo the last block, write nothing
  const int bx = (bb % a.nbx) * N, by = (bb / a.nbx) * N;
  int32_t* tb = t1 + b * N * T::TS;

  const PIX* src = (const PIX*)a.src + (int64_t)by * a.src_stride + bx;
  int32_t sc[N];
#pragma unroll
  for (int r = 0; r < N; ++r) sc[r] = src[(int64_t)r * a.src_stride + i];

  // forward 2-D DCT_DCT of src - pred_k; lane i ends with row i's outputs
  auto fwd = [&](const PIX* pred, int32_t (&v)[N]) {
    int32_t in[N], out[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
      const int32_t x = sc[r] - (int32_t)pred[(int64_t)r * a.pred_stride + i];
      if constexpr (FAST) in[r] = x * (1 << C::s0);
      else in[r] = round_shift_1<-C::s0>(x);
    }
    fwd_1d<N, C::cos_bit_col, FAST>(0, in, out);
#pragma unroll
    for (int r = 0; r < N; ++r) tb[r * T::TS + i] = round_shift_1<-C::s1>(out[r]);
    wave_sync();
#pragma unroll
    for (int c = 0; c < N; ++c) in[c] = tb[i * T::TS + c];
    fwd_1d<N, C::cos_bit_row, FAST>(0, in, out);
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] = round_shift_1<-C::s2>(out[c]);
    wave_sync();  // tb is rewritten by the next reference
  };

  const PIX* preds = (const PIX*)a.preds + (int64_t)by * a.pred_stride + bx;
  int best_k = -1;
  int best_cost = 0x7FFFFFFF;
  int32_t bv[N];
#pragma unroll
  for (int c = 0; c < N; ++c) bv[c] = 0;
  for (int k = 0; k < a.nrefs; ++k) {
    int32_t v[N];
    fwd(preds + (int64_t)k * a.pred_plane, v);
    int s = 0;
#pragma unroll
    for (int c = 0; c < N; ++c) s += abs(v[c]);
    s = seg_sum<N>(s);  // aom_satd over the block
    if (live && i == 0 && a.ref_costs) a.ref_costs[(int64_t)blk * a.nrefs + k] = s;
    if (s < best_cost) {
      best_cost = s;
      best_k = k;
#pragma unroll
      for (int c = 0; c < N; ++c) bv[c] = v[c];
    }
  }

  // get_quantize_error + rate_estimator on the best reference (coefficient
  // rc = c * N + i of the transposed output lives in lane i, slot c)
  int32_t dq[N], qv[N];
  int64_t err = 0, sse = 0;
  int last = 0;
#pragma unroll
  for (int c = 0; c < N; ++c) {
    const int rc = c * N + i;
    const bool ac = rc != 0;
    const int32_t q = quant_one<LS, LAVISH_QUANT_FP, HBD>(bv[c], ac, a.qp);
    qv[c] = q;
    dq[c] = dequant_one<LS>(q, ac, a.qp);
    const int64_t d = (int64_t)bv[c] - dq[c];
    err += d * d;
    sse += (int64_t)bv[c] * bv[c];
    last = q != 0 ? max(last, a.iscan[rc] + 1) : last;
  }
  last = seg_max<N>(last);
  int rate = 0;
#pragma unroll
  for (int c = 0; c < N; ++c) {
    const unsigned al = (unsigned)abs(qv[c]);
    if (a.iscan[c * N + i] < last) rate += msb(al + 1) + 1 + (al > 0);
  }
  rate = seg_sum<N>(rate);
  err = seg_sum64<N>(err);
  sse = seg_sum64<N>(sse);
  if constexpr (HBD) {  // av1_highbd_block_error: round both sums by 2 (bd - 8)
    constexpr int sh = 2 * (B::bd - 8);
    err = (err + (((int64_t)1 << sh) >> 1)) >> sh;
    sse = (sse + (((int64_t)1 << sh) >> 1)) >> sh;
  }
  err >>= T::SHIFT;
  sse >>= T::SHIFT;

  // inverse 2-D DCT_DCT (inv_txfm2d_add_c) of dq, added to the prediction
  {
    int32_t in[N], out[N];
#pragma unroll
    for (int c = 0; c < N; ++c) in[c] = clamp_bits<B::clamp_in_row>(dq[c]);
    inv_1d<N, 12, B::rng_row>(0, in, out);
#pragma unroll
    for (int c = 0; c < N; ++c) tb[i * T::TS + c] = rshift_r(out[c], -C::is0);
    wave_sync();
#pragma unroll
    for (int r = 0; r < N; ++r) in[r] = clamp_bits<B::clamp_in_col>(tb[r * T::TS + i]);
    inv_1d<N, 12, B::rng_col>(0, in, out);
    if (live) {
      constexpr int maxv = (1 << B::bd) - 1;
      const PIX* pb = preds + (int64_t)(best_k < 0 ? 0 : best_k) * a.pred_plane;
      PIX* rec = (PIX*)a.recon + (int64_t)by * a.recon_stride + bx;
#pragma unroll
      for (int r = 0; r < N; ++r) {
        // eob 0: av1_inverse_transform_block leaves the prediction (the
        // inverse of zeros is zero, so the sum below is the same)
        const int v = (int)pb[(int64_t)r * a.pred_stride + i] + rshift_r(out[r], -C::is1);
        rec[(int64_t)r * a.recon_stride + i] = (PIX)(v < 0 ? 0 : (v > maxv ? maxv : v));
      }
    }
  }
  if (live && i == 0) {
    LavishTplBlock o;
    o.best_ref = best_k;
    o.inter_cost = best_cost;
    o.rate_cost = (1 + rate) << 9;  // AV1_PROB_COST_SHIFT
    o.eob = last;
    o.recon_error = err > 1 ? err : 1;
    o.sse = sse > 1 ? sse : 1;
    a.out[blk] = o;
  }
}

template <int N, int BDI, typename PIX>
void launch(const TplArgs& a, hipStream_t s) {
  constexpr int P = TplCfg<N>::P;
  hipLaunchKernelGGL((tpl_kernel<N, BDI, PIX>), dim3((a.nblocks + P - 1) / P), dim3(64), 0, s,
                     a);
}

}  // namespace
}  // namespace lavish

using namespace lavish;

extern "C" int lavish_tpl_block_batch(const void* src, int src_stride, const void* preds,
                                      int64_t pred_plane, int pred_stride, int nrefs, int width,
                                      int height, int bsize, int bit_depth,
                                      const LavishQuantParams* qp, LavishTplBlock* out,
                                      void* recon, int recon_stride, int32_t* ref_costs,
                                      void* stream) {
  if (bsize != 8 && bsize != 16 && bsize != 32) return -1;
  if (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) return -2;
  if (qp == nullptr || out == nullptr || recon == nullptr || src == nullptr) return -3;
  if (nrefs < 1 || preds == nullptr || pred_plane < 0) return -4;
  if (width < bsize || height < bsize || src_stride < width || pred_stride < width ||
      recon_stride < width)
    return -5;
  TplArgs a{};
  a.src = src;
  a.preds = preds;
  a.recon = recon;
  a.out = out;
  a.ref_costs = ref_costs;
  const int ts = bsize == 8 ? 1 : bsize == 16 ? 2 : 3;  // TX_8X8 / 16X16 / 32X32
  a.iscan = dev_iscan(ts, 0);
  a.pred_plane = pred_plane;
  a.src_stride = src_stride;
  a.pred_stride = pred_stride;
  a.recon_stride = recon_stride;
  a.nbx = width / bsize;
  a.nblocks = (width / bsize) * (height / bsize);
  a.nrefs = nrefs;
  for (int k = 0; k < 2; ++k) {
    a.qp.zbin[k] = qp->zbin[k];
    a.qp.round[k] = qp->round[k];
    a.qp.quant[k] = qp->quant[k];
    a.qp.quant_shift[k] = qp->quant_shift[k];
    a.qp.dequant[k] = qp->dequant[k];
  }
  if (a.nblocks == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
#define LAVISH_TPL(N)                                                   \
  if (bsize == N) {                                                     \
    if (bit_depth == 8) launch<N, 0, uint8_t>(a, s);                    \
    else if (bit_depth == 10) launch<N, 1, uint16_t>(a, s);             \
    else launch<N, 2, uint16_t>(a, s);                                  \
  }
  LAVISH_TPL(8)
  LAVISH_TPL(16)
  LAVISH_TPL(32)
#undef LAVISH_TPL
  LAVISH_CHECK(hipGetLastError());
  return 0;
}
