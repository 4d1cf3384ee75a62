// costcoeffs.hip -- the coefficient rate of a batch of transform blocks on
// gfx950.
//
// Reference, per block (av1/encoder/txb_rdopt.c):
//   av1_cost_coeffs_txb (:599-624): eob 0 -> txb_skip_cost[ctx][1]; else
//   warehouse_efficients_txb (:451-536): txb_skip_cost[ctx][0] + the tx-type
//   cost + get_eob_cost (txb_rdopt_utils.h:70-84) + per coefficient of scan
//   index i < eob: base_eob_cost (i = eob - 1, context from the scan index)
//   or base_cost (context get_nz_mag over the |level| map,
//   txb_common.h:150-257), the sign (dc_sign_cost at i = 0, one literal bit
//   otherwise), and for |level| > 2 the base-range cost lps_cost[get_br_ctx]
//   plus the Golomb tail (txb_rdopt_utils.h:86-104);
//   av1_cost_coeffs_txb_laplacian with adjust_eob = 0 (:626-660): the same
//   header, then costLUT / (|last| - 1) << 11 / (const_term + loge_par) per
//   coefficient (av1_cost_coeffs_txb_estimate, :538-569).
//
// The reference walks the scan; every term above depends only on the
// coefficient's own scan index, level and raster neighbours, so each lane
// here takes whole 4-coefficient chunks of the raster block (one 16-byte load,
// one packed LDS level word: 4 consecutive rows of one column) and adds the
// terms of those whose inverse-scan index is below eob.  Per wave: 64 / G
// blocks, G = min(n / 4, 64) lanes each; the padded |level| map of
// av1_txb_init_levels (columns of h + TX_PAD_HOR bytes, 4 zero columns after)
// lives in LDS per block; the selected LV_MAP_COEFF_COST / LV_MAP_EOB_COST
// tables and the inverse scan are staged in LDS once per workgroup, which
// then strides over the batch.  No scatter, no workgroup barrier in the loop
// (each wave owns its blocks' level maps).
#include "coeffcost_dev.h"
#include "lavish_internal.h"

namespace lavish {
namespace {

using namespace cc;
static_assert(sizeof(LavishCoeffCost) == kCostCells * 4, "LavishCoeffCost layout");
static_assert(sizeof(LavishEobCost) == kEobCells * 4, "LavishEobCost layout");

// costLUT (txb_rdopt_utils.h:31-33)
__constant__ int kCostLut[15] = {-1143, 53, 545, 825, 1031, 1209, 1393, 1577,
                                 1763, 1947, 2132, 2317, 2501, 2686, 2871};

struct CcArgs {
  const int32_t* cost;  // the block class's LV_MAP_COEFF_COST
  const int32_t* eobc;  // its LV_MAP_EOB_COST
  const int32_t* qcoeff;
  const uint16_t* eob;
  const LavishTxbCtx* ctx;
  const int16_t* iscan;
  int32_t* rate;
  int nblocks;
  int w, h, bhl;    // av1_get_adjusted_tx_size dims, log2(h)
  int cls;          // tx_type_to_class: 0 2D, 1 horizontal, 2 vertical
  int wlt, wgt;     // tx_size_wide < / > tx_size_high (av1_nz_map_ctx_offset)
  int tx_type_cost;
};

template <int LOGN, bool LAP>
__global__ __launch_bounds__(256) void cost_coeffs_kernel(CcArgs a) {
  constexpr int N = 1 << LOGN;
  constexpr int C = N / 4;              // 4-coefficient chunks per block
  constexpr int G = C < 64 ? C : 64;    // lanes per block
  constexpr int KC = C / G;             // chunks per lane
  constexpr int BPW = 64 / G;           // blocks per wave
  constexpr int BPWG = 4 * BPW;         // blocks per workgroup pass
  constexpr int LVS = 2 * N + 32;       // >= (w + 4) * (h + 4) for every w * h = N
  __shared__ int32_t tab[kCostCells + kEobCells];
  __shared__ int64_t isc_q[N / 4];      // the inverse scan, 4 int16 per cell
  __shared__ uint32_t lvw[LAP ? 1 : BPWG * LVS / 4];
  const int tid = threadIdx.x;
  for (int i = tid; i < kCostCells; i += 256) tab[i] = a.cost[i];
  if (tid < kEobCells) tab[kCostCells + tid] = a.eobc[tid];
  int16_t* isc = reinterpret_cast<int16_t*>(isc_q);
  for (int i = tid; i < N; i += 256) isc[i] = a.iscan[i];
  __syncthreads();

  const int lane = tid & 63;
  const int slot = (tid >> 6) * BPW + lane / G, g = lane % G;
  uint8_t* lv = reinterpret_cast<uint8_t*>(lvw) + slot * LVS;
  const int w = a.w, h = a.h, bhl = a.bhl, stride = h + 4;
  for (int base = blockIdx.x * BPWG; base < a.nblocks; base += gridDim.x * BPWG) {
    const int b = base + slot;
    const bool valid = b < a.nblocks;
    const int bb = valid ? b : a.nblocks - 1;
    const int4* qp = reinterpret_cast<const int4*>(a.qcoeff + (int64_t)bb * N);
    int4 q[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) q[k] = qp[g + k * G];
    const int eob = a.eob[bb];
    if (!LAP) {
      // the padded |level| map (av1_txb_init_levels_c, encodetxb.c:238-254):
      // every in-block byte is written below, so only the 4 pad rows of each
      // column and the 4 pad columns are cleared
      for (int j = g; j < w + stride; j += G) {
        const int word = j < w ? (j * stride + h) >> 2 : ((w * stride) >> 2) + (j - w);
        reinterpret_cast<uint32_t*>(lv)[word] = 0u;
      }
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int pos0 = (g + k * G) * 4;
        const int col = pos0 >> bhl, row0 = pos0 & (h - 1);
        const uint32_t l0 = min(abs(q[k].x), 127), l1 = min(abs(q[k].y), 127);
        const uint32_t l2 = min(abs(q[k].z), 127), l3 = min(abs(q[k].w), 127);
        *reinterpret_cast<uint32_t*>(lv + col * stride + row0) =
            l0 | (l1 << 8) | (l2 << 16) | (l3 << 24);
      }
      wave_sync();
    }
    const int dcctx = a.ctx ? a.ctx[bb].dc_sign_ctx : 0;
    const NbrOff nb = nbr_off(a.cls, stride);
    int cost = 0;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int ch = g + k * G;
      const int pos0 = ch * 4;
      const int col = pos0 >> bhl, row0 = pos0 & (h - 1);
      const int64_t iv = isc_q[ch];
      const int vs[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = (int16_t)(iv >> (16 * e));
        if (i >= eob) continue;
        const int v = vs[e];
        if (LAP) {
          const int level = abs(v);
          cost += i == eob - 1 ? (level - 1) << 11 : kCostLut[min(level, 14)];
          continue;
        }
        cost += coeff_term(tab, nb, a.cls, a.wlt, a.wgt, lv, stride, N, pos0 + e, col, row0 + e,
                           i, eob, v, dcctx);
      }
    }
#pragma unroll
    for (int m = 1; m < G; m <<= 1) cost += __shfl_xor(cost, m);
    if (valid && g == 0) {
      const int skctx = a.ctx ? a.ctx[b].txb_skip_ctx : 0;
      int r = txb_rate(tab, a.cls, skctx, eob, a.tx_type_cost, cost);
      if (LAP && eob > 0) r += (512 + 739) * (eob - 1);  // const_term + loge_par
      a.rate[b] = r;
    }
    if (!LAP) wave_sync();
  }
}

int ilog2(int v) { return 31 - __builtin_clz(v); }

}  // namespace
}  // namespace lavish

using namespace lavish;

extern "C" int lavish_cost_coeffs_txb_batch(const LavishCoeffCosts* costs, const int32_t* qcoeff,
                                            const uint16_t* eob, int nblocks, int plane,
                                            int tx_size, int tx_type,
                                            const LavishTxbCtx* txb_ctx, int tx_type_cost,
                                            int mode, int32_t* rate, void* stream) {
  if (tx_size < 0 || tx_size >= 19 || tx_type < 0 || tx_type >= 16) return -1;
  if (plane < 0 || plane > 2) return -2;
  if (costs == nullptr || qcoeff == nullptr || eob == nullptr || rate == nullptr) return -3;
  if (mode != LAVISH_COEFF_RATE_EXACT && mode != LAVISH_COEFF_RATE_LAPLACIAN) return -4;
  if (nblocks <= 0) return 0;
  const int txw = tx_w(tx_size), txh = tx_h(tx_size);
  const int w = txw > 32 ? 32 : txw, h = txh > 32 ? 32 : txh;
  const int mn = txw < txh ? txw : txh, mx = txw < txh ? txh : txw;
  const int txs_ctx = (ilog2(mn) - 2 + ilog2(mx) - 2 + 1) >> 1;  // get_txsize_entropy_ctx
  const int plane_type = plane > 0;
  const int eob_multi_size = ilog2(w * h) - 4;                    // txsize_log2_minus4
  CcArgs a{};
  a.cost = &costs->coeff_costs[txs_ctx][plane_type].txb_skip_cost[0][0];
  a.eobc = &costs->eob_costs[eob_multi_size][plane_type].eob_cost[0][0];
  a.qcoeff = qcoeff;
  a.eob = eob;
  a.ctx = txb_ctx;
  a.iscan = dev_iscan(tx_size, tx_type);
  a.rate = rate;
  a.nblocks = nblocks;
  a.w = w;
  a.h = h;
  a.bhl = ilog2(h);
  a.cls = cc::tx_class(tx_type);
  a.wlt = txw < txh;
  a.wgt = txw > txh;
  a.tx_type_cost = plane == 0 ? tx_type_cost : 0;  // get_tx_type_cost: 0 for plane > 0
  const int logn = ilog2(w * h);
  const int c = (w * h) / 4, gl = c < 64 ? c : 64, bpwg = 4 * (64 / gl);
  // 8 workgroups per CU at most: each stages the tables once and then
  // strides over the batch (small blocks would otherwise re-stage ~4 KB of
  // tables per few KB of coefficients)
  int grid = (nblocks + bpwg - 1) / bpwg;
  if (grid > 2048) grid = 2048;
  hipStream_t s = (hipStream_t)stream;
  const bool lap = mode == LAVISH_COEFF_RATE_LAPLACIAN;
#define LAVISH_CC(L)                                                                      \
  case L:                                                                                 \
    if (lap) hipLaunchKernelGGL((cost_coeffs_kernel<L, true>), dim3(grid), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((cost_coeffs_kernel<L, false>), dim3(grid), dim3(256), 0, s, a);    \
    break;
  switch (logn) {
    LAVISH_CC(4)
    LAVISH_CC(5)
    LAVISH_CC(6)
    LAVISH_CC(7)
    LAVISH_CC(8)
    LAVISH_CC(9)
    LAVISH_CC(10)
    default: return -1;
  }
#undef LAVISH_CC
  LAVISH_CHECK(hipGetLastError());
  return 0;
}
