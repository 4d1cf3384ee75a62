// trellis.hip -- the coefficient trellis of a batch of transform blocks on
// gfx950.
//
// Reference: av1_optimize_b (av1/encoder/encodemb.c:87-103) ->
// av1_optimize_txb (av1/encoder/txb_rdopt.c:326-449), no quantization
// matrix (the default PSNR metric; a flat iqmatrix changes nothing):
//   rdmult = (x->rdmult * (plane_rd_mult[is_inter][plane_type] << 2(bd-8))
//             + 2) >> (sharpness + 2);
//   the last coefficient: update_coeff_general (|q| >= 2) or its eob cost;
//   update_coeff_eob (:128-244) while at most 2 nonzeros are kept -- each
//   nonzero may become the new last one, dropping those after it;
//   update_skip (:246-262) when the walk reached DC that way;
//   update_coeff_simple (:75-126) down to scan index 1 -- lower |q| by one
//   when RDCOST says so; update_coeff_general (:17-73) at DC;
//   rate = accumulated rate + skip / non-skip (+ tx-type) cost, and
//   av1_get_txb_entropy_context (encodetxb.c:451-467) of the result.
//
// The walk is a chain: every decision reads the |level| map as the decisions
// after it in scan order left it, and update_coeff_eob also reads the
// running rate / distortion.  So one lane runs one block's whole walk; a
// wave holds 64 (32 for 32x32) independent blocks.  The lane's padded
// |level| map (av1_txb_init_levels layout) lives in LDS; the block's
// LV_MAP_COEFF_COST / LV_MAP_EOB_COST and the scan are staged in LDS once per
// workgroup; coefficients are read / rewritten in place in global memory.
#include "coeffcost_dev.h"
#include "lavish_internal.h"

namespace lavish {
namespace {

using namespace cc;

struct TrArgs {
  const int32_t* cost;  // LV_MAP_COEFF_COST of (txs_ctx, plane_type)
  const int32_t* eobc;  // LV_MAP_EOB_COST of (eob_multi_size, plane_type)
  const int32_t* tcoeff;
  int32_t* qcoeff;
  int32_t* dqcoeff;
  uint16_t* eob;
  const LavishTxbCtx* ctx;
  const int16_t* scan;
  int32_t* rate;
  uint8_t* entropy;
  int64_t rdmult;  // the trellis's scaled rdmult
  int nblocks, n, w, h, bhl, cls, wlt, wgt, shift, sharpness;
  int dqv_dc, dqv_ac, tx_type_cost, non_skip_plane;
};

// the lane's walk state and the block-invariant context
struct Walk {
  const int32_t* tab;  // LDS: cost cells, then the eob cells
  const int16_t* scan; // LDS
  uint8_t* lv;         // LDS: this lane's |level| map
  const int32_t* tc;
  int32_t* qc;
  int32_t* dqc;
  int64_t rdmult;
  int n, h, bhl, stride, cls, wlt, wgt, shift, sharpness, dqv_dc, dqv_ac, dc_sign_ctx;
  NbrOff nb;  // the class's neighbour offsets in the level map

  // RDCOST (av1/encoder/rd.h:31-33)
  __device__ __forceinline__ int64_t rd(int64_t r, int64_t d) const {
    return ((r * rdmult + 256) >> 9) + d * 128;
  }
  // get_coeff_dist without a qmatrix (txb_rdopt_utils.h:48-66)
  __device__ __forceinline__ int64_t dist(int32_t t, int32_t d) const {
    const int64_t x = (int32_t)((t - d) * (1 << shift));
    return x * x;
  }
  __device__ __forceinline__ int col_of(int ci) const { return ci >> bhl; }
  __device__ __forceinline__ int row_of(int ci) const { return ci & (h - 1); }
  __device__ __forceinline__ void set_level(int ci, int v) const {
    lv[col_of(ci) * stride + row_of(ci)] = (uint8_t)min(v, 127);
  }
  __device__ __forceinline__ int lower(int ci) const {
    return lower_ctx_off(nb, cls, wlt, wgt, lv, stride, ci, col_of(ci), row_of(ci));
  }
  // get_lower_levels_ctx_eob (txb_common.h:229-234)
  __device__ __forceinline__ int eob_ctx(int si) const {
    return si == 0 ? 0 : (si <= (n >> 3) ? 1 : (si <= (n >> 2) ? 2 : 3));
  }
  __device__ __forceinline__ int sign_cost(int ci, int sign) const {
    return ci == 0 ? tab[kDcSign + dc_sign_ctx * 2 + sign] : 512;
  }
  // get_coeff_cost_eob (txb_rdopt_utils.h:155-172)
  __device__ __forceinline__ int cost_eob(int ci, int a, int sign, int ctx) const {
    int c = tab[kBaseEob + ctx * 3 + min3(a) - 1];
    if (a) {
      c += sign_cost(ci, sign);
      if (a > 2) c += br_cost(tab, br_ctx_eob(cls, ci, col_of(ci), row_of(ci)), a);
    }
    return c;
  }
  // get_coeff_cost_general (txb_rdopt_utils.h:174-194)
  __device__ __forceinline__ int cost_general(bool last, int ci, int a, int sign, int ctx) const {
    if (last) return cost_eob(ci, a, sign, ctx);
    int c = tab[kBase + ctx * 8 + min3(a)];
    if (a) {
      c += sign_cost(ci, sign);
      if (a > 2) c += br_cost(tab, br_ctx_off(nb, cls, lv, stride, ci, col_of(ci), row_of(ci)), a);
    }
    return c;
  }
  // get_eob_cost (txb_rdopt_utils.h:70-84)
  __device__ __forceinline__ int eob_cost(int eob) const {
    const int t = eob < 3 ? eob : 33 - __clz(eob - 1);
    const int bits = t >= 3 ? t - 2 : 0;
    int c = tab[kCostCells + (cls ? 11 : 0) + t - 1];
    if (bits > 0) {
      const int extra = eob - ((1 << (t - 2)) + 1);
      c += tab[kEobExtra + (t - 3) * 2 + ((extra >> (bits - 1)) & 1)] + (bits - 1) * 512;
    }
    return c;
  }
  __device__ __forceinline__ int dqv(int ci) const { return ci ? dqv_ac : dqv_dc; }

  // update_coeff_general (txb_rdopt.c:17-73)
  __device__ __forceinline__ void general(int& accu_rate, int64_t& accu_dist, int si, int eob) const {
    const int ci = scan[si];
    const int32_t q = qc[ci];
    const bool last = si == eob - 1;
    const int ctx = last ? eob_ctx(si) : lower(ci);
    if (q == 0) {
      accu_rate += tab[kBase + ctx * 8];
      return;
    }
    const int sign = q < 0, a = abs(q);
    const int32_t t = tc[ci];
    const int64_t d = dist(t, dqc[ci]), d0 = dist(t, 0);
    const int r = cost_general(last, ci, a, sign, ctx);
    int32_t ql = 0, dql = 0;
    int al = 0, rl;
    int64_t dl;
    if (a == 1) {
      dl = d0;
      rl = tab[kBase + ctx * 8];
    } else {
      al = a - 1;
      const int32_t adl = (al * dqv(ci)) >> shift;
      ql = sign ? -al : al;
      dql = sign ? -adl : adl;
      dl = dist(t, dql);
      rl = cost_general(last, ci, al, sign, ctx);
    }
    if (rd(rl, dl) < rd(r, d)) {
      qc[ci] = ql;
      dqc[ci] = dql;
      set_level(ci, al);
      accu_rate += rl;
      accu_dist += dl - d0;
    } else {
      accu_rate += r;
      accu_dist += d - d0;
    }
  }

  // update_coeff_simple (txb_rdopt.c:75-126) with get_two_coeff_cost_simple
  // and get_br_cost_with_diff (txb_rdopt_utils.h:106-153)
  __device__ __forceinline__ void simple(int& accu_rate, int si) const {
    const int ci = scan[si];
    const int32_t q = qc[ci];
    const int ctx = lower(ci);
    if (q == 0) {
      accu_rate += tab[kBase + ctx * 8];
      return;
    }
    const int a = abs(q);
    int cost = tab[kBase + ctx * 8 + min3(a)] + 512;
    int diff = a <= 3 ? tab[kBase + ctx * 8 + a + 4] : 0;
    if (a > 2) {
      const int* lps = tab + kLps + br_ctx_off(nb, cls, lv, stride, ci, col_of(ci), row_of(ci)) * 26;
      const int br = min(a - 3, 12);
      cost += lps[br];
      if (a <= 15) diff += lps[br + 13];
      if (a >= 15) {
        const int r = a - 14;
        cost += (2 * (32 - __clz(r)) - 1) * 512;
        diff += r == 1 ? 512 : ((r & (r - 1)) == 0 ? 1024 : 0);
      }
    }
    const int32_t at = abs(tc[ci]), adq = abs(dqc[ci]);
    if (adq < at) {
      accu_rate += cost;
      return;
    }
    const int al = a - 1;
    const int32_t adl = (al * dqv(ci)) >> shift;
    if (rd(cost - diff, dist(at, adl)) < rd(cost, dist(at, adq))) {
      const int sign = q < 0;
      qc[ci] = sign ? -al : al;
      dqc[ci] = sign ? -adl : adl;
      set_level(ci, al);
      accu_rate += cost - diff;
    } else {
      accu_rate += cost;
    }
  }

  // update_coeff_eob (txb_rdopt.c:128-244); nz_ci as three registers
  __device__ __forceinline__ void eob_step(int& accu_rate, int64_t& accu_dist, int& eob, int& nz_num, int& nz0,
                           int& nz1, int& nz2, int si) const {
    const int ci = scan[si];
    const int32_t q = qc[ci];
    const int ctx = lower(ci);
    if (q == 0) {
      accu_rate += tab[kBase + ctx * 8];
      return;
    }
    const int a = abs(q), sign = q < 0;
    const int32_t t = tc[ci];
    const int64_t d0 = dist(t, 0);
    int64_t d = dist(t, dqc[ci]) - d0;
    int r = cost_general(false, ci, a, sign, ctx);
    int64_t cur = rd(accu_rate + r, accu_dist + d);
    int32_t ql = 0, dql = 0;
    int al = 0, rl;
    int64_t dl, rdl;
    if (a == 1) {
      dl = 0;
      rl = tab[kBase + ctx * 8];
      rdl = rd(accu_rate + rl, accu_dist);
    } else {
      al = a - 1;
      const int32_t adl = (al * dqv(ci)) >> shift;
      ql = sign ? -al : al;
      dql = sign ? -adl : adl;
      dl = dist(t, dql) - d0;
      rl = cost_general(false, ci, al, sign, ctx);
      rdl = rd(accu_rate + rl, accu_dist + dl);
    }
    const int ctx_ne = eob_ctx(si);
    const int ne_cost = eob_cost(si + 1);
    int r_ne = ne_cost + cost_eob(ci, a, sign, ctx_ne);
    int64_t d_ne = d;
    int64_t rd_ne = rd(r_ne, d_ne);
    bool lower_ne = false;
    if (al > 0) {
      const int r_nel = ne_cost + cost_eob(ci, al, sign, ctx_ne);
      const int64_t rd_nel = rd(r_nel, dl);
      if (rd_nel < rd_ne) {
        lower_ne = true;
        rd_ne = rd_nel;
        r_ne = r_nel;
        d_ne = dl;
      }
    }
    bool lower_level = false;
    if (sharpness == 0 || a > 1) {
      if (rdl < cur) {
        lower_level = true;
        cur = rdl;
        r = rl;
        d = dl;
      }
    }
    if (sharpness == 0 && rd_ne < cur) {
      // the new last coefficient: drop the kept nonzeros after it
      for (int k = 0; k < nz_num; ++k) {
        const int lc = k == 0 ? nz0 : (k == 1 ? nz1 : nz2);
        set_level(lc, 0);
        qc[lc] = 0;
        dqc[lc] = 0;
      }
      eob = si + 1;
      nz_num = 0;
      accu_rate = r_ne;
      accu_dist = d_ne;
      lower_level = lower_ne;
    } else {
      accu_rate += r;
      accu_dist += d;
    }
    if (lower_level) {
      qc[ci] = ql;
      dqc[ci] = dql;
      set_level(ci, al);
    }
    if (qc[ci]) {
      if (nz_num == 0) nz0 = ci;
      else if (nz_num == 1) nz1 = ci;
      else nz2 = ci;
      ++nz_num;
    }
  }
};

template <int N>
__global__ __launch_bounds__(64) void trellis_kernel(TrArgs a) {
  constexpr int BPW = N >= 1024 ? 32 : 64;  // blocks (lanes) per wave: LDS <= 48 KB
  // max (w + 4) * (h + 4) over the adjusted sizes with w * h = N
  constexpr int LVB = N == 16 ? 64 : N == 32 ? 96 : N == 64 ? 160 : N == 128 ? 240
                    : N == 256 ? 432 : N == 512 ? 720 : 1296;
  __shared__ int32_t tab[kTabCells];
  __shared__ int16_t scan[N];
  __shared__ __attribute__((aligned(4))) uint8_t lvs[BPW * LVB];
  const int lane = threadIdx.x;
  for (int i = lane; i < kCostCells; i += 64) tab[i] = a.cost[i];
  if (lane < kEobCells) tab[kCostCells + lane] = a.eobc[lane];
  for (int i = lane; i < N; i += 64) scan[i] = a.scan[i];
  __syncthreads();
  const int b = blockIdx.x * BPW + lane;
  if (lane >= BPW || b >= a.nblocks) return;

  Walk w;
  w.tab = tab;
  w.scan = scan;
  w.lv = lvs + lane * LVB;
  w.tc = a.tcoeff + (int64_t)b * N;
  w.qc = a.qcoeff + (int64_t)b * N;
  w.dqc = a.dqcoeff + (int64_t)b * N;
  w.rdmult = a.rdmult;
  w.n = N;
  w.h = a.h;
  w.bhl = a.bhl;
  w.stride = a.h + 4;
  w.cls = a.cls;
  w.nb = nbr_off(a.cls, w.stride);
  w.wlt = a.wlt;
  w.wgt = a.wgt;
  w.shift = a.shift;
  w.sharpness = a.sharpness;
  w.dqv_dc = a.dqv_dc;
  w.dqv_ac = a.dqv_ac;
  const LavishTxbCtx tc = a.ctx ? a.ctx[b] : LavishTxbCtx{0, 0};
  w.dc_sign_ctx = tc.dc_sign_ctx;
  const int skip_cost = tab[kSkip + tc.txb_skip_ctx * 2 + 1];
  const int non_skip_cost = tab[kSkip + tc.txb_skip_ctx * 2];

  int eob = a.eob[b];
  if (eob == 0) {  // av1_optimize_b's early exit: av1_cost_skip_txb
    a.rate[b] = skip_cost;
    if (a.entropy) a.entropy[b] = 0;
    return;
  }
  if (eob > 1) {  // av1_txb_init_levels_c
    const int stride = w.stride, h = a.h;
    for (int i = 0; i < (a.w + 4) * stride; ++i) w.lv[i] = 0;
    for (int col = 0; col < a.w; ++col)
      for (int row = 0; row < h; ++row)
        w.lv[col * stride + row] = (uint8_t)min(abs(w.qc[col * h + row]), 127);
  }
  int accu_rate = w.eob_cost(eob);
  int64_t accu_dist = 0;
  int si = eob - 1;
  {
    const int ci = scan[si];
    const int32_t q = w.qc[ci];
    if (abs(q) >= 2) {
      w.general(accu_rate, accu_dist, si, eob);
    } else {
      accu_rate += w.cost_eob(ci, abs(q), q < 0, w.eob_ctx(si));
      accu_dist += w.dist(w.tc[ci], w.dqc[ci]) - w.dist(w.tc[ci], 0);
    }
  }
  int nz_num = 1, nz0 = scan[si], nz1 = 0, nz2 = 0;
  --si;
  for (; si >= 0 && nz_num <= 2; --si)
    w.eob_step(accu_rate, accu_dist, eob, nz_num, nz0, nz1, nz2, si);
  if (si == -1 && nz_num <= 2) {  // update_skip
    if (w.rd(skip_cost, 0) < w.rd(accu_rate + non_skip_cost, accu_dist) && a.sharpness == 0) {
      for (int k = 0; k < nz_num; ++k) {
        const int lc = k == 0 ? nz0 : (k == 1 ? nz1 : nz2);
        w.qc[lc] = 0;
        w.dqc[lc] = 0;
      }
      accu_rate = 0;
      eob = 0;
    }
  }
  for (; si >= 1; --si) w.simple(accu_rate, si);
  if (si == 0) {
    int64_t dummy = 0;
    w.general(accu_rate, dummy, 0, eob);
  }
  accu_rate += eob == 0 ? skip_cost : non_skip_cost + a.tx_type_cost;
  a.rate[b] = accu_rate;
  a.eob[b] = (uint16_t)eob;
  if (a.entropy) {
    int cul = 0;
    for (int c = 0; c < eob && cul <= 7; ++c) cul += abs(w.qc[scan[c]]);
    cul = min(cul, 7);
    if (eob > 0) {
      const int32_t dc = w.qc[0];
      if (dc < 0) cul |= 1 << 3;
      else if (dc > 0) cul += 2 << 3;
    }
    a.entropy[b] = (uint8_t)cul;
  }
}

int ilog2i(int v) { return 31 - __builtin_clz(v); }

}  // namespace
}  // namespace lavish

using namespace lavish;

extern "C" int lavish_optimize_b_batch(const LavishCoeffCosts* costs, const int32_t* tcoeff,
                                       int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob,
                                       int nblocks, int plane, int tx_size, int tx_type,
                                       int bit_depth, int is_inter, int rdmult, int sharpness,
                                       const int16_t* dequant, const LavishTxbCtx* txb_ctx,
                                       int tx_type_cost, int32_t* rate, uint8_t* entropy_ctx,
                                       void* stream) {
  if (tx_size < 0 || tx_size >= 19 || tx_type < 0 || tx_type >= 16) return -1;
  if (plane < 0 || plane > 2 || (is_inter != 0 && is_inter != 1)) return -2;
  if (costs == nullptr || tcoeff == nullptr || qcoeff == nullptr || dqcoeff == nullptr ||
      eob == nullptr || rate == nullptr || dequant == nullptr)
    return -3;
  if (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) return -4;
  if (sharpness < 0 || sharpness > 7) return -5;
  if (nblocks <= 0) return 0;
  static const int plane_rd_mult[2][2] = {{17, 13}, {16, 10}};  // encodetxb.h:266-269
  const int txw = tx_w(tx_size), txh = tx_h(tx_size);
  const int w = txw > 32 ? 32 : txw, h = txh > 32 ? 32 : txh;
  const int mn = txw < txh ? txw : txh, mx = txw < txh ? txh : txw;
  const int txs_ctx = (ilog2i(mn) - 2 + ilog2i(mx) - 2 + 1) >> 1;  // get_txsize_entropy_ctx
  const int pt = plane > 0;
  TrArgs a{};
  a.cost = &costs->coeff_costs[txs_ctx][pt].txb_skip_cost[0][0];
  a.eobc = &costs->eob_costs[ilog2i(w * h) - 4][pt].eob_cost[0][0];
  a.tcoeff = tcoeff;
  a.qcoeff = qcoeff;
  a.dqcoeff = dqcoeff;
  a.eob = eob;
  a.ctx = txb_ctx;
  a.scan = dev_scan(tx_size, tx_type);
  a.rate = rate;
  a.entropy = entropy_ctx;
  a.rdmult = (((int64_t)rdmult * (plane_rd_mult[is_inter][pt] << (2 * (bit_depth - 8)))) + 2) >>
             (sharpness + 2);
  a.nblocks = nblocks;
  a.n = w * h;
  a.w = w;
  a.h = h;
  a.bhl = ilog2i(h);
  a.cls = cc::tx_class(tx_type);
  a.wlt = txw < txh;
  a.wgt = txw > txh;
  a.shift = tx_scale(tx_size);
  a.sharpness = sharpness;
  a.dqv_dc = dequant[0];
  a.dqv_ac = dequant[1];
  a.tx_type_cost = plane == 0 ? tx_type_cost : 0;  // get_tx_type_cost: 0 for plane > 0
  hipStream_t s = (hipStream_t)stream;
  const int bpw = a.n >= 1024 ? 32 : 64;
  const int grid = (nblocks + bpw - 1) / bpw;
#define LAVISH_TR(NN) \
  case NN: hipLaunchKernelGGL((trellis_kernel<NN>), dim3(grid), dim3(64), 0, s, a); break;
  switch (a.n) {
    LAVISH_TR(16)
    LAVISH_TR(32)
    LAVISH_TR(64)
    LAVISH_TR(128)
    LAVISH_TR(256)
    LAVISH_TR(512)
    LAVISH_TR(1024)
    default: return -1;
  }
#undef LAVISH_TR
  LAVISH_CHECK(hipGetLastError());
  return 0;
}
