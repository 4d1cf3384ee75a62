// rdo.hip -- C4 host side: the per-size decision launches (kernels in
// rdo_kern.h, instantiated per mode in rdo_m0..3.hip), the frame-level step
// (every candidate size, the per-SB TX-size decision, the reconstruction),
// the 64-point pixel-domain path and the captured step (HIP graph).
#include <cstddef>
#include "rdo_kern.h"

namespace lavish {

namespace {

int fill_types(RdoArgs& a, int tx_size, uint32_t type_mask) {
  a.ntypes = 0;
  for (int t = 0; t < 16; ++t) {
    if (!((type_mask >> t) & 1)) continue;
    if (!tx_type_valid(tx_size, t)) return -5;
    a.iscan_type[a.ntypes] = dev_iscan(tx_size, t);
    a.scan_kind[a.ntypes] = scan_kind(t);
    a.types[a.ntypes++] = t;
  }
  a.scan_rows = dev_iscan_rows(tx_size);
  int n = 0;
  for (int vk = 0; vk < 4; ++vk) {
    bool first = true;
    for (int i = 0; i < a.ntypes; ++i) {
      if (((kVtxPacked >> (2 * a.types[i])) & 3) != (uint32_t)vk) continue;
      a.order[n] = i;
      a.newcol[n++] = first;
      first = false;
    }
  }
  return a.ntypes == 0 ? -5 : 0;
}

QP qp_of(const LavishQuantParams* p) {
  QP q{};
  for (int i = 0; i < 2; ++i) {
    q.zbin[i] = p->zbin[i];
    q.round[i] = p->round[i];
    q.quant[i] = p->quant[i];
    q.quant_shift[i] = p->quant_shift[i];
    q.dequant[i] = p->dequant[i];
  }
  return q;
}

}  // namespace

// lavish_txq_plane for the 64-point sizes (called from txq.hip)
int txq_plane_64(const int16_t* residual, int stride, int width, int height, int tx_size,
                 uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
                 int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff,
                 hipStream_t s) {
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  RdoArgs a{};
  a.res = residual;
  a.stride = stride;
  a.bw = width / W;
  a.nblocks = (width / W) * (height / H);
  const int rc = fill_types(a, tx_size, type_mask);
  if (rc) return rc;
  a.bd = bd;
  a.quant_kind = quant_kind;
  a.highbd = bd > 8;
  if (qp) a.qp = qp_of(qp);
  a.qcoeff = qcoeff;
  a.dqcoeff = dqcoeff;
  a.eob = eob;
  a.coeff = coeff;
  return rdo_launch_m0(tx_size, a, s);
}

// 64-point sizes with pixel-domain distortion (one candidate type: DCT_DCT):
// the TX-domain decision kernel, then the inverse of its winner into a
// scratch copy of the prediction, the pixel SSE and the reference's
// TX_64X64 / high-energy rules (px64_finish_kernel).
int rdo_plane_px64(RdoArgs& a, int tx_size, int width, int height, hipStream_t s);

int rdo_plane(const uint16_t* src, const uint16_t* pred, int stride, int width, int height,
              int tx_size, uint32_t type_mask, int bd, const LavishQuantParams* qp, int rdmult,
              LavishRdoBlock* out, int32_t* qcoeff, int32_t* dqcoeff, hipStream_t s, int px,
              const uint16_t* block_mask, const uint8_t* block_map, const RateCfg* rate,
              RdoArgs* args_only) {
  if (tx_size < 0 || tx_size >= 19) return -1;
  if (qp == nullptr || out == nullptr || qcoeff == nullptr || dqcoeff == nullptr) return -3;
  if (bd != 8 && bd != 10 && bd != 12) return -3;
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  if (width <= 0 || height <= 0 || stride < width) return -4;
  RdoArgs a{};
  a.src = src;
  a.pred = pred;
  a.stride = stride;
  a.bw = width / W;
  a.nblocks = (width / W) * (height / H);
  const int rc = fill_types(a, tx_size, type_mask);
  if (rc) return rc;
  a.bd = bd;
  a.rdmult = rdmult;
  a.qp = qp_of(qp);
  a.iscan_dct = dev_iscan(tx_size, 0);
  a.out = out;
  a.qcoeff = qcoeff;
  a.dqcoeff = dqcoeff;
  a.block_mask = block_mask;
  a.block_map = block_map;
  if (rate != nullptr) {
    if (px) return -7;  // the coefficient rate is built for TX-domain distortion
    if (rate->costs == nullptr) return -3;
    const int txw = W, txh = H;
    const int w = txw > 32 ? 32 : txw, h = txh > 32 ? 32 : txh;
    const int mn = txw < txh ? txw : txh, mx = txw < txh ? txh : txw;
    const int lg_mn = 31 - __builtin_clz(mn), lg_mx = 31 - __builtin_clz(mx);
    const int txs_ctx = (lg_mn - 2 + lg_mx - 2 + 1) >> 1;        // get_txsize_entropy_ctx
    const int eob_multi = 31 - __builtin_clz(w * h) - 4;         // txsize_log2_minus4
    a.cc_cost = &rate->costs->coeff_costs[txs_ctx][0].txb_skip_cost[0][0];
    a.cc_eob = &rate->costs->eob_costs[eob_multi][0].eob_cost[0][0];
    a.txb_ctx = rate->txb_ctx;
    for (int t = 0; t < 16; ++t) a.tx_type_cost[t] = rate->tx_type_costs ? rate->tx_type_costs[t] : 0;
    a.nz_wlt = txw < txh;
    a.nz_wgt = txw > txh;
    return rdo_launch_m3(tx_size, a, s);
  }
  if (px) {
    if (W > 32 || H > 32) {
      if (block_mask || block_map) return -6;  // single-type path
      return rdo_plane_px64(a, tx_size, width, height, s);
    }
    return rdo_launch_m2(tx_size, a, s);
  }
  if (args_only != nullptr) {  // the caller launches (rdo_frame's small-size launch)
    *args_only = a;
    return 0;
  }
  return rdo_launch_m1(tx_size, a, s);
}

// ---------------------------------------------------------------------------
// frame level: every candidate TX size of a frame, the per-superblock TX-size
// decision and the reconstruction
// ---------------------------------------------------------------------------
int rdo_frame(const uint16_t* src, const uint16_t* pred, int stride, int width, int height,
              uint32_t size_mask, const uint32_t* type_masks, int bd,
              const LavishQuantParams* qp, int rdmult, LavishRdoBlock* const* out,
              int32_t* const* qcoeff, int32_t* const* dqcoeff, hipStream_t caller, int px = 0) {
  int order[19], n = 0;
  for (int s = 0; s < 19; ++s)
    if ((size_mask >> s) & 1) order[n++] = s;
  // most work first, dealt round-robin over the internal streams (measured
  // against least work first, so the few-wave, latency-bound large sizes
  // start beside the small sizes' kernels: that was slower, 0.821-0.840 vs
  // 0.811-0.829 ms per 4K step, profiles/r04_v13_ab_notes.txt)
  auto work = [&](int s) {
    return (long)__builtin_popcount(type_masks[s]) * (width / tx_w(s)) * (height / tx_h(s)) *
           max_eob(s);
  };
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && work(order[j]) > work(order[j - 1]); --j) {
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  // small rectangles: 16x16, 8x8 and 4x4 (all three present, each in the
  // split form with four kind groups) as one launch on the caller's stream,
  // the other sizes on the internal streams beside it
  bool small = !px && fan_width() > 1;
  RdoSmall sm{};
  const int ssz[3] = {2, 1, 0};
  for (int k = 0; k < 3 && small; ++k) {
    const int t = ssz[k];
    if (!((size_mask >> t) & 1)) {
      small = false;
      break;
    }
    const int tiles = (width / tx_w(t)) * (height / tx_h(t)) * tx_w(t) / 64;  // P = 64 / w
    int groups = 0;
    RdoArgs& a = sm.a[k];
    const int rc = rdo_plane(src, pred, stride, width, height, t, type_masks[t], bd, qp, rdmult,
                             out[t], qcoeff[t], dqcoeff[t], caller, 0, nullptr, nullptr, nullptr,
                             &a);
    if (rc) return rc;
    for (int i = 0; i < a.ntypes; ++i) groups += a.newcol[i];
    if (groups != 4 || tiles >= kRdoSplitTiles) small = false;
    sm.first[k + 1] = sm.first[k] + (a.nblocks + 64 / tx_w(t) - 1) / (64 / tx_w(t));
  }
  hipStream_t* fs = fan_out(caller);
  int rc = 0;
  if (small) rc = rdo_small_launch_m1(sm, caller);
  for (int i = 0, k = 0; i < n && rc == 0; ++i) {
    const int s = order[i];
    if (small && (s == 0 || s == 1 || s == 2)) continue;
    // (small: the internal streams first, the caller's stream runs the
    // small-size launch)
    const int w = fan_width();
    // (measured against all of them on one internal stream or on the
    // caller's after the small-size launch: 0.1595 vs 0.1619 / 0.1608 ms per
    // C5 rank at G = 8, 3.36 vs 3.65 / 3.86 ms for the row wavefront)
    hipStream_t st = small && w > 1 ? fs[1 + k++ % (w - 1)] : fs[i % w];
    rc = rdo_plane(src, pred, stride, width, height, s, type_masks[s], bd, qp, rdmult, out[s],
                   qcoeff[s], dqcoeff[s], st, px);
  }
  fan_in(caller);
  return rc;
}

namespace {

__constant__ uint8_t kTxWd[19] = {4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64};
__constant__ uint8_t kTxHd[19] = {4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16};
__device__ __forceinline__ int tx_w_dev(int s) { return kTxWd[s]; }
__device__ __forceinline__ int tx_h_dev(int s) { return kTxHd[s]; }
// av1_get_max_eob (av1/common/blockd.h:1596-1604)
__device__ __forceinline__ int max_eob_dev(int s) {
  const int w = kTxWd[s], h = kTxHd[s];
  if (w == 64 || h == 64) return (w == 16 || h == 16) ? 512 : 1024;
  return w * h;
}

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
  return a > INT64_MAX - b ? INT64_MAX : a + b;
}

// sb_decide reads a block's (best_type, eob) as one 8-byte word
static_assert(offsetof(LavishRdoBlock, best_type) == 0 && offsetof(LavishRdoBlock, eob) == 4,
              "LavishRdoBlock layout");

struct SbArgs {
  int nsizes;
  int sizes[19];                       // candidate order: largest area first
  const LavishRdoBlock* rec[19];
  LavishInvJob* jobs[19];              // per size: one slot of `cap` jobs per SB
  uint16_t* cnt[19];                   // per size and SB: its live jobs
  int sbw, sbh;                        // superblocks per row / column
  int width, height, stride;
  uint8_t* sb_tx_size;
  const uint16_t* pred;                // the SB's recon = pred, before the inverse adds
  uint16_t* recon;
};

// per SB64: the candidate TX size whose blocks' summed RD cost is lowest
// (sizes that do not tile the SB with full blocks are skipped; ties keep
// the earlier, larger size), then the inverse-transform jobs of that size's
// blocks with eob > 0 -- a block with eob 0 adds nothing
// (av1_inverse_transform_block, idct.c:308) and the other sizes' blocks are
// not reconstructed at all.
// One wave64 per SB: lanes stride the SB's blocks of a size, a 64-bit xor
// reduction sums their costs; the size scan stays sequential (strict <).
// The wave also writes the SB's reconstruction base (recon = pred), which
// the inverse adds then build on.
// Jobs go to the SB's own slot of each size's list (no atomics, nothing to
// zero first): the chosen size's coded blocks, compacted by ballot, and a
// count of 0 in every other size's slot.
__global__ __launch_bounds__(256) void sb_decide_kernel(SbArgs a) {
  const int sb = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (sb >= a.sbw * a.sbh) return;
  const int sy = sb / a.sbw, sx = sb - sy * a.sbw;
  const int y1 = min(64, a.height - sy * 64), x1 = min(64, a.width - sx * 64);
  // recon = pred over the SB: 16-byte rows when the SB is whole and aligned.
  // Every load of the wave -- the copy's rows, and per candidate size its
  // blocks' costs and (type, eob) pairs -- is issued before the first store
  // or use, so the decision and the job list cost one memory latency, not
  // three (copy, costs, then the chosen size's records).
  const size_t o = (size_t)sy * 64 * a.stride + (size_t)sx * 64;
  const uint16_t* p = a.pred + o;
  uint16_t* r = a.recon + o;
  const bool vec = x1 == 64 && ((((uintptr_t)p | (uintptr_t)r | ((uintptr_t)a.stride * 2)) & 15) == 0);
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  u4 cp[8];
  if (vec) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = i * 8 + (lane >> 3);
      if (row < y1) cp[i] = *(const u4*)(p + (size_t)row * a.stride + 8 * (lane & 7));
    }
  }
  int64_t best = INT64_MAX;
  int best_s = 255, best_i = -1;
  // costs are >= 0; a block without a candidate costs INT64_MAX, so the sums
  // saturate there instead of wrapping (a sum of non-negative costs
  // saturating at INT64_MAX is order-free).  nblk <= 256: up to 4 blocks
  // per lane; the first kMaxSbSizes sizes' loads are all in flight together
  constexpr int kMaxSbSizes = 5;
  int64_t vv[kMaxSbSizes][4];
  uint64_t mm[kMaxSbSizes][4];  // (best_type, eob) of the same blocks
#pragma unroll
  for (int i = 0; i < kMaxSbSizes; ++i) {
    const int s = i < a.nsizes ? a.sizes[i] : a.sizes[0];
    const int W = tx_w_dev(s), H = tx_h_dev(s);
    const bool tiles = i < a.nsizes && !(y1 % H || x1 % W);
    const int bw = a.width / W, nx = max(x1 / W, 1), nblk = tiles ? (x1 / W) * (y1 / H) : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = lane + 64 * q;
      const int y = k / nx, x = k - y * nx;
      const LavishRdoBlock* rb = a.rec[s] + ((sy * 64 / H + y) * bw + sx * 64 / W + x);
      vv[i][q] = k < nblk ? rb->rdcost : 0;
      mm[i][q] = k < nblk ? *(const uint64_t*)rb : 0;
    }
  }
  if (vec) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = i * 8 + (lane >> 3);
      if (row < y1) *(u4*)(r + (size_t)row * a.stride + 8 * (lane & 7)) = cp[i];
    }
  } else {
    for (int row = 0; row < y1; ++row)
      if (lane < x1) r[(size_t)row * a.stride + lane] = p[(size_t)row * a.stride + lane];
  }
  for (int i = 0; i < a.nsizes; ++i) {
    const int s = a.sizes[i];
    const int W = tx_w_dev(s), H = tx_h_dev(s);
    if (y1 % H || x1 % W) continue;
    const int bw = a.width / W, nx = x1 / W, nblk = nx * (y1 / H);
    int64_t v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = lane + 64 * q;
      const int y = k / nx, x = k - y * nx;
      v[q] = i < kMaxSbSizes ? vv[i < kMaxSbSizes ? i : 0][q]
                             : (k < nblk ? a.rec[s][(sy * 64 / H + y) * bw + sx * 64 / W + x].rdcost : 0);
    }
    int64_t sum = sat_add(sat_add(v[0], v[1]), sat_add(v[2], v[3]));
    sum = (int64_t)lane_reduce64<64>((uint64_t)sum, [](uint64_t x, uint64_t y) {
      return (uint64_t)sat_add((int64_t)x, (int64_t)y);
    });
    if (sum < best) {
      best = sum;
      best_s = s;
      best_i = i;
    }
  }
  if (lane == 0) {
    a.sb_tx_size[sb] = (uint8_t)best_s;
    for (int i = 0; i < a.nsizes; ++i)
      if (a.sizes[i] != best_s) a.cnt[a.sizes[i]][sb] = 0;
  }
  if (best_s == 255) return;  // no candidate tiles this SB: recon = pred
  const int s = best_s;
  const int W = tx_w_dev(s), H = tx_h_dev(s);
  const int bw = a.width / W, nx = x1 / W, nblk = nx * (y1 / H), n = max_eob_dev(s);
  LavishInvJob* const slot = a.jobs[s] + (size_t)sb * ((64 / W) * (64 / H));
  int base = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (64 * q >= nblk) break;
    const int k = 64 * q + lane;
    const int y = k / nx, x = k - y * nx;
    const int blk = (sy * 64 / H + y) * bw + sx * 64 / W + x;
    const bool live = k < nblk;
    // the chosen size's (type, eob): from the batch above (a select over the
    // sizes, no indexed private array), or loaded for a 6th+ size
    uint64_t te = 0;
#pragma unroll
    for (int i = 0; i < kMaxSbSizes; ++i) te = best_i == i ? mm[i][q] : te;
    if (best_i >= kMaxSbSizes) te = live ? *(const uint64_t*)(a.rec[s] + blk) : 0;
    const int32_t btype = (int32_t)(uint32_t)te, beob = (int32_t)(te >> 32);
    const bool coded = live && beob != 0;
    const uint64_t m = __builtin_amdgcn_ballot_w64(coded);
    if (coded) {
      const int at = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      LavishInvJob j;
      j.dst_off = (int64_t)(sy * 64 + y * H) * a.stride + sx * 64 + x * W;
      j.coeff_off = (int64_t)blk * n;
      j.tx_type = btype;
      j.eob = beob;
      slot[at] = j;
    }
    base += __popcll(m);
  }
  if (lane == 0) a.cnt[s][sb] = (uint16_t)base;
}

// inverse-transform job list of lavish_rdo_reconstruct: reused call after
// call, possibly from different streams (e.g. per-band streams of a shard),
// so reuse is ordered by StreamScratch's event
thread_local StreamScratch t_rs;

}  // namespace

namespace {

// px64 helpers: inverse jobs of the TX-domain winners, then per block the
// pixel SSE and the distortion rules of search_tx_type (tx_search.c:2187-2231)
__global__ void px64_jobs_kernel(const LavishRdoBlock* rec, int nblocks, int bw, int W, int H,
                                 int n, int stride, LavishInvJob* jobs) {
  const int blk = blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= nblocks) return;
  const int by = blk / bw, bx = blk - by * bw;
  LavishInvJob j;
  j.dst_off = (int64_t)by * H * stride + (int64_t)bx * W;
  j.coeff_off = (int64_t)blk * n;
  j.tx_type = rec[blk].best_type;
  j.eob = rec[blk].eob;
  jobs[blk] = j;
}

__global__ __launch_bounds__(256) void px64_finish_kernel(const uint16_t* src, const uint16_t* pred,
                                                          const uint16_t* recon, int stride,
                                                          int bw, int W, int H, int is64, int bd,
                                                          int rdmult, LavishRdoBlock* rec) {
  const int blk = blockIdx.x;
  const int by = blk / bw, bx = blk - by * bw;
  const size_t base = (size_t)by * H * stride + (size_t)bx * W;
  uint64_t s1 = 0, s2 = 0;
  for (int i = threadIdx.x; i < W * H; i += 256) {
    const size_t o = base + (size_t)(i / W) * stride + (i % W);
    const int64_t d1 = (int64_t)src[o] - pred[o], d2 = (int64_t)src[o] - recon[o];
    s1 += (uint64_t)(d1 * d1);
    s2 += (uint64_t)(d2 * d2);
  }
  __shared__ uint64_t r1[4], r2[4];
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    s1 += __shfl_xor(s1, m);
    s2 += __shfl_xor(s2, m);
  }
  if ((threadIdx.x & 63) == 0) {
    r1[threadIdx.x >> 6] = s1;
    r2[threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  s1 = r1[0] + r1[1] + r1[2] + r1[3];
  s2 = r2[0] + r2[1] + r2[2] + r2[3];
  const int sh = 2 * (bd - 8);
  if (sh > 0) {
    s1 = (s1 + ((uint64_t)1 << (sh - 1))) >> sh;
    s2 = (s2 + ((uint64_t)1 << (sh - 1))) >> sh;
  }
  const int64_t bsse = (int64_t)s1 * 16;
  LavishRdoBlock o = rec[blk];
  int64_t dist = o.dist;
  if (o.eob == 0) {
    dist = bsse;
  } else {
    const bool high = bsse >= (int64_t)128 * 128 * W * H;
    const int64_t sse_diff = bsse - o.sse;
    if (!is64 || !high || sse_diff * 2 < o.sse) {
      const int64_t pxd = (int64_t)(uint32_t)(16u * (uint32_t)s2);
      dist = (high && pxd < dist) ? dist : pxd;
    } else {
      dist += sse_diff;
    }
  }
  o.dist = dist;
  o.sse = bsse;
  o.rdcost = (((int64_t)o.rate * rdmult + 256) >> 9) + dist * 128;
  rec[blk] = o;
}

// per TX size: rdo_frame_px deals the 64-point sizes over concurrent fan-out
// streams, so each size owns its scratch plane / job list, and reuse across
// calls (any stream) waits for the previous user's event
thread_local StreamScratch t_px_plane[19], t_px_jobs[19];

}  // namespace

int rdo_plane_px64(RdoArgs& a, int tx_size, int width, int height, hipStream_t s) {
  if (a.ntypes != 1) return -6;  // 64-point sizes have one candidate type
  int rc = rdo_launch_m1(tx_size, a, s);
  if (rc || a.nblocks == 0) return rc;
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  uint16_t* plane = (uint16_t*)t_px_plane[tx_size].acquire(
      (size_t)a.stride * height * sizeof(uint16_t), s);
  LavishInvJob* jobs =
      (LavishInvJob*)t_px_jobs[tx_size].acquire((size_t)a.nblocks * sizeof(LavishInvJob), s);
  LAVISH_CHECK(hipMemcpy2DAsync(plane, (size_t)a.stride * 2, a.pred, (size_t)a.stride * 2,
                                (size_t)width * 2, height, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(px64_jobs_kernel, dim3((a.nblocks + 255) / 256), dim3(256), 0, s, a.out,
                     a.nblocks, a.bw, W, H, max_eob(tx_size), a.stride, jobs);
  LAVISH_CHECK(hipGetLastError());
  rc = inv_txfm_add_batch(a.dqcoeff, tx_size, jobs, a.nblocks, plane, a.stride, a.bd, 1, s);
  if (rc == 0) {
    hipLaunchKernelGGL(px64_finish_kernel, dim3(a.nblocks), dim3(256), 0, s, a.src, a.pred,
                       plane, a.stride, a.bw, W, H, tx_size == 4 ? 1 : 0, a.bd, a.rdmult,
                       a.out);
    LAVISH_CHECK(hipGetLastError());
  }
  // both scratches are released on every path: the copy and the job kernel
  // are already queued on `s`, so a later acquire must wait for them
  t_px_plane[tx_size].release(s);
  t_px_jobs[tx_size].release(s);
  return rc;
}

// reconstruction scratch: per candidate size one slot of (64 / w) x (64 / h)
// jobs per SB, then the SBs' job counts; offsets into it
size_t recon_scratch_layout(const SbArgs& a, int nsb, size_t (&joff)[19], size_t (&coff)[19]) {
  size_t bytes = 0;
  for (int i = 0; i < a.nsizes; ++i) {
    const int t = a.sizes[i];
    joff[t] = bytes;
    bytes += (size_t)nsb * (64 / tx_w(t)) * (64 / tx_h(t)) * sizeof(LavishInvJob);
  }
  for (int i = 0; i < a.nsizes; ++i) {
    const int t = a.sizes[i];
    coff[t] = bytes;
    bytes += ((size_t)nsb * sizeof(uint16_t) + 15) & ~(size_t)15;
  }
  return bytes;
}

// scratch_out: nullptr -> the per-thread stream-ordered scratch; else the
// caller's buffer of recon_scratch_bytes() (a captured graph owns one)
int rdo_reconstruct_impl(uint32_t size_mask, const LavishRdoBlock* const* rec,
                         const int32_t* const* dqcoeff, int width, int height,
                         const uint16_t* pred, uint16_t* recon, int stride, int bd,
                         uint8_t* sb_tx_size, hipStream_t s, char* own_scratch,
                         size_t* scratch_bytes);

int rdo_reconstruct(uint32_t size_mask, const LavishRdoBlock* const* rec,
                    const int32_t* const* dqcoeff, int width, int height, const uint16_t* pred,
                    uint16_t* recon, int stride, int bd, uint8_t* sb_tx_size, hipStream_t s) {
  return rdo_reconstruct_impl(size_mask, rec, dqcoeff, width, height, pred, recon, stride, bd,
                              sb_tx_size, s, nullptr, nullptr);
}

int rdo_reconstruct_impl(uint32_t size_mask, const LavishRdoBlock* const* rec,
                         const int32_t* const* dqcoeff, int width, int height,
                         const uint16_t* pred, uint16_t* recon, int stride, int bd,
                         uint8_t* sb_tx_size, hipStream_t s, char* own_scratch,
                         size_t* scratch_bytes) {
  SbArgs a{};
  for (int t = 0; t < 19; ++t)
    if ((size_mask >> t) & 1) a.sizes[a.nsizes++] = t;
  if (a.nsizes == 0) return -1;
  for (int i = 1; i < a.nsizes; ++i)  // largest area first
    for (int j = i; j > 0 && tx_w(a.sizes[j]) * tx_h(a.sizes[j]) >
                                 tx_w(a.sizes[j - 1]) * tx_h(a.sizes[j - 1]); --j) {
      const int t = a.sizes[j];
      a.sizes[j] = a.sizes[j - 1];
      a.sizes[j - 1] = t;
    }
  for (int i = 0; i < a.nsizes; ++i) a.rec[a.sizes[i]] = rec[a.sizes[i]];
  a.sbw = (width + 63) / 64;
  a.sbh = (height + 63) / 64;
  a.width = width;
  a.height = height;
  a.stride = stride;
  a.sb_tx_size = sb_tx_size;
  a.pred = pred;
  a.recon = recon;
  const int nsb = a.sbw * a.sbh;
  size_t joff[19] = {}, coff[19] = {};
  const size_t bytes = recon_scratch_layout(a, nsb, joff, coff);
  if (scratch_bytes != nullptr) {  // size query
    *scratch_bytes = bytes;
    if (own_scratch == nullptr) return 0;
  }
  const bool shared = own_scratch == nullptr;
  char* scratch = shared ? (char*)t_rs.acquire(bytes, s) : own_scratch;
  for (int i = 0; i < a.nsizes; ++i) {
    const int t = a.sizes[i];
    a.jobs[t] = (LavishInvJob*)(scratch + joff[t]);
    a.cnt[t] = (uint16_t*)(scratch + coff[t]);
  }
  // the decision and recon = pred, then the chosen coded blocks' residuals
  // added by one launch over every size (recon_sb_kernel, inv.hip): every SB
  // chose one size, so the tiles write disjoint pixels
  hipLaunchKernelGGL(sb_decide_kernel, dim3((nsb + 3) / 4), dim3(256), 0, s, a);
  LAVISH_CHECK(hipGetLastError());
  InvSbArgs ia{};
  for (int i = 0; i < a.nsizes; ++i) {
    const int t = a.sizes[i];
    ia.dq[t] = dqcoeff[t];
    ia.jobs[t] = a.jobs[t];
    ia.cnt[t] = a.cnt[t];
  }
  ia.sb_tx_size = sb_tx_size;
  ia.nsb = nsb;
  ia.dst = recon;
  ia.stride = stride;
  const int rc = recon_sb_launch(ia, bd, s);
  if (shared) t_rs.release(s);
  return rc;
}

}  // namespace lavish

extern "C" int lavish_rdo_plane(const uint16_t* src, const uint16_t* pred, int stride, int width,
                                int height, int tx_size, uint32_t type_mask, int bit_depth,
                                const LavishQuantParams* qp, int rdmult, LavishRdoBlock* out,
                                int32_t* qcoeff, int32_t* dqcoeff, void* stream) {
  return lavish::rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream);
}

extern "C" int lavish_rdo_plane_px(const uint16_t* src, const uint16_t* pred, int stride,
                                   int width, int height, int tx_size, uint32_t type_mask,
                                   int bit_depth, const LavishQuantParams* qp, int rdmult,
                                   LavishRdoBlock* out, int32_t* qcoeff, int32_t* dqcoeff,
                                   void* stream) {
  return lavish::rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream, 1);
}

extern "C" int lavish_rdo_frame(const uint16_t* src, const uint16_t* pred, int stride, int width,
                                int height, uint32_t size_mask, const uint32_t* type_masks,
                                int bit_depth, const LavishQuantParams* qp, int rdmult,
                                LavishRdoBlock* const* out, int32_t* const* qcoeff,
                                int32_t* const* dqcoeff, void* stream) {
  return lavish::rdo_frame(src, pred, stride, width, height, size_mask, type_masks, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream);
}

extern "C" int lavish_rdo_frame_px(const uint16_t* src, const uint16_t* pred, int stride,
                                   int width, int height, uint32_t size_mask,
                                   const uint32_t* type_masks, int bit_depth,
                                   const LavishQuantParams* qp, int rdmult,
                                   LavishRdoBlock* const* out, int32_t* const* qcoeff,
                                   int32_t* const* dqcoeff, void* stream) {
  return lavish::rdo_frame(src, pred, stride, width, height, size_mask, type_masks, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream, 1);
}

extern "C" int lavish_rdo_reconstruct(uint32_t size_mask, const LavishRdoBlock* const* records,
                                      const int32_t* const* dqcoeff, int width, int height,
                                      const uint16_t* pred, uint16_t* recon, int stride,
                                      int bit_depth, uint8_t* sb_tx_size, void* stream) {
  return lavish::rdo_reconstruct(size_mask, records, dqcoeff, width, height, pred, recon, stride,
                                 bit_depth, sb_tx_size, (hipStream_t)stream);
}

extern "C" int lavish_rdo_plane_masked(const uint16_t* src, const uint16_t* pred, int stride,
                                       int width, int height, int tx_size, uint32_t type_mask,
                                       int bit_depth, const LavishQuantParams* qp, int rdmult,
                                       const uint16_t* block_mask, const uint8_t* block_map,
                                       int pixel_domain, LavishRdoBlock* out, int32_t* qcoeff,
                                       int32_t* dqcoeff, void* stream) {
  return lavish::rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream, pixel_domain ? 1 : 0,
                           block_mask, block_map);
}

extern "C" int lavish_rdo_plane_rate(const uint16_t* src, const uint16_t* pred, int stride,
                                     int width, int height, int tx_size, uint32_t type_mask,
                                     int bit_depth, const LavishQuantParams* qp, int rdmult,
                                     const LavishCoeffCosts* costs, const LavishTxbCtx* txb_ctx,
                                     const int32_t* tx_type_costs, const uint16_t* block_mask,
                                     const uint8_t* block_map, LavishRdoBlock* out,
                                     int32_t* qcoeff, int32_t* dqcoeff, void* stream) {
  const lavish::RateCfg rc{costs, txb_ctx, tx_type_costs};
  return lavish::rdo_plane(src, pred, stride, width, height, tx_size, type_mask, bit_depth, qp,
                           rdmult, out, qcoeff, dqcoeff, (hipStream_t)stream, 0, block_mask,
                           block_map, &rc);
}

// ---------------------------------------------------------------------------
// A captured C4 step: lavish_rdo_frame + lavish_rdo_reconstruct for fixed
// buffers recorded once into a HIP graph, replayed with one launch.  For
// callers that run the step on many small rectangles (the C5 row wavefront's
// chunks), where ~15 kernel launches and the fan-out events per call cost
// more host time than the rectangle's GPU work.  The graph owns the
// reconstruction's job scratch, so replays on any stream are independent of
// the per-thread scratch; two replays of one graph must not overlap.
// ---------------------------------------------------------------------------
struct LavishRdoGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  void* scratch = nullptr;
  lavish::FanSet* fan = nullptr;  // the capture's own fork / join set (freed once instantiated)
};

extern "C" int lavish_rdo_graph_create(const uint16_t* src, const uint16_t* pred, int stride,
                                       int width, int height, uint32_t size_mask,
                                       const uint32_t* type_masks, int bit_depth,
                                       const LavishQuantParams* qp, int rdmult,
                                       LavishRdoBlock* const* records, int32_t* const* qcoeff,
                                       int32_t* const* dqcoeff, uint16_t* recon,
                                       uint8_t* sb_tx_size, void* stream,
                                       LavishRdoGraph** out) {
  if (out == nullptr) return -3;
  *out = nullptr;
  size_t bytes = 0;
  int rc = lavish::rdo_reconstruct_impl(size_mask, (const LavishRdoBlock* const*)records,
                                        (const int32_t* const*)dqcoeff, width, height, pred,
                                        recon, stride, bit_depth, sb_tx_size, nullptr, nullptr,
                                        &bytes);
  if (rc) return rc;
  LavishRdoGraph* g = new LavishRdoGraph();
  LAVISH_CHECK(hipMalloc(&g->scratch, bytes > 0 ? bytes : 16));
  // the warm-up and the capture fork / join over a private stream + event
  // set: with the shared per-thread set, graphs captured after an uncaptured
  // whole-4K-frame step on the same thread crashed the host inside
  // hipGraphLaunch (round 5, tools/repro_c5test.py; not with the private set)
  g->fan = lavish::fan_create();
  lavish::fan_use(g->fan);
  hipStream_t cs;
  LAVISH_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  // the warm-up below reads src / pred and writes every output buffer: order
  // it after the caller's pending work on them (e.g. a fill of the
  // reconstruction plane still queued on the caller's stream)
  hipEvent_t after;
  LAVISH_CHECK(hipEventCreateWithFlags(&after, hipEventDisableTiming));
  LAVISH_CHECK(hipEventRecord(after, (hipStream_t)stream));
  LAVISH_CHECK(hipStreamWaitEvent(cs, after, 0));
  LAVISH_CHECK(hipEventDestroy(after));
  // one uncaptured run first: the library's lazily created state (internal
  // streams, device scan tables: synchronous uploads) must exist before the
  // capture, which may only record stream work
  rc = lavish::rdo_frame(src, pred, stride, width, height, size_mask, type_masks, bit_depth, qp,
                         rdmult, records, qcoeff, dqcoeff, cs);
  if (rc == 0)
    rc = lavish::rdo_reconstruct_impl(size_mask, (const LavishRdoBlock* const*)records,
                                      (const int32_t* const*)dqcoeff, width, height, pred, recon,
                                      stride, bit_depth, sb_tx_size, cs, (char*)g->scratch,
                                      &bytes);
  LAVISH_CHECK(hipStreamSynchronize(cs));
  if (rc != 0) {
    lavish::fan_use(nullptr);
    LAVISH_CHECK(hipStreamDestroy(cs));
    lavish_rdo_graph_destroy(g);
    return rc;
  }
  LAVISH_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
  rc = lavish::rdo_frame(src, pred, stride, width, height, size_mask, type_masks, bit_depth, qp,
                         rdmult, records, qcoeff, dqcoeff, cs);
  if (rc == 0)
    rc = lavish::rdo_reconstruct_impl(size_mask, (const LavishRdoBlock* const*)records,
                                      (const int32_t* const*)dqcoeff, width, height, pred, recon,
                                      stride, bit_depth, sb_tx_size, cs, (char*)g->scratch,
                                      &bytes);
  hipGraph_t graph = nullptr;
  LAVISH_CHECK(hipStreamEndCapture(cs, &graph));
  lavish::fan_use(nullptr);
  LAVISH_CHECK(hipStreamDestroy(cs));
  g->graph = graph;
  if (rc == 0 && graph != nullptr)
    LAVISH_CHECK(hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0));
  // the fork / join set served the warm-up and the capture only: the
  // instantiated graph's branches run on the runtime's own streams, so the
  // set goes now instead of holding 2 streams + 3 events per graph for the
  // graph's lifetime (every replay test runs after this release)
  lavish::fan_destroy(g->fan);
  g->fan = nullptr;
  if (rc != 0 || g->exec == nullptr) {
    lavish_rdo_graph_destroy(g);
    return rc ? rc : -8;
  }
  *out = g;
  return 0;
}

extern "C" int lavish_rdo_graph_launch(LavishRdoGraph* g, void* stream) {
  if (g == nullptr || g->exec == nullptr) return -3;
  LAVISH_CHECK(hipGraphLaunch(g->exec, (hipStream_t)stream));
  return 0;
}

extern "C" void lavish_rdo_graph_destroy(LavishRdoGraph* g) {
  if (g == nullptr) return;
  if (g->exec) LAVISH_CHECK(hipGraphExecDestroy(g->exec));
  if (g->graph) LAVISH_CHECK(hipGraphDestroy(g->graph));
  if (g->scratch) LAVISH_CHECK(hipFree(g->scratch));
  lavish::fan_destroy(g->fan);
  delete g;
}
