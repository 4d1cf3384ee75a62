// txq.hip -- batched forward transform + quantization for gfx950.
//
// The reference evaluates, per TX block and per candidate TX type, av1_xform
// (av1/encoder/encodemb.c:295 -> hybrid_fwd_txfm.c:233-313 ->
// av1_fwd_txfm2d.c:56-127) followed by av1_quant (encodemb.c:308 ->
// av1_quantize.c:36-122 / aom_dsp/quantize.c:108-169), one block at a time
// on one CPU thread.  Here one 256-thread workgroup owns P = 256/min(W,H)
// blocks of one TX size and walks every requested TX type over them:
//
//   residual (HBM, read once) -> registers (one column per thread)
//   per type: column 1-D transform (registers) -> LDS t1 (padded rows)
//             row 1-D transform + fp/b quantizer + eob reduction
//                                               -> LDS t2 (coefficient order)
//             coalesced 16-byte copy-out of qcoeff, dqcoeff (recomputed from
//             qcoeff: dq = sign * ((|q| * dequant) >> log_scale))
//
// The transforms are fully unrolled straight-line integer code (txfm_dev.h);
// no MFMA: AV1 butterflies with per-stage 64-bit rounding are not a matrix
// product.  HBM traffic is the residual once plus 8 bytes per output
// coefficient per type, so the kernel is bounded by the output write stream.
#include <atomic>

#include "txq_dev.h"

namespace lavish {

// runtime-kind wrapper for the generic per-block quantizer kernel
template <int LS>
__device__ __forceinline__ int32_t quant_rt(int32_t c, bool ac, int kind, int highbd,
                                            const QP& qp) {
  if (kind == LAVISH_QUANT_FP)
    return highbd ? quant_one<LS, LAVISH_QUANT_FP, true>(c, ac, qp)
                  : quant_one<LS, LAVISH_QUANT_FP, false>(c, ac, qp);
  return highbd ? quant_one<LS, LAVISH_QUANT_B, true>(c, ac, qp)
                : quant_one<LS, LAVISH_QUANT_B, false>(c, ac, qp);
}

constexpr int kFrameStreams = 3;  // the caller + 2 internal streams
constexpr int kFanDefault = 3;

template <int W, int H>
__global__ __launch_bounds__(256, 2) void txq_plane_kernel(TxqArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[TxqLds<W, H>::kBytes];
  txq_plane_body<W, H>(a, blockIdx.x, lds);
}

template <int CLS>
__global__ __launch_bounds__(256, 2) void txq_multi_kernel(TxqDispatch d, TxqArgs a0, TxqArgs a1,
                                                           TxqArgs a2, TxqArgs a3, TxqArgs a4,
                                                           TxqArgs a5, TxqArgs a6, TxqArgs a7,
                                                           TxqArgs a8) {
  __shared__ __attribute__((aligned(16))) char lds[class_lds(CLS)];
  txq_multi_body<CLS>(d, a0, a1, a2, a3, a4, a5, a6, a7, a8, blockIdx.x, lds);
}

// generic quantizer: one workgroup per block, any scan order.
template <int LS>
__global__ __launch_bounds__(256) void quant_kernel(const int32_t* coeff, int n,
                                                     const int16_t* scan, int kind,
                                                     int highbd, QP qp,
                                                     int32_t* qcoeff, int32_t* dqcoeff,
                                                     uint16_t* eob) {
  __shared__ int red[4];
  const size_t base = (size_t)blockIdx.x * n;
  const int tid = threadIdx.x;
  int last = 0;
  for (int i = tid; i < n; i += 256) {
    const int rc = scan[i];
    const int32_t q = quant_rt<LS>(coeff[base + rc], rc != 0, kind, highbd, qp);
    qcoeff[base + rc] = q;
    dqcoeff[base + rc] = dequant_one<LS>(q, rc != 0, qp);
    if (q != 0) last = max(last, i + 1);
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) last = max(last, __shfl_xor(last, m));
  if ((tid & 63) == 0) red[tid >> 6] = last;
  __syncthreads();
  if (tid == 0) eob[blockIdx.x] = (uint16_t)max(max(red[0], red[1]), max(red[2], red[3]));
}

// ----------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------
// Type chunks: one per vertical 1-D kind present (DCT, ADST, FLIPADST,
// IDTX; the 16 types are all 4 x 4 (vertical, horizontal) pairs, so a block
// needs 4 column passes, not 16), split further -- largest first -- until the
// grid has enough workgroups to give every CU several (>= ~8 per CU over 256
// CUs).  Each extra chunk re-reads the residual tile (2 bytes/pixel against
// 8 bytes/coefficient/type written) and repeats one column pass.
static void build_chunks(TxqArgs& a, int nbg) {
  int cnt = 0, sz[16] = {}, ti[16][16];
  for (int vk = 0; vk < 4; ++vk) {
    int n = 0;
    for (int i = 0; i < a.ntypes; ++i)
      if (((kVtxPacked >> (2 * a.types[i])) & 3) == (uint32_t)vk) ti[cnt][n++] = i;
    if (n) sz[cnt++] = n;
  }
  while (nbg * cnt < 2048 && cnt < 16) {
    int big = 0;
    for (int g = 1; g < cnt; ++g)
      if (sz[g] > sz[big]) big = g;
    if (sz[big] < 2) break;
    const int keep = (sz[big] + 1) / 2;
    for (int i = keep; i < sz[big]; ++i) ti[cnt][i - keep] = ti[big][i];
    sz[cnt++] = sz[big] - keep;
    sz[big] = keep;
  }
  int o = 0;
  for (int g = 0; g < cnt; ++g) {
    a.chunk_off[g] = o;
    for (int i = 0; i < sz[g]; ++i) a.chunk_ti[o++] = ti[g][i];
  }
  a.chunk_off[cnt] = o;
  a.tgroups = cnt;
}

// the grid of one size (0: nothing to do); fills the type chunks of `a`
template <int W, int H>
static int plan_plane(TxqArgs& a) {
  constexpr int P = Tile<W, H>::P * 4;  // blocks per workgroup (4 wave tiles)
  const int nbg = (a.nblocks + P - 1) / P;
  if (nbg == 0) return 0;
  build_chunks(a, nbg);
  return ((nbg + 7) / 8) * 8 * a.tgroups;
}

template <int W, int H>
static void launch_plane(TxqArgs a, hipStream_t s) {
  const int grid = plan_plane<W, H>(a);
  if (grid == 0) return;
  hipLaunchKernelGGL((txq_plane_kernel<W, H>), dim3(grid), dim3(256), 0, s, a);
  LAVISH_CHECK(hipGetLastError());
}

static int plan_size(int tx_size, TxqArgs& a) {
  switch (tx_size) {
    case 0: return plan_plane<4, 4>(a);
    case 1: return plan_plane<8, 8>(a);
    case 2: return plan_plane<16, 16>(a);
    case 3: return plan_plane<32, 32>(a);
    case 5: return plan_plane<4, 8>(a);
    case 6: return plan_plane<8, 4>(a);
    case 7: return plan_plane<8, 16>(a);
    case 8: return plan_plane<16, 8>(a);
    case 9: return plan_plane<16, 32>(a);
    case 10: return plan_plane<32, 16>(a);
    case 13: return plan_plane<4, 16>(a);
    case 14: return plan_plane<16, 4>(a);
    case 15: return plan_plane<8, 32>(a);
    case 16: return plan_plane<32, 8>(a);
    default: return -1;
  }
}

static QP to_qp(const LavishQuantParams* p) {
  QP q{};
  if (p) {
    for (int i = 0; i < 2; ++i) {
      q.zbin[i] = p->zbin[i];
      q.round[i] = p->round[i];
      q.quant[i] = p->quant[i];
      q.quant_shift[i] = p->quant_shift[i];
      q.dequant[i] = p->dequant[i];
    }
  }
  return q;
}

int txq_args(const int16_t* residual, int stride, int width, int height, int tx_size,
             uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
             int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff, TxqArgs& a);

int txq_plane(const int16_t* residual, int stride, int width, int height, int tx_size,
              uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
              int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff,
              hipStream_t s) {
  if (tx_size < 0 || tx_size >= 19) return -1;
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  if (quant_kind < 0 || quant_kind > 2) return -3;
  if (quant_kind != LAVISH_QUANT_NONE && qp == nullptr) return -3;
  if (width <= 0 || height <= 0 || stride < width) return -4;
  if (W > 32 || H > 32)  // 64-point sizes: rdo.hip, mode 0
    return txq_plane_64(residual, stride, width, height, tx_size, type_mask, bd, quant_kind, qp,
                        qcoeff, dqcoeff, eob, coeff, s);
  TxqArgs a{};
  const int rc = txq_args(residual, stride, width, height, tx_size, type_mask, bd, quant_kind,
                          qp, qcoeff, dqcoeff, eob, coeff, a);
  if (rc) return rc;
  switch (tx_size) {
    case 0: launch_plane<4, 4>(a, s); break;
    case 1: launch_plane<8, 8>(a, s); break;
    case 2: launch_plane<16, 16>(a, s); break;
    case 3: launch_plane<32, 32>(a, s); break;
    case 5: launch_plane<4, 8>(a, s); break;
    case 6: launch_plane<8, 4>(a, s); break;
    case 7: launch_plane<8, 16>(a, s); break;
    case 8: launch_plane<16, 8>(a, s); break;
    case 9: launch_plane<16, 32>(a, s); break;
    case 10: launch_plane<32, 16>(a, s); break;
    case 13: launch_plane<4, 16>(a, s); break;
    case 14: launch_plane<16, 4>(a, s); break;
    case 15: launch_plane<8, 32>(a, s); break;
    case 16: launch_plane<32, 8>(a, s); break;
    default: return -2;
  }
  return 0;
}

// TxqArgs of one (size <= 32 points, plane) job; 0 or the API's error code
int txq_args(const int16_t* residual, int stride, int width, int height, int tx_size,
             uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
             int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff, TxqArgs& a) {
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  a = TxqArgs{};
  a.res = residual;
  a.stride = stride;
  a.bw = width / W;
  a.nblocks = (width / W) * (height / H);
  for (int t = 0; t < 16; ++t) {
    if (!((type_mask >> t) & 1)) continue;
    if (!tx_type_valid(tx_size, t)) return -5;
    a.types[a.ntypes++] = t;
  }
  if (a.ntypes == 0) return -5;
  a.quant_kind = quant_kind;
  a.highbd = bd > 8;
  a.qp = to_qp(qp);
  a.iscan_default = dev_iscan(tx_size, 0);
  a.qcoeff = qcoeff;
  a.dqcoeff = dqcoeff;
  a.eob = eob;
  a.coeff = coeff;
  return 0;
}

int quantize_batch(const int32_t* coeff, int n, int nblocks, const int16_t* scan,
                   int log_scale, int bd, int quant_kind, const LavishQuantParams* qp,
                   int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, hipStream_t s) {
  if (n <= 0 || nblocks <= 0 || qp == nullptr) return -1;
  if (quant_kind != LAVISH_QUANT_FP && quant_kind != LAVISH_QUANT_B) return -3;
  const QP q = to_qp(qp);
  const int hb = bd > 8;
  switch (log_scale) {
    case 0:
      hipLaunchKernelGGL(quant_kernel<0>, dim3(nblocks), dim3(256), 0, s, coeff, n, scan,
                         quant_kind, hb, q, qcoeff, dqcoeff, eob);
      break;
    case 1:
      hipLaunchKernelGGL(quant_kernel<1>, dim3(nblocks), dim3(256), 0, s, coeff, n, scan,
                         quant_kind, hb, q, qcoeff, dqcoeff, eob);
      break;
    case 2:
      hipLaunchKernelGGL(quant_kernel<2>, dim3(nblocks), dim3(256), 0, s, coeff, n, scan,
                         quant_kind, hb, q, qcoeff, dqcoeff, eob);
      break;
    default:
      return -2;
  }
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

// Frame batch: every requested TX size over the same residual plane.  The
// per-size kernels are independent, so they are spread over the caller's
// stream plus two internal streams (forked from / joined back to the caller
// with events): register-heavy 16/32-point kernels and light 4/8-point
// kernels then share the CUs, which a single in-order stream cannot do.  The
// caller's stream takes every third kernel (the largest first) so it never
// waits on a fork; a cross-stream event wait costs tens of microseconds.
struct FrameStreams {
  int device = -1;
  hipStream_t s[kFrameStreams] = {};  // s[0] = the caller's stream (set per call)
  hipEvent_t fork = nullptr, join[kFrameStreams] = {};
};
static thread_local FrameStreams t_fs;
struct FanSet {
  FrameStreams fs;
};
static thread_local FanSet* t_fan_own = nullptr;  // fan_use: a private set

static void frame_streams_init(FrameStreams& f, int dev) {
  for (int i = 1; i < kFrameStreams; ++i) {
    LAVISH_CHECK(hipStreamCreateWithFlags(&f.s[i], hipStreamNonBlocking));
    LAVISH_CHECK(hipEventCreateWithFlags(&f.join[i], hipEventDisableTiming));
  }
  LAVISH_CHECK(hipEventCreateWithFlags(&f.fork, hipEventDisableTiming));
  f.device = dev;
}

static FrameStreams& frame_streams() {
  if (t_fan_own != nullptr) return t_fan_own->fs;
  int dev = 0;
  LAVISH_CHECK(hipGetDevice(&dev));
  if (t_fs.device != dev) frame_streams_init(t_fs, dev);
  return t_fs;
}

FanSet* fan_create() {
  int dev = 0;
  LAVISH_CHECK(hipGetDevice(&dev));
  FanSet* f = new FanSet();
  frame_streams_init(f->fs, dev);
  return f;
}

void fan_destroy(FanSet* f) {
  if (f == nullptr) return;
  if (t_fan_own == f) t_fan_own = nullptr;
  for (int i = 1; i < kFrameStreams; ++i) {
    LAVISH_CHECK(hipStreamDestroy(f->fs.s[i]));
    LAVISH_CHECK(hipEventDestroy(f->fs.join[i]));
  }
  LAVISH_CHECK(hipEventDestroy(f->fs.fork));
  delete f;
}

void fan_use(FanSet* f) { t_fan_own = f; }

// streams the per-size work of lavish_rdo_frame / lavish_rdo_reconstruct is
// dealt over: the caller + fan_width() - 1 internal streams (default 3; 1:
// every size on the caller's stream, isolated per-kernel timings under a
// profiler), set by lavish_set_fan_width.  (Wider fans, up to 6 streams,
// measured slower on the C5 tiles: 0.19 vs 0.178 ms per rank at G = 8.)
static std::atomic<int> g_fan_width{kFanDefault};
int fan_width() { return g_fan_width.load(std::memory_order_relaxed); }
int set_fan_width(int w) {
  if (w < 1 || w > kFrameStreams) return -1;
  g_fan_width.store(w, std::memory_order_relaxed);
  return 0;
}

// fork: the internal streams wait for everything queued on `caller`; slot 0
// is the caller itself
hipStream_t* fan_out(hipStream_t caller) {
  FrameStreams& fs = frame_streams();
  fs.s[0] = caller;
  LAVISH_CHECK(hipEventRecord(fs.fork, caller));
  for (int i = 1; i < kFrameStreams; ++i) LAVISH_CHECK(hipStreamWaitEvent(fs.s[i], fs.fork, 0));
  return fs.s;
}

// join: `caller` waits for everything queued on the internal streams
void fan_in(hipStream_t caller) {
  FrameStreams& fs = frame_streams();
  for (int i = 1; i < kFrameStreams; ++i) {
    LAVISH_CHECK(hipEventRecord(fs.join[i], fs.s[i]));
    LAVISH_CHECK(hipStreamWaitEvent(caller, fs.join[i], 0));
  }
}

// the sizes of one class in one launch's dispatch table (heaviest first)
int txq_frame_plan(const int16_t* residual, int stride, int width, int height, uint32_t size_mask,
                   const uint32_t* type_masks, int bd, int quant_kind, const LavishQuantParams* qp,
                   int32_t* const* qcoeff, int32_t* const* dqcoeff, uint16_t* const* eob, int cls,
                   TxqMulti& m, int& grid) {
  int order[19], n = 0;
  for (int s = 0; s < 19; ++s)
    if (((size_mask >> s) & 1) && tx_w(s) <= 32 && tx_h(s) <= 32 && (txq_class(s) ? 1 : 0) == cls)
      order[n++] = s;
  auto work = [&](int s) {
    return (long)__builtin_popcount(type_masks[s]) * max_eob(s) * (width / tx_w(s)) *
           (height / tx_h(s));
  };
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && work(order[j]) > work(order[j - 1]); --j) {
      const int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  m = TxqMulti{};
  int g = 0;
  for (int i = 0; i < n; ++i) {
    const int s = order[i];
    if (m.d.n == kMultiMax) return -2;
    TxqArgs& a = m.a[txq_slot(s)];
    const int rc = txq_args(residual, stride, width, height, s, type_masks[s], bd, quant_kind, qp,
                            qcoeff[s], dqcoeff[s], eob[s], nullptr, a);
    if (rc) return rc;
    const int sg = plan_size(s, a);
    if (sg <= 0) continue;
    m.d.code[m.d.n] = s;
    m.d.wg0[m.d.n] = g;
    g += sg;
    ++m.d.n;
  }
  m.d.wg0[m.d.n] = g;
  grid = g;
  return 0;
}

int txq_frame(const int16_t* residual, int stride, int width, int height, uint32_t size_mask,
              const uint32_t* type_masks, int bd, int quant_kind, const LavishQuantParams* qp,
              int32_t* const* qcoeff, int32_t* const* dqcoeff, uint16_t* const* eob,
              hipStream_t caller) {
  // 64-point sizes: their own path, first
  for (int s = 0; s < 19; ++s) {
    if (!((size_mask >> s) & 1) || (tx_w(s) <= 32 && tx_h(s) <= 32)) continue;
    const int rc = txq_plane(residual, stride, width, height, s, type_masks[s], bd, quant_kind,
                             qp, qcoeff[s], dqcoeff[s], eob[s], nullptr, caller);
    if (rc) return rc;
  }
  // one launch per class, on the caller's stream: the 32-point class (few,
  // register-heavy workgroups) first, then the <= 16-point class.  (Measured
  // and dropped: the round-2 per-size kernels over the caller + 2 internal
  // streams, ~50 us of fork / join per frame; the 32-point class on an
  // internal stream beside the other, C2 0.565 -> 0.577 ms,
  // profiles/r04_v5_c2_streams_ab.txt; an LDS pad so fewer C2 workgroups fit
  // a CU beside a concurrent leg -- C2 alone 0.51 -> 0.55 / 1.31 ms at 3 / 2
  // workgroups per CU, profiles/r04_v11_ab_notes.txt.)
  for (int cls = 1; cls >= 0; --cls) {
    TxqMulti m;
    int g = 0;
    const int rc = txq_frame_plan(residual, stride, width, height, size_mask, type_masks, bd,
                                  quant_kind, qp, qcoeff, dqcoeff, eob, cls, m, g);
    if (rc) return rc;
    if (g == 0) continue;
    if (cls == 0)
      hipLaunchKernelGGL(txq_multi_kernel<0>, dim3(g), dim3(256), 0, caller, m.d, m.a[0], m.a[1],
                         m.a[2], m.a[3], m.a[4], m.a[5], m.a[6], m.a[7], m.a[8]);
    else
      hipLaunchKernelGGL(txq_multi_kernel<1>, dim3(g), dim3(256), 0, caller, m.d, m.a[0], m.a[1],
                         m.a[2], m.a[3], m.a[4], m.a[5], m.a[6], m.a[7], m.a[8]);
    LAVISH_CHECK(hipGetLastError());
  }
  return 0;
}

}  // namespace lavish

extern "C" int lavish_set_fan_width(int streams) { return lavish::set_fan_width(streams); }

extern "C" int lavish_txq_frame(const int16_t* residual, int stride, int width, int height,
                                uint32_t size_mask, const uint32_t* type_masks, int bit_depth,
                                int quant_kind, const LavishQuantParams* qp,
                                int32_t* const* qcoeff, int32_t* const* dqcoeff,
                                uint16_t* const* eob, void* stream) {
  return lavish::txq_frame(residual, stride, width, height, size_mask, type_masks, bit_depth,
                           quant_kind, qp, qcoeff, dqcoeff, eob, (hipStream_t)stream);
}

extern "C" int lavish_txq_plane(const int16_t* residual, int stride, int width, int height,
                                int tx_size, uint32_t type_mask, int bit_depth,
                                int quant_kind, const LavishQuantParams* qp,
                                int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob,
                                int32_t* coeff, void* stream) {
  return lavish::txq_plane(residual, stride, width, height, tx_size, type_mask, bit_depth,
                           quant_kind, qp, qcoeff, dqcoeff, eob, coeff,
                           (hipStream_t)stream);
}

extern "C" int lavish_quantize_batch(const int32_t* coeff, int n, int nblocks,
                                     const int16_t* scan, const int16_t* iscan,
                                     int log_scale, int bit_depth, int quant_kind,
                                     const LavishQuantParams* qp, int32_t* qcoeff,
                                     int32_t* dqcoeff, uint16_t* eob, void* stream) {
  (void)iscan;  // the reference quantizers walk `scan` only
  return lavish::quantize_batch(coeff, n, nblocks, scan, log_scale, bit_depth, quant_kind,
                                qp, qcoeff, dqcoeff, eob, (hipStream_t)stream);
}
