// capi.hip -- host side of liblavish_hip.so: library state, quantizer and
// scan tables, and the per-call RTCD shims that stage the reference's host
// buffers through a per-thread device scratch.
#include <mutex>
#include <string.h>
#include <vector>

#include "lavish_internal.h"
#include "qlookup_tables.h"

namespace lavish {

int txq_plane(const int16_t*, int, int, int, int, uint32_t, int, int, const LavishQuantParams*,
              int32_t*, int32_t*, uint16_t*, int32_t*, hipStream_t);
int quantize_batch(const int32_t*, int, int, const int16_t*, int, int, int,
                   const LavishQuantParams*, int32_t*, int32_t*, uint16_t*, hipStream_t);

// ---------------------------------------------------------------- status --
static int g_status = 0;
static char g_status_str[512] = "ok";
static int g_abort_on_error = 1;
static std::mutex g_mu;

void set_error(const char* what, hipError_t e, const char* file, int line) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_status == 0) {
      g_status = (int)e;
      snprintf(g_status_str, sizeof(g_status_str), "%s failed: %s (%d) at %s:%d", what,
               hipGetErrorString(e), (int)e, file, line);
    }
  }
  fprintf(stderr, "[lavish_hip] %s failed: %s (%d) at %s:%d\n", what, hipGetErrorString(e),
          (int)e, file, line);
  if (g_abort_on_error) abort();
}

// ------------------------------------------------------------ tx tables --
static const int kW[19] = {4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64};
static const int kH[19] = {4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16};

int tx_w(int s) { return kW[s]; }
int tx_h(int s) { return kH[s]; }
int max_eob(int s) {  // av1_get_max_eob, av1/common/blockd.h:1596-1604
  if (s == 17 || s == 18) return 512;
  if (kW[s] == 64 || kH[s] == 64) return 1024;
  return kW[s] * kH[s];
}
int tx_scale(int s) {  // av1_get_tx_scale, av1/common/idct.c:24-28
  const int p = kW[s] * kH[s];
  return (p > 256) + (p > 1024);
}
bool tx_type_valid(int s, int t) {  // EXT_TX_SET_{DCTONLY,DCT_IDTX,ALL16}
  const int m = kW[s] > kH[s] ? kW[s] : kH[s];
  if (t < 0 || t > 15) return false;
  if (m == 64) return t == 0;
  if (m == 32) return t == 0 || t == 9;
  return true;
}
int scan_kind(int t) { return t < 10 ? 0 : ((t & 1) ? 1 : 2); }

// ----------------------------------------------------------------- scans --
// Scan orders of av1/common/scan.c, generated: the coefficient buffer is
// column-major (rc = col*H + row); mcol = identity, mrow walks rows, default
// walks anti-diagonals (square: zig-zag, tall: high->low column, wide:
// low->high column); 64-point sizes use the 32-point scan of the kept
// quadrant.  tests/test_capi_cpu.py compares all 19x16 orders with the tables
// parsed from the reference.
struct ScanSet {
  std::vector<int16_t> scan[3], iscan[3];
  const int16_t* dscan[3] = {nullptr, nullptr, nullptr};
  const int16_t* discan[3] = {nullptr, nullptr, nullptr};
  const int16_t* discan_rows = nullptr;
};
static ScanSet g_scans[19];
static std::once_flag g_scan_once;

static void gen_scan(int W, int H, int kind, std::vector<int16_t>& s) {
  s.resize(W * H);
  int k = 0;
  if (kind == 1) {
    for (int i = 0; i < W * H; ++i) s[i] = (int16_t)i;
    return;
  }
  if (kind == 2) {
    for (int i = 0; i < W * H; ++i) s[i] = (int16_t)((i % W) * H + i / W);
    return;
  }
  for (int d = 0; d < W + H - 1; ++d) {
    const bool down = (W == H) ? (d & 1) : (W < H);
    const int cmin = d - (H - 1) > 0 ? d - (H - 1) : 0;
    const int cmax = d < W - 1 ? d : W - 1;
    if (down)
      for (int c = cmax; c >= cmin; --c) s[k++] = (int16_t)(c * H + (d - c));
    else
      for (int c = cmin; c <= cmax; ++c) s[k++] = (int16_t)(c * H + (d - c));
  }
}

static void init_scans() {
  std::call_once(g_scan_once, [] {
    for (int s = 0; s < 19; ++s) {
      const int W = kW[s] > 32 ? 32 : kW[s], H = kH[s] > 32 ? 32 : kH[s];
      for (int kind = 0; kind < 3; ++kind) {
        gen_scan(W, H, kind, g_scans[s].scan[kind]);
        g_scans[s].iscan[kind].resize(W * H);
        for (int i = 0; i < W * H; ++i) g_scans[s].iscan[kind][g_scans[s].scan[kind][i]] = (int16_t)i;
      }
    }
  });
}

const int16_t* host_scan(int s, int t) {
  init_scans();
  return g_scans[s].scan[scan_kind(t)].data();
}
const int16_t* host_iscan(int s, int t) {
  init_scans();
  return g_scans[s].iscan[scan_kind(t)].data();
}

static const int16_t* upload(const std::vector<int16_t>& v) {
  void* d = nullptr;
  LAVISH_CHECK(hipMalloc(&d, v.size() * sizeof(int16_t)));
  LAVISH_CHECK(hipMemcpy(d, v.data(), v.size() * sizeof(int16_t), hipMemcpyHostToDevice));
  return (const int16_t*)d;
}

// Device tables are uploaded once per process for the current device.  The
// library is used one device per process (one rank per GPU).
const int16_t* dev_iscan(int s, int t) {
  init_scans();
  std::lock_guard<std::mutex> lk(g_mu);
  const int k = scan_kind(t);
  if (!g_scans[s].discan[k]) g_scans[s].discan[k] = upload(g_scans[s].iscan[k]);
  return g_scans[s].discan[k];
}
// The three scan kinds' inverse scans of size s in lane-row order,
// [kind][r][c] = iscan[kind][c * KH + r] (KW, KH = the kept dimensions, <= 32):
// the rdo kernels' lane owning kept row r reads its KW positions as one
// contiguous run (staged into LDS per workgroup).
const int16_t* dev_iscan_rows(int s) {
  init_scans();
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_scans[s].discan_rows) {
    const int KW = kW[s] > 32 ? 32 : kW[s], KH = kH[s] > 32 ? 32 : kH[s];
    std::vector<int16_t> v((size_t)3 * KW * KH);
    for (int k = 0; k < 3; ++k)
      for (int r = 0; r < KH; ++r)
        for (int c = 0; c < KW; ++c)
          v[((size_t)k * KH + r) * KW + c] = g_scans[s].iscan[k][c * KH + r];
    g_scans[s].discan_rows = upload(v);
  }
  return g_scans[s].discan_rows;
}

const int16_t* dev_scan(int s, int t) {
  init_scans();
  std::lock_guard<std::mutex> lk(g_mu);
  const int k = scan_kind(t);
  if (!g_scans[s].dscan[k]) g_scans[s].dscan[k] = upload(g_scans[s].scan[k]);
  return g_scans[s].dscan[k];
}

// ------------------------------------------------------- shim scratch --
struct Scratch {
  void* ptr = nullptr;
  size_t cap = 0;
  hipStream_t stream = nullptr;
  ~Scratch() {
    // process teardown: the runtime may already be gone; leak deliberately
  }
};
static thread_local Scratch t_scratch;

hipStream_t shim_stream() {
  if (!t_scratch.stream) LAVISH_CHECK(hipStreamCreateWithFlags(&t_scratch.stream, hipStreamNonBlocking));
  return t_scratch.stream;
}

void* shim_scratch(size_t bytes) {
  if (bytes > t_scratch.cap) {
    if (t_scratch.ptr) LAVISH_CHECK(hipFree(t_scratch.ptr));
    size_t cap = 1 << 20;
    while (cap < bytes) cap <<= 1;
    LAVISH_CHECK(hipMalloc(&t_scratch.ptr, cap));
    t_scratch.cap = cap;
  }
  return t_scratch.ptr;
}

void shim_reject(const char* what, int rc) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_status == 0) {
      g_status = rc < 0 ? rc : -rc;
      snprintf(g_status_str, sizeof(g_status_str), "%s rejected its arguments (rc %d)", what, rc);
    }
  }
  fprintf(stderr, "[lavish_hip] %s rejected its arguments (rc %d)\n", what, rc);
  if (g_abort_on_error) abort();
}

void* StreamScratch::acquire(size_t bytes, hipStream_t s) {
  int dev = 0;
  LAVISH_CHECK(hipGetDevice(&dev));
  if (device != dev) {  // a device switch frees the old device's buffer and starts afresh
    if (device >= 0) {
      LAVISH_CHECK(hipSetDevice(device));
      if (pending) LAVISH_CHECK(hipEventSynchronize(done));
      if (ptr) LAVISH_CHECK(hipFree(ptr));
      LAVISH_CHECK(hipEventDestroy(done));
      LAVISH_CHECK(hipSetDevice(dev));
    }
    ptr = nullptr;
    cap = 0;
    pending = false;
    LAVISH_CHECK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    device = dev;
  }
  if (bytes > cap) {
    if (ptr) {
      if (pending) LAVISH_CHECK(hipEventSynchronize(done));
      LAVISH_CHECK(hipFree(ptr));
    }
    size_t c = (size_t)1 << 16;
    while (c < bytes) c <<= 1;
    LAVISH_CHECK(hipMalloc(&ptr, c));
    cap = c;
    pending = false;
  } else if (pending) {
    LAVISH_CHECK(hipStreamWaitEvent(s, done, 0));
  }
  return ptr;
}

void StreamScratch::release(hipStream_t s) {
  LAVISH_CHECK(hipEventRecord(done, s));
  pending = true;
}

// ------------------------------------------------------------ quantizer --
static int16_t dc_q(int q, int delta, int bd) {
  int i = q + delta;
  i = i < 0 ? 0 : (i > 255 ? 255 : i);
  return bd == 8 ? kDcQ8[i] : (bd == 10 ? kDcQ10[i] : kDcQ12[i]);
}
static int16_t ac_q(int q, int delta, int bd) {
  int i = q + delta;
  i = i < 0 ? 0 : (i > 255 ? 255 : i);
  return bd == 8 ? kAcQ8[i] : (bd == 10 ? kAcQ10[i] : kAcQ12[i]);
}

// invert_quant (av1/encoder/av1_quantize.c:580-588)
static void invert_quant(int16_t* quant, int16_t* shift, int d) {
  uint32_t t = (uint32_t)d;
  int l = 0;
  for (; t > 1; ++l) t >>= 1;
  const int m = 1 + (1 << (16 + l)) / d;
  *quant = (int16_t)(m - (1 << 16));
  *shift = (int16_t)(1 << (16 - l));
}

}  // namespace lavish

using namespace lavish;

extern "C" {

int lavish_hip_status(void) { return g_status; }
const char* lavish_hip_status_string(void) { return g_status_str; }
void lavish_hip_set_abort_on_error(int on) { g_abort_on_error = on; }
int lavish_hip_version(void) { return 0x000100; }

int lavish_hip_init(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    set_error("hipGetDeviceCount", e == hipSuccess ? hipErrorNoDevice : e, __FILE__, __LINE__);
    return -1;
  }
  if (device >= 0) LAVISH_CHECK(hipSetDevice(device));
  return 0;
}

// av1_build_quantizer (av1/encoder/av1_quantize.c:590-686) for luma, one
// qindex, including the fork's quant_sharpness adjustment (:602-619).
int lavish_build_quant_params(int bd, int q, int sharpness, int y_dc_delta_q, int kind,
                              LavishQuantParams* out) {
  if (!out || (bd != 8 && bd != 10 && bd != 12) || q < 0 || q > 255) return -1;
  const int dc8 = dc_q(q, 0, bd);
  const int thr = bd == 8 ? 148 : (bd == 10 ? 592 : 2368);
  int zf = q == 0 ? 64 : (dc8 < thr ? 84 : 80);  // get_qzbin_factor
  int rf = q == 0 ? 64 : 48;
  int adj = 16 * (7 - sharpness) / 7;
  if (sharpness > 0 && q > 0) {
    zf = 64 + adj;
    rf = 64 - adj;
  } else if (sharpness < 0 && q > 0) {
    adj = 16 * (7 + sharpness) / 7;
    zf = 64 + adj;
    rf = 64 - adj;
  }
  const int rf_fp = sharpness != 0 ? 64 - adj : 64;
  for (int i = 0; i < 2; ++i) {
    const int qv = i == 0 ? dc_q(q, y_dc_delta_q, bd) : ac_q(q, 0, bd);
    invert_quant(&out->quant[i], &out->quant_shift[i], qv);
    out->zbin[i] = (int16_t)((zf * qv + 64) >> 7);
    out->dequant[i] = (int16_t)qv;
    if (kind == LAVISH_QUANT_FP) {
      out->quant[i] = (int16_t)((1 << 16) / qv);
      out->round[i] = (int16_t)((rf_fp * qv) >> 7);
    } else {
      out->round[i] = (int16_t)((rf * qv) >> 7);
    }
  }
  return 0;
}

const int16_t* lavish_scan(int tx_size, int tx_type) {
  if (tx_size < 0 || tx_size > 18 || tx_type < 0 || tx_type > 15) return nullptr;
  return host_scan(tx_size, tx_type);
}
const int16_t* lavish_iscan(int tx_size, int tx_type) {
  if (tx_size < 0 || tx_size > 18 || tx_type < 0 || tx_type > 15) return nullptr;
  return host_iscan(tx_size, tx_type);
}

// ------------------------------------------------------ per-call shims --
// Forward 2-D transform of one block (host pointers): stage the H x stride
// input, run the plane kernel on a single block with quantization off, copy
// the W*H coefficient words back.
static void fwd2d_shim(int tx_size, const int16_t* input, int32_t* output, int stride,
                       int tx_type) {
  const int W = tx_w(tx_size), H = tx_h(tx_size);
  if (tx_size < 0 || tx_size >= 19 || !tx_type_valid(tx_size, tx_type)) {
    shim_reject("av1_fwd_txfm2d (tx_size / tx_type)", -5);
    return;
  }
  hipStream_t s = shim_stream();
  const int n = max_eob(tx_size);
  const size_t in_bytes = (size_t)H * W * sizeof(int16_t);
  const size_t in_pad = (in_bytes + 255) & ~(size_t)255;
  char* scratch = (char*)shim_scratch(in_pad + (size_t)n * sizeof(int32_t));
  int16_t* din = (int16_t*)scratch;
  int32_t* dout = (int32_t*)(scratch + in_pad);
  // only the H x W window of the caller's rows is read
  LAVISH_CHECK(hipMemcpy2DAsync(din, (size_t)W * sizeof(int16_t), input,
                                (size_t)stride * sizeof(int16_t), (size_t)W * sizeof(int16_t), H,
                                hipMemcpyHostToDevice, s));
  const int rc = txq_plane(din, W, W, H, tx_size, 1u << tx_type, 8, LAVISH_QUANT_NONE, nullptr,
                           nullptr, nullptr, nullptr, dout, s);
  if (rc != 0) {
    shim_reject("txq_plane", rc);
    return;
  }
  LAVISH_CHECK(hipMemcpyAsync(output, dout, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost,
                              s));
  LAVISH_CHECK(hipStreamSynchronize(s));
  // 64-point sizes: the reference zeroes and re-packs in place
  // (av1_fwd_txfm2d.c:248-311), which leaves, past the n packed words, the
  // original copies of columns KW/2..KW-1 (rows < 32) of a 64-high buffer
  // and zeros everywhere else.
  for (int pos = n; pos < W * H; ++pos) {
    int32_t v = 0;
    if (H == 64) {
      const int c = pos / 64, r = pos % 64;
      if (c < (W < 32 ? W : 32) && r < 32) v = output[c * 32 + r];
    }
    output[pos] = v;
  }
}

#define FWD2D_SHIM(w, h, sz)                                                          \
  void av1_fwd_txfm2d_##w##x##h##_hip(const int16_t* input, int32_t* output, int stride, \
                                      uint8_t tx_type, int bd) {                      \
    (void)bd; /* feeds only the disabled range checks (av1_fwd_txfm2d.c:41-54) */     \
    fwd2d_shim(sz, input, output, stride, tx_type);                                   \
  }
FWD2D_SHIM(4, 4, 0)
FWD2D_SHIM(64, 64, 4)
FWD2D_SHIM(32, 64, 11)
FWD2D_SHIM(64, 32, 12)
FWD2D_SHIM(16, 64, 17)
FWD2D_SHIM(64, 16, 18)
FWD2D_SHIM(8, 8, 1)
FWD2D_SHIM(16, 16, 2)
FWD2D_SHIM(32, 32, 3)
FWD2D_SHIM(4, 8, 5)
FWD2D_SHIM(8, 4, 6)
FWD2D_SHIM(8, 16, 7)
FWD2D_SHIM(16, 8, 8)
FWD2D_SHIM(16, 32, 9)
FWD2D_SHIM(32, 16, 10)
FWD2D_SHIM(4, 16, 13)
FWD2D_SHIM(16, 4, 14)
FWD2D_SHIM(8, 32, 15)
FWD2D_SHIM(32, 8, 16)
#undef FWD2D_SHIM

// av1_lowbd_fwd_txfm_c -> av1_highbd_fwd_txfm (hybrid_fwd_txfm.c:244-313):
// only the 4x4 case looks at `lossless` (highbd_fwd_txfm_4x4, :77-88), where
// it takes the Walsh-Hadamard transform (wht.hip)
void av1_lowbd_fwd_txfm_hip(const int16_t* src_diff, int32_t* coeff, int diff_stride,
                            LavishTxfmParam* p) {
  if (p->lossless && p->tx_size == 0) {
    av1_fwht4x4_hip(src_diff, coeff, diff_stride);
    return;
  }
  fwd2d_shim(p->tx_size, src_diff, coeff, diff_stride, p->tx_type);
}

// av1_quick_txfm (hybrid_fwd_txfm.c:315-336): the TPL model's transform --
// aom_hadamard_{4x4..32x32} or the DCT_DCT forward transform
void av1_quick_txfm_hip(int use_hadamard, uint8_t tx_size, LavishBitDepthInfo bd_info,
                        const int16_t* src_diff, int src_stride, int32_t* coeff) {
  (void)bd_info;  // feeds only the forward transform's disabled range checks
  if (use_hadamard) {
    switch (tx_size) {
      case 0: aom_hadamard_4x4_hip(src_diff, src_stride, coeff); return;
      case 1: aom_hadamard_8x8_hip(src_diff, src_stride, coeff); return;
      case 2: aom_hadamard_16x16_hip(src_diff, src_stride, coeff); return;
      case 3: aom_hadamard_32x32_hip(src_diff, src_stride, coeff); return;
      default: shim_reject("av1_quick_txfm (hadamard size)", -2); return;
    }
  }
  fwd2d_shim(tx_size, src_diff, coeff, src_stride, 0);
}

// Quantizer shims: the reference passes pointers into its 8-wide QUANTS
// rows; only [0] (DC) and [1] (AC) are read.
static void quant_shim(const int32_t* coeff, intptr_t n, const int16_t* zbin,
                       const int16_t* round, const int16_t* quant, const int16_t* qshift,
                       int32_t* qcoeff, int32_t* dqcoeff, const int16_t* dequant,
                       uint16_t* eob, const int16_t* scan, int log_scale, int kind, int bd) {
  LavishQuantParams qp;
  for (int i = 0; i < 2; ++i) {
    qp.zbin[i] = zbin ? zbin[i] : 0;
    qp.round[i] = round[i];
    qp.quant[i] = quant[i];
    qp.quant_shift[i] = qshift ? qshift[i] : 0;
    qp.dequant[i] = dequant[i];
  }
  hipStream_t s = shim_stream();
  const size_t cb = (size_t)n * sizeof(int32_t);
  const size_t sb = ((size_t)n * sizeof(int16_t) + 255) & ~(size_t)255;
  char* base = (char*)shim_scratch(3 * cb + sb + 256);
  int32_t* dc = (int32_t*)base;
  int32_t* dq = (int32_t*)(base + cb);
  int32_t* ddq = (int32_t*)(base + 2 * cb);
  int16_t* dscan = (int16_t*)(base + 3 * cb);
  uint16_t* deob = (uint16_t*)(base + 3 * cb + sb);
  LAVISH_CHECK(hipMemcpyAsync(dc, coeff, cb, hipMemcpyHostToDevice, s));
  LAVISH_CHECK(hipMemcpyAsync(dscan, scan, (size_t)n * sizeof(int16_t), hipMemcpyHostToDevice, s));
  quantize_batch(dc, (int)n, 1, dscan, log_scale, bd, kind, &qp, dq, ddq, deob, s);
  LAVISH_CHECK(hipMemcpyAsync(qcoeff, dq, cb, hipMemcpyDeviceToHost, s));
  LAVISH_CHECK(hipMemcpyAsync(dqcoeff, ddq, cb, hipMemcpyDeviceToHost, s));
  LAVISH_CHECK(hipMemcpyAsync(eob, deob, sizeof(uint16_t), hipMemcpyDeviceToHost, s));
  LAVISH_CHECK(hipStreamSynchronize(s));
}

#define QUANT_SHIM(name, ls, kind, bd)                                                   \
  void name(const int32_t* coeff_ptr, intptr_t n_coeffs, const int16_t* zbin_ptr,       \
            const int16_t* round_ptr, const int16_t* quant_ptr,                         \
            const int16_t* quant_shift_ptr, int32_t* qcoeff_ptr, int32_t* dqcoeff_ptr,  \
            const int16_t* dequant_ptr, uint16_t* eob_ptr, const int16_t* scan,         \
            const int16_t* iscan) {                                                     \
    (void)iscan;                                                                        \
    quant_shim(coeff_ptr, n_coeffs, zbin_ptr, round_ptr, quant_ptr, quant_shift_ptr,    \
               qcoeff_ptr, dqcoeff_ptr, dequant_ptr, eob_ptr, scan, ls, kind, bd);      \
  }
QUANT_SHIM(av1_quantize_fp_hip, 0, LAVISH_QUANT_FP, 8)
QUANT_SHIM(av1_quantize_fp_32x32_hip, 1, LAVISH_QUANT_FP, 8)
QUANT_SHIM(av1_quantize_fp_64x64_hip, 2, LAVISH_QUANT_FP, 8)
QUANT_SHIM(aom_quantize_b_hip, 0, LAVISH_QUANT_B, 8)
QUANT_SHIM(aom_quantize_b_32x32_hip, 1, LAVISH_QUANT_B, 8)
QUANT_SHIM(aom_quantize_b_64x64_hip, 2, LAVISH_QUANT_B, 8)
QUANT_SHIM(aom_highbd_quantize_b_hip, 0, LAVISH_QUANT_B, 10)
QUANT_SHIM(aom_highbd_quantize_b_32x32_hip, 1, LAVISH_QUANT_B, 10)
QUANT_SHIM(aom_highbd_quantize_b_64x64_hip, 2, LAVISH_QUANT_B, 10)
#undef QUANT_SHIM

void av1_highbd_quantize_fp_hip(const int32_t* coeff_ptr, intptr_t count,
                                const int16_t* zbin_ptr, const int16_t* round_ptr,
                                const int16_t* quant_ptr, const int16_t* quant_shift_ptr,
                                int32_t* qcoeff_ptr, int32_t* dqcoeff_ptr,
                                const int16_t* dequant_ptr, uint16_t* eob_ptr,
                                const int16_t* scan, const int16_t* iscan, int log_scale) {
  (void)iscan;
  quant_shim(coeff_ptr, count, zbin_ptr, round_ptr, quant_ptr, quant_shift_ptr, qcoeff_ptr,
             dqcoeff_ptr, dequant_ptr, eob_ptr, scan, log_scale, LAVISH_QUANT_FP, 10);
}

}  // extern "C"
