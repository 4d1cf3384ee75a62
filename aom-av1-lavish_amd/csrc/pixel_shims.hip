// pixel_shims.hip -- per-call RTCD shims (host pointers) for the pixel-domain
// kernels of pixel.hip: SAD, variance, MSE, SSE, subtract, sum of squares,
// Hadamard, SATD, block error.  Each call stages the caller's block(s) into a
// per-thread device scratch (hipMemcpy2DAsync, so only the w x h window of a
// strided plane is read), runs the batch kernel on a single job, and copies
// the result back.  Drop-in parity, not speed (SURVEY.md 8(b) "Granularity").
// Highbd pixel pointers arrive tagged (CONVERT_TO_BYTEPTR, aom_ports/mem.h:79-80).
#include <string.h>

#include "lavish_internal.h"

namespace lavish {
namespace {

template <typename T>
T* untag(const uint8_t* p) {
  if constexpr (sizeof(T) == 2) return (T*)((uintptr_t)p << 1);
  else return (T*)p;
}

// bump allocator over the per-thread scratch for one shim call
struct Stage {
  char* base;
  size_t used = 0;
  hipStream_t s;
  explicit Stage(size_t cap) : base((char*)shim_scratch(cap)), s(shim_stream()) {}
  void* take(size_t bytes) {
    void* p = base + used;
    used += (bytes + 255) & ~(size_t)255;
    return p;
  }
  // copy a w x h window (stride in elements) into a compact device block
  template <typename T>
  T* block(const T* host, ptrdiff_t stride, int w, int h) {
    T* d = (T*)take((size_t)w * h * sizeof(T));
    LAVISH_CHECK(hipMemcpy2DAsync(d, (size_t)w * sizeof(T), host, (size_t)stride * sizeof(T),
                                  (size_t)w * sizeof(T), h, hipMemcpyHostToDevice, s));
    return d;
  }
  template <typename T>
  T* copy_in(const T* host, size_t n) {
    T* d = (T*)take(n * sizeof(T));
    LAVISH_CHECK(hipMemcpyAsync(d, host, n * sizeof(T), hipMemcpyHostToDevice, s));
    return d;
  }
  template <typename T>
  void copy_out(T* host, const T* dev, size_t n) {
    LAVISH_CHECK(hipMemcpyAsync(host, dev, n * sizeof(T), hipMemcpyDeviceToHost, s));
  }
  void sync() { LAVISH_CHECK(hipStreamSynchronize(s)); }
};

constexpr size_t kStageCap = 4u << 20;  // 128x128 u16 x (src + 4 refs + second) + outputs

void must(int rc, const char* what) {
  if (rc != 0) shim_reject(what, rc);
}

template <typename Pix>
void sad_shim(const uint8_t* src8, int ss, const uint8_t* const* refs8, int nrefs, int rs, int w,
              int h, int mode, const uint8_t* second8, uint32_t* out) {
  Stage st(kStageCap);
  const Pix* src = st.block(untag<Pix>(src8), ss, w, h);
  Pix* ref = (Pix*)st.take((size_t)nrefs * w * h * sizeof(Pix));
  LavishPixJob jb{};
  for (int k = 0; k < nrefs; ++k) {
    LAVISH_CHECK(hipMemcpy2DAsync(ref + (size_t)k * w * h, (size_t)w * sizeof(Pix),
                                  untag<Pix>(refs8[k]), (size_t)rs * sizeof(Pix),
                                  (size_t)w * sizeof(Pix), h, hipMemcpyHostToDevice, st.s));
    jb.ref_off[k] = (int64_t)k * w * h;
  }
  const Pix* second = mode == 2 ? st.copy_in(untag<Pix>(second8), (size_t)w * h) : nullptr;
  const LavishPixJob* djob = st.copy_in(&jb, 1);
  uint32_t* dout = (uint32_t*)st.take(4 * sizeof(uint32_t));
  must(lavish_sad_batch(src, w, ref, w, w, h, djob, 1, nrefs, mode, second, sizeof(Pix) == 2,
                        dout, st.s),
       "lavish_sad_batch");
  st.copy_out(out, dout, nrefs);
  st.sync();
}

template <typename Pix>
uint32_t sad1(const uint8_t* src, int ss, const uint8_t* ref, int rs, int w, int h, int mode,
              const uint8_t* second) {
  uint32_t r;
  const uint8_t* refs[1] = {ref};
  sad_shim<Pix>(src, ss, refs, 1, rs, w, h, mode, second, &r);
  return r;
}

// variance family: returns var_out; sse / sum through the pointers
template <typename Pix>
uint32_t var_shim(const uint8_t* a8, int as, const uint8_t* b8, int bs, int w, int h, int kind,
                  int bd, int xoff, int yoff, const uint8_t* second8, uint32_t* sse, int* sum) {
  Stage st(kStageCap);
  const bool sub = kind == 3 || kind == 5;
  const Pix* a = st.block(untag<Pix>(a8), as, sub ? w + 1 : w, sub ? h + 1 : h);
  const Pix* b = st.block(untag<Pix>(b8), bs, w, h);
  const Pix* second = kind == 5 ? st.copy_in(untag<Pix>(second8), (size_t)w * h) : nullptr;
  LavishPixJob jb{};
  jb.xoff = xoff;
  jb.yoff = yoff;
  const LavishPixJob* djob = st.copy_in(&jb, 1);
  uint32_t* dv = (uint32_t*)st.take(64);
  uint32_t* ds = (uint32_t*)st.take(64);
  int32_t* dsum = (int32_t*)st.take(64);
  must(lavish_variance_batch(a, sub ? w + 1 : w, b, w, w, h, djob, 1, kind, bd, sizeof(Pix) == 2,
                             second, dv, ds, dsum, nullptr, st.s),
       "lavish_variance_batch");
  uint32_t v = 0;
  st.copy_out(&v, dv, 1);
  if (sse) st.copy_out(sse, ds, 1);
  if (sum) st.copy_out(sum, dsum, 1);
  st.sync();
  return v;
}

template <typename Pix>
int64_t sse_shim(const uint8_t* a8, int as, const uint8_t* b8, int bs, int w, int h) {
  Stage st(kStageCap + (size_t)w * h * 2 * sizeof(Pix));
  const Pix* a = st.block(untag<Pix>(a8), as, w, h);
  const Pix* b = st.block(untag<Pix>(b8), bs, w, h);
  LavishPixJob jb{};
  const LavishPixJob* djob = st.copy_in(&jb, 1);
  int64_t* d = (int64_t*)st.take(64);
  must(lavish_variance_batch(a, w, b, w, w, h, djob, 1, 4, 8, sizeof(Pix) == 2, nullptr, nullptr,
                             nullptr, nullptr, d, st.s),
       "lavish_variance_batch");
  int64_t r = 0;
  st.copy_out(&r, d, 1);
  st.sync();
  return r;
}

template <typename Pix>
void subtract_shim(int rows, int cols, int16_t* diff, ptrdiff_t ds, const uint8_t* src8,
                   ptrdiff_t ss, const uint8_t* pred8, ptrdiff_t ps) {
  Stage st(kStageCap + (size_t)rows * cols * 4 * sizeof(Pix));
  const Pix* src = st.block(untag<Pix>(src8), ss, cols, rows);
  const Pix* pred = st.block(untag<Pix>(pred8), ps, cols, rows);
  int16_t* dd = (int16_t*)st.take((size_t)rows * cols * sizeof(int16_t));
  LavishPixJob jb{};
  const LavishPixJob* djob = st.copy_in(&jb, 1);
  must(lavish_subtract_batch(rows, cols, dd, cols, src, cols, pred, cols, djob, 1,
                             sizeof(Pix) == 2, st.s),
       "lavish_subtract_batch");
  LAVISH_CHECK(hipMemcpy2DAsync(diff, (size_t)ds * sizeof(int16_t), dd, (size_t)cols * 2,
                                (size_t)cols * 2, rows, hipMemcpyDeviceToHost, st.s));
  st.sync();
}

void hadamard_shim(int n, int highbd, const int16_t* src, ptrdiff_t stride, int32_t* coeff) {
  Stage st(kStageCap);
  const int16_t* d = st.block(src, stride, n, n);
  int32_t* dc = (int32_t*)st.take((size_t)n * n * sizeof(int32_t));
  LavishPixJob jb{};
  const LavishPixJob* djob = st.copy_in(&jb, 1);
  must(lavish_hadamard_batch(n, highbd, d, n, djob, 1, dc, st.s), "lavish_hadamard_batch");
  st.copy_out(coeff, dc, (size_t)n * n);
  st.sync();
}

int64_t block_error_shim(const int32_t* coeff, const int32_t* dqcoeff, intptr_t n, int64_t* ssz,
                         int bd) {
  Stage st(kStageCap + (size_t)n * 8);
  const int32_t* c = st.copy_in(coeff, n);
  const int32_t* dq = st.copy_in(dqcoeff, n);
  int64_t* de = (int64_t*)st.take(64);
  int64_t* dz = (int64_t*)st.take(64);
  must(lavish_block_error_batch(c, dq, (int)n, 1, bd, de, dz, st.s), "lavish_block_error_batch");
  int64_t e = 0;
  st.copy_out(&e, de, 1);
  st.copy_out(ssz, dz, 1);
  st.sync();
  return e;
}

// one block of av1_inv_txfm2d_add_* / av1_[highbd_]inv_txfm_add on host
// buffers: stage the coefficients and the destination window, run the batch
// kernel on a single job, copy the window back.
template <typename Pix>
void inv_shim(int tx_size, const int32_t* input, Pix* dst, int stride, int tx_type, int bd) {
  if (tx_size < 0 || tx_size >= 19 || !tx_type_valid(tx_size, tx_type)) {
    shim_reject("inverse transform (tx_size / tx_type)", -5);
    return;
  }
  const int W = tx_w(tx_size), H = tx_h(tx_size), n = max_eob(tx_size);
  Stage st(kStageCap);
  const int32_t* dc = st.copy_in(input, (size_t)n);
  Pix* dd = st.block(dst, stride, W, H);
  LavishInvJob jb{};
  jb.tx_type = tx_type;
  jb.eob = 1;  // the 2-D functions ignore eob
  const LavishInvJob* djob = st.copy_in(&jb, 1);
  must(lavish_inv_txfm_add_batch(dc, tx_size, djob, 1, dd, W, bd, sizeof(Pix) == 2, st.s),
       "lavish_inv_txfm_add_batch");
  LAVISH_CHECK(hipMemcpy2DAsync(dst, (size_t)stride * sizeof(Pix), dd, (size_t)W * sizeof(Pix),
                                (size_t)W * sizeof(Pix), H, hipMemcpyDeviceToHost, st.s));
  st.sync();
}

// the lossless branch of av1_highbd_inv_txfm_add_4x4_c (idct.c:42-57): only
// TX_4X4 looks at `lossless`; it adds the inverse Walsh-Hadamard transform
// (av1_highbd_iwht4x4_add, eob > 1 -> the 16-coefficient form).  Returns 1
// when it handled the block.
template <typename Pix>
int lossless_inv(const int32_t* input, Pix* dst, int stride, const LavishTxfmParam* p) {
  if (!p->lossless || p->tx_size != 0) return 0;
  uint16_t blk[16];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) blk[r * 4 + c] = dst[r * stride + c];
  iwht_host(input, blk, 4, p->eob, p->bd);
  // av1_inv_txfm_add_c (idct.c:281-302) copies back through (uint8_t)
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) dst[r * stride + c] = (Pix)blk[r * 4 + c];
  return 1;
}

// one block through the inter-prediction kernel with the caller's own
// kernels (path: 0 copy, 1 x_sr, 2 y_sr, 3 2d_sr); only the source window
// the C function reads is staged
template <typename Pix>
void conv_shim(const Pix* src, ptrdiff_t ss, Pix* dst, ptrdiff_t ds, int w, int h, int path,
               const LavishInterpFilterParams* fpx, int subx, const LavishInterpFilterParams* fpy,
               int suby, int r0, int r1, int bd) {
  int16_t c[28] = {0};
  int tx = 8, ty = 8;
  if (path & 1) {
    tx = fpx->taps;
    if (tx > 12) lavish::set_error("convolve shim: taps > 12", hipErrorInvalidValue, __FILE__, __LINE__);
    for (int k = 0; k < tx; ++k) c[4 + k] = fpx->filter_ptr[tx * (subx & 15) + k];
  }
  if (path & 2) {
    ty = fpy->taps;
    if (ty > 12) lavish::set_error("convolve shim: taps > 12", hipErrorInvalidValue, __FILE__, __LINE__);
    for (int k = 0; k < ty; ++k) c[16 + k] = fpy->filter_ptr[ty * (suby & 15) + k];
  }
  c[0] = (int16_t)path;
  c[1] = (int16_t)tx;
  c[2] = (int16_t)ty;
  const int foh = (path & 1) ? tx / 2 - 1 : 0, fov = (path & 2) ? ty / 2 - 1 : 0;
  const int ww = w + ((path & 1) ? tx - 1 : 0), wh = h + ((path & 2) ? ty - 1 : 0);
  Stage st(kStageCap);
  const Pix* win = st.block(src - fov * ss - foh, ss, ww, wh);
  st.take(64);  // slack for the kernel's dword-aligned over-read
  LavishInterPredJob jb{};
  jb.ref_off = (int64_t)fov * ww + foh;
  const LavishInterPredJob* djob = st.copy_in(&jb, 1);
  const int16_t* dc = st.copy_in(c, 28);
  Pix* dout = (Pix*)st.take((size_t)w * h * sizeof(Pix));
  must(inter_pred_batch(win, ww, 0, 0, 0, 0, w, h, djob, 1, nullptr, dout, w, bd,
                        sizeof(Pix) == 2, dc, r0, r1, st.s),
       "inter_pred_batch");
  LAVISH_CHECK(hipMemcpy2DAsync(dst, (size_t)ds * sizeof(Pix), dout, (size_t)w * sizeof(Pix),
                                (size_t)w * sizeof(Pix), h, hipMemcpyDeviceToHost, st.s));
  st.sync();
}

}  // namespace
}  // namespace lavish

using namespace lavish;

extern "C" {

#define SAD_SHIMS(w, h)                                                                          \
  unsigned int aom_sad##w##x##h##_hip(const uint8_t* s, int ss, const uint8_t* r, int rs) {      \
    return sad1<uint8_t>(s, ss, r, rs, w, h, 0, nullptr);                                        \
  }                                                                                              \
  unsigned int aom_sad_skip_##w##x##h##_hip(const uint8_t* s, int ss, const uint8_t* r,          \
                                            int rs) {                                            \
    return sad1<uint8_t>(s, ss, r, rs, w, h, 1, nullptr);                                        \
  }                                                                                              \
  unsigned int aom_sad##w##x##h##_avg_hip(const uint8_t* s, int ss, const uint8_t* r, int rs,    \
                                          const uint8_t* sp) {                                   \
    return sad1<uint8_t>(s, ss, r, rs, w, h, 2, sp);                                             \
  }                                                                                              \
  void aom_sad##w##x##h##x4d_hip(const uint8_t* s, int ss, const uint8_t* const r[4], int rs,    \
                                 uint32_t out[4]) {                                              \
    sad_shim<uint8_t>(s, ss, r, 4, rs, w, h, 0, nullptr, out);                                   \
  }                                                                                              \
  /* x3d forwards to x4d in the reference (sad.c:122-128) */                                     \
  void aom_sad##w##x##h##x3d_hip(const uint8_t* s, int ss, const uint8_t* const r[4], int rs,    \
                                 uint32_t out[4]) {                                              \
    sad_shim<uint8_t>(s, ss, r, 4, rs, w, h, 0, nullptr, out);                                   \
  }                                                                                              \
  void aom_sad##w##x##h##x4d_avg_hip(const uint8_t* s, int ss, const uint8_t* const r[4],        \
                                     int rs, const uint8_t* sp, uint32_t out[4]) {               \
    sad_shim<uint8_t>(s, ss, r, 4, rs, w, h, 2, sp, out);                                        \
  }                                                                                              \
  void aom_sad_skip_##w##x##h##x4d_hip(const uint8_t* s, int ss, const uint8_t* const r[4],      \
                                       int rs, uint32_t out[4]) {                                \
    sad_shim<uint8_t>(s, ss, r, 4, rs, w, h, 1, nullptr, out);                                   \
  }                                                                                              \
  unsigned int aom_highbd_sad##w##x##h##_hip(const uint8_t* s, int ss, const uint8_t* r,         \
                                             int rs) {                                           \
    return sad1<uint16_t>(s, ss, r, rs, w, h, 0, nullptr);                                       \
  }                                                                                              \
  unsigned int aom_highbd_sad_skip_##w##x##h##_hip(const uint8_t* s, int ss, const uint8_t* r,   \
                                                   int rs) {                                     \
    return sad1<uint16_t>(s, ss, r, rs, w, h, 1, nullptr);                                       \
  }                                                                                              \
  unsigned int aom_highbd_sad##w##x##h##_avg_hip(const uint8_t* s, int ss, const uint8_t* r,     \
                                                 int rs, const uint8_t* sp) {                    \
    return sad1<uint16_t>(s, ss, r, rs, w, h, 2, sp);                                            \
  }                                                                                              \
  void aom_highbd_sad##w##x##h##x4d_hip(const uint8_t* s, int ss, const uint8_t* const r[],      \
                                        int rs, uint32_t* out) {                                 \
    sad_shim<uint16_t>(s, ss, r, 4, rs, w, h, 0, nullptr, out);                                  \
  }                                                                                              \
  void aom_highbd_sad##w##x##h##x3d_hip(const uint8_t* s, int ss, const uint8_t* const r[],      \
                                        int rs, uint32_t* out) {                                 \
    sad_shim<uint16_t>(s, ss, r, 4, rs, w, h, 0, nullptr, out);                                  \
  }                                                                                              \
  void aom_highbd_sad_skip_##w##x##h##x4d_hip(const uint8_t* s, int ss,                          \
                                              const uint8_t* const r[], int rs, uint32_t* out) { \
    sad_shim<uint16_t>(s, ss, r, 4, rs, w, h, 1, nullptr, out);                                  \
  }

#define VAR_SHIMS_BD(pre, Pix, bd, w, h)                                                       \
  unsigned int pre##variance##w##x##h##_hip(const uint8_t* s, int ss, const uint8_t* r, int rs, \
                                            uint32_t* sse) {                                    \
    return var_shim<Pix>(s, ss, r, rs, w, h, 0, bd, 0, 0, nullptr, sse, nullptr);              \
  }                                                                                             \
  uint32_t pre##sub_pixel_variance##w##x##h##_hip(const uint8_t* s, int ss, int xo, int yo,     \
                                                  const uint8_t* r, int rs, uint32_t* sse) {    \
    return var_shim<Pix>(s, ss, r, rs, w, h, 3, bd, xo, yo, nullptr, sse, nullptr);            \
  }                                                                                             \
  uint32_t pre##sub_pixel_avg_variance##w##x##h##_hip(const uint8_t* s, int ss, int xo, int yo, \
                                                      const uint8_t* r, int rs, uint32_t* sse,  \
                                                      const uint8_t* sp) {                      \
    return var_shim<Pix>(s, ss, r, rs, w, h, 5, bd, xo, yo, sp, sse, nullptr);                 \
  }
#define VAR_SHIMS(w, h)                          \
  VAR_SHIMS_BD(aom_, uint8_t, 8, w, h)           \
  VAR_SHIMS_BD(aom_highbd_8_, uint16_t, 8, w, h) \
  VAR_SHIMS_BD(aom_highbd_10_, uint16_t, 10, w, h) \
  VAR_SHIMS_BD(aom_highbd_12_, uint16_t, 12, w, h)

LAVISH_ENCODER_BLOCK_SIZES(SAD_SHIMS)
LAVISH_ENCODER_BLOCK_SIZES(VAR_SHIMS)

#define MSE_SHIMS(pre, Pix, bd)                                                                 \
  void pre##get16x16var_hip(const uint8_t* s, int ss, const uint8_t* r, int rs,                 \
                            unsigned int* sse, int* sum) {                                      \
    var_shim<Pix>(s, ss, r, rs, 16, 16, 2, bd, 0, 0, nullptr, sse, sum);                        \
  }                                                                                             \
  void pre##get8x8var_hip(const uint8_t* s, int ss, const uint8_t* r, int rs, unsigned int* sse, \
                          int* sum) {                                                           \
    var_shim<Pix>(s, ss, r, rs, 8, 8, 2, bd, 0, 0, nullptr, sse, sum);                          \
  }                                                                                             \
  unsigned int pre##mse16x16_hip(const uint8_t* s, int ss, const uint8_t* r, int rs,            \
                                 unsigned int* sse) {                                           \
    return var_shim<Pix>(s, ss, r, rs, 16, 16, 1, bd, 0, 0, nullptr, sse, nullptr);             \
  }                                                                                             \
  unsigned int pre##mse16x8_hip(const uint8_t* s, int ss, const uint8_t* r, int rs,             \
                                unsigned int* sse) {                                            \
    return var_shim<Pix>(s, ss, r, rs, 16, 8, 1, bd, 0, 0, nullptr, sse, nullptr);              \
  }                                                                                             \
  unsigned int pre##mse8x16_hip(const uint8_t* s, int ss, const uint8_t* r, int rs,             \
                                unsigned int* sse) {                                            \
    return var_shim<Pix>(s, ss, r, rs, 8, 16, 1, bd, 0, 0, nullptr, sse, nullptr);              \
  }                                                                                             \
  unsigned int pre##mse8x8_hip(const uint8_t* s, int ss, const uint8_t* r, int rs,              \
                               unsigned int* sse) {                                             \
    return var_shim<Pix>(s, ss, r, rs, 8, 8, 1, bd, 0, 0, nullptr, sse, nullptr);               \
  }
MSE_SHIMS(aom_, uint8_t, 8)
MSE_SHIMS(aom_highbd_8_, uint16_t, 8)
MSE_SHIMS(aom_highbd_10_, uint16_t, 10)
MSE_SHIMS(aom_highbd_12_, uint16_t, 12)

void aom_subtract_block_hip(int rows, int cols, int16_t* diff, ptrdiff_t ds, const uint8_t* src,
                            ptrdiff_t ss, const uint8_t* pred, ptrdiff_t ps) {
  subtract_shim<uint8_t>(rows, cols, diff, ds, src, ss, pred, ps);
}
void aom_highbd_subtract_block_hip(int rows, int cols, int16_t* diff, ptrdiff_t ds,
                                   const uint8_t* src, ptrdiff_t ss, const uint8_t* pred,
                                   ptrdiff_t ps) {
  subtract_shim<uint16_t>(rows, cols, diff, ds, src, ss, pred, ps);
}

int64_t aom_sse_hip(const uint8_t* a, int as, const uint8_t* b, int bs, int w, int h) {
  return sse_shim<uint8_t>(a, as, b, bs, w, h);
}
int64_t aom_highbd_sse_hip(const uint8_t* a, int as, const uint8_t* b, int bs, int w, int h) {
  return sse_shim<uint16_t>(a, as, b, bs, w, h);
}

uint64_t aom_sum_squares_2d_i16_hip(const int16_t* src, int stride, int w, int h) {
  Stage st(kStageCap + (size_t)w * h * 2);
  const int16_t* d = st.block(src, stride, w, h);
  LavishPixJob jb{};
  const LavishPixJob* djob = st.copy_in(&jb, 1);
  uint64_t* dout = (uint64_t*)st.take(64);
  must(lavish_sum_squares_batch(d, w, w, h, djob, 1, dout, st.s), "lavish_sum_squares_batch");
  uint64_t r = 0;
  st.copy_out(&r, dout, 1);
  st.sync();
  return r;
}

void aom_hadamard_4x4_hip(const int16_t* s, ptrdiff_t st, int32_t* c) { hadamard_shim(4, 0, s, st, c); }
void aom_hadamard_8x8_hip(const int16_t* s, ptrdiff_t st, int32_t* c) { hadamard_shim(8, 0, s, st, c); }
void aom_hadamard_16x16_hip(const int16_t* s, ptrdiff_t st, int32_t* c) {
  hadamard_shim(16, 0, s, st, c);
}
void aom_hadamard_32x32_hip(const int16_t* s, ptrdiff_t st, int32_t* c) {
  hadamard_shim(32, 0, s, st, c);
}
void aom_highbd_hadamard_8x8_hip(const int16_t* s, ptrdiff_t st, int32_t* c) {
  hadamard_shim(8, 1, s, st, c);
}
void aom_highbd_hadamard_16x16_hip(const int16_t* s, ptrdiff_t st, int32_t* c) {
  hadamard_shim(16, 1, s, st, c);
}
void aom_highbd_hadamard_32x32_hip(const int16_t* s, ptrdiff_t st, int32_t* c) {
  hadamard_shim(32, 1, s, st, c);
}

int aom_satd_hip(const int32_t* coeff, int length) {
  Stage st(kStageCap + (size_t)length * 4);
  const int32_t* d = st.copy_in(coeff, length);
  int* dout = (int*)st.take(64);
  must(lavish_satd_batch(d, length, 1, dout, st.s), "lavish_satd_batch");
  int r = 0;
  st.copy_out(&r, dout, 1);
  st.sync();
  return r;
}

// aom_hadamard_lp_{8x8,16x16} and the dual form (two 8x8 side by side,
// avg.c:238-245); aom_satd_lp; av1_block_error_lp
static void hadamard_lp_shim(int n, int nblk, const int16_t* src, ptrdiff_t stride,
                             int16_t* coeff) {
  Stage st(kStageCap);
  const int16_t* d = st.block(src, stride, n * nblk, n);
  int16_t* dc = (int16_t*)st.take((size_t)nblk * n * n * sizeof(int16_t));
  LavishPixJob jb[2] = {};
  for (int k = 0; k < nblk; ++k) {
    jb[k].src_off = (int64_t)k * n;
    jb[k].aux_off = (int64_t)k * n * n;
  }
  const LavishPixJob* djob = st.copy_in(jb, nblk);
  must(lavish_hadamard_lp_batch(n, d, n * nblk, djob, nblk, dc, st.s), "lavish_hadamard_lp_batch");
  st.copy_out(coeff, dc, (size_t)nblk * n * n);
  st.sync();
}
void aom_hadamard_lp_8x8_hip(const int16_t* s, ptrdiff_t st, int16_t* c) {
  hadamard_lp_shim(8, 1, s, st, c);
}
void aom_hadamard_lp_16x16_hip(const int16_t* s, ptrdiff_t st, int16_t* c) {
  hadamard_lp_shim(16, 1, s, st, c);
}
void aom_hadamard_lp_8x8_dual_hip(const int16_t* s, ptrdiff_t st, int16_t* c) {
  hadamard_lp_shim(8, 2, s, st, c);
}

int aom_satd_lp_hip(const int16_t* coeff, int length) {
  Stage st(kStageCap + (size_t)length * 2);
  const int16_t* d = st.copy_in(coeff, length);
  int* dout = (int*)st.take(64);
  must(lavish_satd_lp_batch(d, length, 1, dout, st.s), "lavish_satd_lp_batch");
  int r = 0;
  st.copy_out(&r, dout, 1);
  st.sync();
  return r;
}

int64_t av1_block_error_lp_hip(const int16_t* coeff, const int16_t* dqcoeff, intptr_t n) {
  Stage st(kStageCap + (size_t)n * 4);
  const int16_t* c = st.copy_in(coeff, n);
  const int16_t* dq = st.copy_in(dqcoeff, n);
  int64_t* de = (int64_t*)st.take(64);
  must(lavish_block_error_lp_batch(c, dq, (int)n, 1, de, st.s), "lavish_block_error_lp_batch");
  int64_t e = 0;
  st.copy_out(&e, de, 1);
  st.sync();
  return e;
}

// (sum, sse) of an int16 block through lavish_sum_sse_batch
static void sum_sse_shim(const int16_t* src, int stride, int w, int h, int32_t* sum,
                         int64_t* sse) {
  Stage st(kStageCap + (size_t)w * h * 2);
  const int16_t* d = st.block(src, stride, w, h);
  LavishPixJob jb{};
  const LavishPixJob* djob = st.copy_in(&jb, 1);
  int32_t* dsum = (int32_t*)st.take(64);
  int64_t* dsse = (int64_t*)st.take(64);
  must(lavish_sum_sse_batch(d, w, w, h, djob, 1, dsum, dsse, st.s), "lavish_sum_sse_batch");
  st.copy_out(sum, dsum, 1);
  st.copy_out(sse, dsse, 1);
  st.sync();
}
// aom_sum_sse_2d_i16 (sum_squares.c:75-90): *sum accumulates (the caller
// initialises it), the return is the sum of squares
uint64_t aom_sum_sse_2d_i16_hip(const int16_t* src, int src_stride, int width, int height,
                                int* sum) {
  int32_t s = 0;
  int64_t ss = 0;
  sum_sse_shim(src, src_stride, width, height, &s, &ss);
  *sum += s;
  return (uint64_t)ss;
}
// aom_get_blk_sse_sum (blk_sse_sum.c:14-27)
void aom_get_blk_sse_sum_hip(const int16_t* data, int stride, int bw, int bh, int* x_sum,
                             int64_t* x2_sum) {
  int32_t s = 0;
  sum_sse_shim(data, stride, bw, bh, &s, x2_sum);
  *x_sum = s;
}

int64_t av1_block_error_hip(const int32_t* coeff, const int32_t* dqcoeff, intptr_t n,
                            int64_t* ssz) {
  return block_error_shim(coeff, dqcoeff, n, ssz, 0);
}
int64_t av1_highbd_block_error_hip(const int32_t* coeff, const int32_t* dqcoeff, intptr_t n,
                                   int64_t* ssz, int bd) {
  return block_error_shim(coeff, dqcoeff, n, ssz, bd);
}


// ---- inverse transforms (av1/common/av1_rtcd_defs.pl:137-243) ----
static int size_of(int w, int h) {
  for (int s = 0; s < 19; ++s)
    if (tx_w(s) == w && tx_h(s) == h) return s;
  return -1;
}
#define INV2D_SHIM(w, h)                                                                      \
  void av1_inv_txfm2d_add_##w##x##h##_hip(const int32_t* input, uint16_t* output, int stride,  \
                                          uint8_t tx_type, int bd) {                          \
    inv_shim<uint16_t>(size_of(w, h), input, output, stride, tx_type, bd);                    \
  }
LAVISH_TX_SIZES_ALL(INV2D_SHIM)

// av1_inv_txfm_add_c (idct.c:281-302): u8 destination, bd 8
void av1_inv_txfm_add_hip(const int32_t* dqcoeff, uint8_t* dst, int stride,
                          const LavishTxfmParam* p) {
  if (lossless_inv<uint8_t>(dqcoeff, dst, stride, p)) return;
  inv_shim<uint8_t>(p->tx_size, dqcoeff, dst, stride, p->tx_type, 8);
}
// av1_highbd_inv_txfm_add_c (idct.c:212-279): tagged u16 destination
void av1_highbd_inv_txfm_add_hip(const int32_t* input, uint8_t* dest, int stride,
                                 const LavishTxfmParam* p) {
  if (lossless_inv<uint16_t>(input, untag<uint16_t>(dest), stride, p)) return;
  inv_shim<uint16_t>(p->tx_size, input, untag<uint16_t>(dest), stride, p->tx_type, p->bd);
}
#define HBD_INV_SHIM(w, h)                                                                    \
  void av1_highbd_inv_txfm_add_##w##x##h##_hip(const int32_t* input, uint8_t* dest,           \
                                               int stride, const LavishTxfmParam* p) {        \
    if (w == 4 && h == 4 && lossless_inv<uint16_t>(input, untag<uint16_t>(dest), stride, p))  \
      return;                                                                                 \
    inv_shim<uint16_t>(size_of(w, h), input, untag<uint16_t>(dest), stride, p->tx_type,      \
                       p->bd);                                                                \
  }
HBD_INV_SHIM(4, 4) HBD_INV_SHIM(8, 8) HBD_INV_SHIM(4, 8) HBD_INV_SHIM(8, 4)
HBD_INV_SHIM(4, 16) HBD_INV_SHIM(16, 4) HBD_INV_SHIM(8, 16) HBD_INV_SHIM(16, 8)
HBD_INV_SHIM(16, 32) HBD_INV_SHIM(32, 16) HBD_INV_SHIM(32, 32) HBD_INV_SHIM(32, 64)
HBD_INV_SHIM(64, 32) HBD_INV_SHIM(64, 64) HBD_INV_SHIM(8, 32) HBD_INV_SHIM(32, 8)
HBD_INV_SHIM(16, 64) HBD_INV_SHIM(64, 16)

// ---- TX-pruning features (av1/common/av1_rtcd_defs.pl:469) ----
void av1_get_horver_correlation_full_hip(const int16_t* diff, int stride, int w, int h,
                                         float* hcorr, float* vcorr) {
  Stage st(kStageCap);
  const int16_t* d = st.block(diff, stride, w, h);
  float* dout = (float*)st.take(2 * sizeof(float));
  must(lavish_horver_correlation_batch(d, w, w, h, w, h, dout, dout + 1, st.s),
       "lavish_horver_correlation_batch");
  float r[2];
  st.copy_out(r, dout, 2);
  st.sync();
  *hcorr = r[0];
  *vcorr = r[1];
}

void av1_nn_predict_hip(const float* input_nodes, const LavishNNConfig* cfg, int reduce_prec,
                        float* output) {
  Stage st(kStageCap);
  const float* din = st.copy_in(input_nodes, (size_t)cfg->num_inputs);
  float* dout = (float*)st.take((size_t)cfg->num_outputs * sizeof(float));
  must(lavish_nn_predict_batch(din, cfg, reduce_prec, dout, 1, st.s), "lavish_nn_predict_batch");
  st.copy_out(output, dout, (size_t)cfg->num_outputs);
  st.sync();
}

void av1_convolve_2d_sr_hip(const uint8_t* src, int src_stride, uint8_t* dst, int dst_stride,
                            int w, int h, const LavishInterpFilterParams* fpx,
                            const LavishInterpFilterParams* fpy, const int subpel_x_qn,
                            const int subpel_y_qn, LavishConvolveParams* cp) {
  conv_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, 3, fpx, subpel_x_qn, fpy,
                     subpel_y_qn, cp->round_0, cp->round_1, 8);
}
void av1_convolve_x_sr_hip(const uint8_t* src, int src_stride, uint8_t* dst, int dst_stride,
                           int w, int h, const LavishInterpFilterParams* fpx,
                           const int subpel_x_qn, LavishConvolveParams* cp) {
  conv_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, 1, fpx, subpel_x_qn, nullptr, 0,
                     cp->round_0, cp->round_1, 8);
}
void av1_convolve_y_sr_hip(const uint8_t* src, int src_stride, uint8_t* dst, int dst_stride,
                           int w, int h, const LavishInterpFilterParams* fpy,
                           const int subpel_y_qn) {
  conv_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, 2, nullptr, 0, fpy, subpel_y_qn, 3,
                     11, 8);
}
void av1_highbd_convolve_2d_sr_hip(const uint16_t* src, int src_stride, uint16_t* dst,
                                   int dst_stride, int w, int h,
                                   const LavishInterpFilterParams* fpx,
                                   const LavishInterpFilterParams* fpy, const int subpel_x_qn,
                                   const int subpel_y_qn, LavishConvolveParams* cp, int bd) {
  conv_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, 3, fpx, subpel_x_qn, fpy,
                      subpel_y_qn, cp->round_0, cp->round_1, bd);
}
void av1_highbd_convolve_x_sr_hip(const uint16_t* src, int src_stride, uint16_t* dst,
                                  int dst_stride, int w, int h,
                                  const LavishInterpFilterParams* fpx, const int subpel_x_qn,
                                  LavishConvolveParams* cp, int bd) {
  conv_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, 1, fpx, subpel_x_qn, nullptr, 0,
                      cp->round_0, cp->round_1, bd);
}
void av1_highbd_convolve_y_sr_hip(const uint16_t* src, int src_stride, uint16_t* dst,
                                  int dst_stride, int w, int h,
                                  const LavishInterpFilterParams* fpy, const int subpel_y_qn,
                                  int bd) {
  conv_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, 2, nullptr, 0, fpy, subpel_y_qn,
                      3, 11, bd);
}
void aom_convolve_copy_hip(const uint8_t* src, ptrdiff_t src_stride, uint8_t* dst,
                           ptrdiff_t dst_stride, int w, int h) {
  conv_shim<uint8_t>(src, src_stride, dst, dst_stride, w, h, 0, nullptr, 0, nullptr, 0, 3, 11, 8);
}
void aom_highbd_convolve_copy_hip(const uint16_t* src, ptrdiff_t src_stride, uint16_t* dst,
                                  ptrdiff_t dst_stride, int w, int h) {
  conv_shim<uint16_t>(src, src_stride, dst, dst_stride, w, h, 0, nullptr, 0, nullptr, 0, 3, 11,
                      12);
}

}  // extern "C"
