// pixel.hip -- batched pixel-domain kernels of the RDO hot path for gfx950:
// SAD (+skip, +avg, x4d), variance / MSE / get_var, bilinear sub-pixel
// variance, SSE, residual subtract, sum of squares, Hadamard 4..32, SATD and
// block error.  Each job is one block; one wave owns a job (or, for the tiny
// per-coefficient ones, a group of lanes), and reductions use wave shuffles.
//
// Semantics (all integer, bit-exact):
//   sad/_skip/_avg/x4d      aom_dsp/sad.c:22-129, aom_comp_avg_pred_c
//                           aom_dsp/variance.c:285-298
//   variance / mse / getvar aom_dsp/variance.c:38-55,123-130,187-238
//   highbd 8/10/12 variance aom_dsp/variance.c:321-408
//   sub-pixel variance      aom_dsp/variance.c:73-145,454-520
//   sse                     aom_dsp/sse.c:19-54
//   subtract                aom_dsp/subtract.c:20-54
//   sum_squares_2d_i16      aom_dsp/sum_squares.c:16-30
//   hadamard / satd         aom_dsp/avg.c:102-348,509-516
//   hadamard_lp / satd_lp   aom_dsp/avg.c:207-316,518-524
//   block_error (+_lp)      av1/encoder/rdopt.c:635-682
//   sum_sse_2d_i16          aom_dsp/sum_squares.c:75-90
//   get_blk_sse_sum         aom_dsp/blk_sse_sum.c:14-27
#include "lavish_internal.h"

namespace lavish {

__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

// ---------------------------------------------------------------- SAD ----
// mode 0: SAD, 1: 2 x SAD of even rows (sad_skip), 2: SAD against the
// rounded average of ref and second_pred (w x h, stride w) (sad_avg).
template <typename Pix>
__global__ __launch_bounds__(64) void sad_kernel(const Pix* src, int ss, const Pix* ref, int rs,
                                                 int w, int h, const LavishPixJob* jobs,
                                                 int nrefs, int mode, const Pix* second,
                                                 uint32_t* out) {
  const LavishPixJob jb = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  const int rows = mode == 1 ? h / 2 : h;
  const int rstep = mode == 1 ? 2 : 1;
  const Pix* s = src + jb.src_off;
  for (int k = 0; k < nrefs; ++k) {
    const Pix* r = ref + jb.ref_off[k];
    uint32_t acc = 0;
    for (int i = lane; i < rows * w; i += 64) {
      const int y = i / w, x = i - y * w;
      const int sv = s[(int64_t)y * rstep * ss + x];
      int rv = r[(int64_t)y * rstep * rs + x];
      if (mode == 2) rv = (second[jb.aux_off + (int64_t)y * w + x] + rv + 1) >> 1;
      acc += (uint32_t)abs(sv - rv);
    }
    acc = wave_sum32(acc);
    if (lane == 0) out[(int64_t)blockIdx.x * nrefs + k] = mode == 1 ? 2 * acc : acc;
  }
}

// ----------------------------------------------- 8-bit SAD / variance ----
// The u8 forms of sad_kernel / var_kernel (modes 0-2, kinds 0-2 and 4) on
// 4-byte words: a job's rows are cut into chunks of C = min(4, w / 4) words,
// each lane takes whole chunks with byte-addressed loads (16 / 8 / 4 bytes;
// the queues allow unaligned access), and a wave holds 64 / LPJ jobs of LPJ
// = min(64, chunks) lanes each, so a 4x4 job uses 4 lanes, not a wave.
//   SAD: v_sad_u8 per word (the avg mode first takes v_lerp_u8 of ref and
//        second_pred, ROUND_POWER_OF_TWO(a + b, 1) per byte);
//   variance: sum = sad(a, 0) - sad(b, 0), sse = a.a + b.b - 2 a.b with
//        v_dot4_u32_u8 (exact mod 2^32; the true sse < 2^32 for 8-bit).
struct U8Shape {
  int lw4;   // log2(w / 4)
  int lc;    // log2(words per chunk)
  int lcpr;  // log2(chunks per row)
  int lpj;   // lanes per job (power of two, <= 64)
  int chunks;
};

__device__ __forceinline__ void load_words(const uint8_t* p, int c, uint32_t (&w)[4]) {
  if (c == 4) {
    const u32x4u v = *(const __attribute__((address_space(1))) u32x4u*)p;
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else if (c == 2) {
    const u32x2u v = *(const __attribute__((address_space(1))) u32x2u*)p;
    w[0] = v.x; w[1] = v.y; w[2] = 0; w[3] = 0;
  } else {
    w[0] = *(const __attribute__((address_space(1))) u32u*)p;
    w[1] = 0; w[2] = 0; w[3] = 0;
  }
}

// sum over the LPJ-lane group of a job (every lane of the group gets it)
__device__ __forceinline__ uint32_t group_sum(uint32_t v, int lpj) {
  for (int m = 1; m < lpj; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

__global__ __launch_bounds__(256) void sad_u8_kernel(const uint8_t* __restrict__ src, int ss,
                                                     const uint8_t* __restrict__ ref, int rs,
                                                     U8Shape sh, const LavishPixJob* __restrict__ jobs,
                                                     int njobs, int nrefs, int mode,
                                                     const uint8_t* __restrict__ second, int w,
                                                     uint32_t* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int j = t >> __builtin_ctz(sh.lpj);
  const int q = t & (sh.lpj - 1);
  const bool live = j < njobs;
  const LavishPixJob jb = jobs[live ? j : njobs - 1];
  const int rstep = mode == 1 ? 2 : 1;
  const int c = 1 << sh.lc;
  for (int k = 0; k < nrefs; ++k) {
    uint32_t acc = 0;
    for (int i = q; i < sh.chunks; i += sh.lpj) {
      const int y = i >> sh.lcpr, x = (i & ((1 << sh.lcpr) - 1)) << (sh.lc + 2);
      uint32_t a[4], b[4];
      load_words(src + jb.src_off + (int64_t)y * rstep * ss + x, c, a);
      load_words(ref + jb.ref_off[k] + (int64_t)y * rstep * rs + x, c, b);
      if (mode == 2) {
        uint32_t p[4];
        load_words(second + jb.aux_off + (int64_t)y * w + x, c, p);
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = __builtin_amdgcn_lerp(b[u], p[u], 0x01010101u);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_sad_u8(a[u], b[u], acc);
    }
    acc = group_sum(acc, sh.lpj);
    if (live && q == 0) out[(int64_t)j * nrefs + k] = mode == 1 ? 2 * acc : acc;
  }
}

__global__ __launch_bounds__(256) void var_u8_kernel(const uint8_t* __restrict__ a, int as,
                                                     const uint8_t* __restrict__ b, int bs,
                                                     U8Shape sh, int w, int h,
                                                     const LavishPixJob* __restrict__ jobs,
                                                     int njobs, int kind,
                                                     uint32_t* __restrict__ var_out,
                                                     uint32_t* __restrict__ sse_out,
                                                     int32_t* __restrict__ sum_out,
                                                     int64_t* __restrict__ sse64_out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int j = t >> __builtin_ctz(sh.lpj);
  const int q = t & (sh.lpj - 1);
  const bool live = j < njobs;
  const LavishPixJob jb = jobs[live ? j : njobs - 1];
  const int c = 1 << sh.lc;
  uint32_t sa = 0, sb = 0, aa = 0, bb = 0, ab = 0;
  for (int i = q; i < sh.chunks; i += sh.lpj) {
    const int y = i >> sh.lcpr, x = (i & ((1 << sh.lcpr) - 1)) << (sh.lc + 2);
    uint32_t va[4], vb[4];
    load_words(a + jb.src_off + (int64_t)y * as + x, c, va);
    load_words(b + jb.ref_off[0] + (int64_t)y * bs + x, c, vb);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sa = __builtin_amdgcn_sad_u8(va[u], 0u, sa);
      sb = __builtin_amdgcn_sad_u8(vb[u], 0u, sb);
      aa = __builtin_amdgcn_udot4(va[u], va[u], aa, false);
      bb = __builtin_amdgcn_udot4(vb[u], vb[u], bb, false);
      ab = __builtin_amdgcn_udot4(va[u], vb[u], ab, false);
    }
  }
  const int sum = (int)group_sum(sa, sh.lpj) - (int)group_sum(sb, sh.lpj);
  const uint32_t sse = group_sum(aa, sh.lpj) + group_sum(bb, sh.lpj) - 2u * group_sum(ab, sh.lpj);
  if (!live || q != 0) return;
  if (kind == 4) {
    sse64_out[j] = (int64_t)sse;
    return;
  }
  if (sse_out) sse_out[j] = sse;
  if (sum_out) sum_out[j] = sum;
  if (var_out) var_out[j] = kind == 1 ? sse : sse - (uint32_t)(((int64_t)sum * sum) / (w * h));
}

// ---------------------------------------------- u16 (highbd) SAD / variance ----
// The same word-chunk layout over u16 samples (a 4-byte word = 2 samples,
// chunks of up to 8 samples = one 16-byte load): SAD on v_sad_u16; variance
// with exact 64-bit per-lane sums, then highbd_variance64's rounding for
// 10 / 12 bits (aom_dsp/variance.c:321-408) as var_kernel does it.
__device__ __forceinline__ void load_words16(const uint16_t* p, int c, uint32_t (&w)[4]) {
  load_words((const uint8_t*)p, c, w);
}

__global__ __launch_bounds__(256) void sad_u16_kernel(const uint16_t* __restrict__ src, int ss,
                                                      const uint16_t* __restrict__ ref, int rs,
                                                      U8Shape sh, const LavishPixJob* __restrict__ jobs,
                                                      int njobs, int nrefs, int mode,
                                                      const uint16_t* __restrict__ second, int w,
                                                      uint32_t* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int j = t >> __builtin_ctz(sh.lpj);
  const int q = t & (sh.lpj - 1);
  const bool live = j < njobs;
  const LavishPixJob jb = jobs[live ? j : njobs - 1];
  const int rstep = mode == 1 ? 2 : 1;
  const int c = 1 << sh.lc;  // words per chunk (2 samples each)
  for (int k = 0; k < nrefs; ++k) {
    uint32_t acc = 0;
    for (int i = q; i < sh.chunks; i += sh.lpj) {
      const int y = i >> sh.lcpr, x = (i & ((1 << sh.lcpr) - 1)) << (sh.lc + 1);
      uint32_t a[4], b[4];
      load_words16(src + jb.src_off + (int64_t)y * rstep * ss + x, c, a);
      load_words16(ref + jb.ref_off[k] + (int64_t)y * rstep * rs + x, c, b);
      if (mode == 2) {
        uint32_t p[4];
        load_words16(second + jb.aux_off + (int64_t)y * w + x, c, p);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t lo = ((b[u] & 0xFFFF) + (p[u] & 0xFFFF) + 1) >> 1;
          const uint32_t hi = ((b[u] >> 16) + (p[u] >> 16) + 1) >> 1;
          b[u] = lo | (hi << 16);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_sad_u16(a[u], b[u], acc);
    }
    acc = group_sum(acc, sh.lpj);
    if (live && q == 0) out[(int64_t)j * nrefs + k] = mode == 1 ? 2 * acc : acc;
  }
}

__global__ __launch_bounds__(256) void var_u16_kernel(const uint16_t* __restrict__ a, int as,
                                                      const uint16_t* __restrict__ b, int bs,
                                                      U8Shape sh, int w, int h,
                                                      const LavishPixJob* __restrict__ jobs,
                                                      int njobs, int kind, int bd,
                                                      uint32_t* __restrict__ var_out,
                                                      uint32_t* __restrict__ sse_out,
                                                      int32_t* __restrict__ sum_out,
                                                      int64_t* __restrict__ sse64_out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int j = t >> __builtin_ctz(sh.lpj);
  const int q = t & (sh.lpj - 1);
  const bool live = j < njobs;
  const LavishPixJob jb = jobs[live ? j : njobs - 1];
  const int c = 1 << sh.lc;
  int64_t sum = 0;
  uint64_t sse = 0;
  for (int i = q; i < sh.chunks; i += sh.lpj) {
    const int y = i >> sh.lcpr, x = (i & ((1 << sh.lcpr) - 1)) << (sh.lc + 1);
    uint32_t va[4], vb[4];
    load_words16(a + jb.src_off + (int64_t)y * as + x, c, va);
    load_words16(b + jb.ref_off[0] + (int64_t)y * bs + x, c, vb);
    int s = 0;
    uint32_t q2 = 0;  // <= 8 squares of 12-bit differences: < 2^28
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int d0 = (int)(va[u] & 0xFFFF) - (int)(vb[u] & 0xFFFF);
      const int d1 = (int)(va[u] >> 16) - (int)(vb[u] >> 16);
      s += d0 + d1;
      q2 += (uint32_t)(d0 * d0) + (uint32_t)(d1 * d1);
    }
    sum += s;
    sse += q2;
  }
  for (int m = 1; m < sh.lpj; m <<= 1) {
    sum += __shfl_xor(sum, m);
    sse += (uint64_t)__shfl_xor((int64_t)sse, m);
  }
  if (!live || q != 0) return;
  if (kind == 4) {
    sse64_out[j] = (int64_t)sse;
    return;
  }
  uint32_t s32;
  int sm;
  if (bd == 8) {
    s32 = (uint32_t)sse;
    sm = (int)sum;
  } else {
    const int ss_ = bd == 10 ? 4 : 8, sh2 = bd == 10 ? 2 : 4;
    s32 = (uint32_t)((sse + ((1ull << ss_) >> 1)) >> ss_);
    sm = (int)((sum + ((1ll << sh2) >> 1)) >> sh2);
  }
  if (sse_out) sse_out[j] = s32;
  if (sum_out) sum_out[j] = sm;
  if (var_out) {
    if (kind == 1) {
      var_out[j] = s32;
    } else if (bd == 8) {
      var_out[j] = s32 - (uint32_t)(((int64_t)sm * sm) / (w * h));
    } else {
      const int64_t v = (int64_t)s32 - (((int64_t)sm * sm) / (w * h));
      var_out[j] = v >= 0 ? (uint32_t)v : 0;
    }
  }
}

static int ilog2(int v) { return 31 - __builtin_clz(v); }

// the u16 word-chunk layout (2 samples per word, chunks of <= 8 samples)
static bool u16_shape(int w, int rows, U8Shape& sh) {
  if (w < 2 || (w & (w - 1)) || rows < 1 || (rows & (rows - 1))) return false;
  sh.lw4 = ilog2(w / 2);  // log2(words per row)
  sh.lc = sh.lw4 < 2 ? sh.lw4 : 2;
  sh.lcpr = sh.lw4 - sh.lc;
  sh.chunks = rows << sh.lcpr;
  sh.lpj = sh.chunks < 64 ? sh.chunks : 64;
  return true;
}

// the u8 word-chunk layout of a w x h block with `rows` rows read; false when
// w or rows is not a power of two >= 4 / >= 1
static bool u8_shape(int w, int rows, U8Shape& sh) {
  if (w < 4 || (w & (w - 1)) || rows < 1 || (rows & (rows - 1))) return false;
  sh.lw4 = ilog2(w / 4);
  sh.lc = sh.lw4 < 2 ? sh.lw4 : 2;
  sh.lcpr = sh.lw4 - sh.lc;
  sh.chunks = rows << sh.lcpr;
  sh.lpj = sh.chunks < 64 ? sh.chunks : 64;
  return true;
}

// ------------------------------------------------------------ variance ----
// d = a - b with a = the first rtcd pointer (src; the bilinear-filtered one
// for sub-pixel variance) at job.src_off and b = the second at job.ref_off[0].  kind 0: variance, 1: mse (returns sse), 2: get_var
// (sse + sum), 3: sub-pixel variance of the bilinear-filtered `a`
// (xoff/yoff per job), 4: sse only with uint64 result (aom_sse, highbd sse),
// 5: as 3 with the filtered block first averaged with second_pred (w x h,
// stride w, at job.aux_off): sub_pixel_avg_variance.
// bd: 8 for lowbd; 8/10/12 for the highbd rounding variants (Pix=uint16).
template <typename Pix>
__global__ __launch_bounds__(64) void var_kernel(const Pix* a, int as, const Pix* b, int bs,
                                                 int w, int h, const LavishPixJob* jobs,
                                                 int kind, int bd, const Pix* second,
                                                 uint32_t* var_out,
                                                 uint32_t* sse_out, int32_t* sum_out,
                                                 int64_t* sse64_out) {
  constexpr uint8_t kBil[8][2] = {{128, 0}, {112, 16}, {96, 32}, {80, 48},
                                  {64, 64}, {48, 80},  {32, 96}, {16, 112}};
  const LavishPixJob jb = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  const Pix* pa = a + jb.src_off;
  const Pix* pb = b + jb.ref_off[0];
  int64_t sum = 0;
  uint64_t sse = 0;
  const int xo = jb.xoff, yo = jb.yoff;
  for (int i = lane; i < w * h; i += 64) {
    const int y = i / w, x = i - y * w;
    int av;
    if (kind == 3 || kind == 5) {
      // first pass rows y and y+1 at column x, then the vertical tap
      const Pix* r0 = pa + (int64_t)y * as + x;
      const Pix* r1 = r0 + as;
      const int f0 = kBil[xo][0], f1 = kBil[xo][1];
      const int h0 = (r0[0] * f0 + r0[1] * f1 + 64) >> 7;
      const int h1 = (r1[0] * f0 + r1[1] * f1 + 64) >> 7;
      av = (h0 * kBil[yo][0] + h1 * kBil[yo][1] + 64) >> 7;
      if (sizeof(Pix) == 1) av &= 0xFF;  // lowbd second pass stores uint8
      else av &= 0xFFFF;
      if (kind == 5) av = (second[jb.aux_off + (int64_t)y * w + x] + av + 1) >> 1;
    } else {
      av = pa[(int64_t)y * as + x];
    }
    const int d = av - (int)pb[(int64_t)y * bs + x];
    sum += d;
    sse += (uint32_t)(d * d);
  }
  sum = wave_sum64(sum);
  sse = (uint64_t)wave_sum64((int64_t)sse);
  if (lane != 0) return;
  const int64_t j = blockIdx.x;
  if (kind == 4) {
    sse64_out[j] = (int64_t)sse;
    return;
  }
  uint32_t s32;
  int sm;
  if (bd == 8) {
    s32 = (uint32_t)sse;
    sm = (int)sum;
  } else {
    const int ss_ = bd == 10 ? 4 : 8, sh = bd == 10 ? 2 : 4;
    s32 = (uint32_t)((sse + ((1ull << ss_) >> 1)) >> ss_);
    sm = (int)((sum + ((1ll << sh) >> 1)) >> sh);
  }
  if (sse_out) sse_out[j] = s32;
  if (sum_out) sum_out[j] = sm;
  if (var_out) {
    if (kind == 1) {
      var_out[j] = s32;
    } else if (sizeof(Pix) == 1 || bd == 8) {
      var_out[j] = s32 - (uint32_t)(((int64_t)sm * sm) / (w * h));
    } else {
      const int64_t v = (int64_t)s32 - (((int64_t)sm * sm) / (w * h));
      var_out[j] = v >= 0 ? (uint32_t)v : 0;
    }
  }
}

// ------------------------------------------------------------ subtract ----
template <typename Pix>
__global__ void subtract_kernel(int rows, int cols, int16_t* diff, int ds, const Pix* src, int ss,
                                const Pix* pred, int ps, const LavishPixJob* jobs) {
  const LavishPixJob jb = jobs[blockIdx.x];
  for (int i = threadIdx.x; i < rows * cols; i += blockDim.x) {
    const int y = i / cols, x = i - y * cols;
    diff[jb.aux_off + (int64_t)y * ds + x] =
        (int16_t)((int)src[jb.src_off + (int64_t)y * ss + x] -
                  (int)pred[jb.ref_off[0] + (int64_t)y * ps + x]);
  }
}

// --------------------------------------------------------- sum squares ----
__global__ __launch_bounds__(64) void sum_squares_kernel(const int16_t* src, int stride, int w,
                                                         int h, const LavishPixJob* jobs,
                                                         uint64_t* out) {
  const LavishPixJob jb = jobs[blockIdx.x];
  uint64_t acc = 0;
  for (int i = threadIdx.x; i < w * h; i += 64) {
    const int y = i / w, x = i - y * w;
    const int v = src[jb.src_off + (int64_t)y * stride + x];
    acc += (uint64_t)(v * v);
  }
  acc = (uint64_t)wave_sum64((int64_t)acc);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// ------------------------------------------------------------ hadamard ----
// int16 butterflies with the reference's output permutations.
__device__ __forceinline__ void had_col8(const int16_t* s, int st, int16_t* o) {
  int16_t b[8], c[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    b[2 * k] = (int16_t)(s[2 * k * st] + s[(2 * k + 1) * st]);
    b[2 * k + 1] = (int16_t)(s[2 * k * st] - s[(2 * k + 1) * st]);
  }
  c[0] = (int16_t)(b[0] + b[2]);
  c[1] = (int16_t)(b[1] + b[3]);
  c[2] = (int16_t)(b[0] - b[2]);
  c[3] = (int16_t)(b[1] - b[3]);
  c[4] = (int16_t)(b[4] + b[6]);
  c[5] = (int16_t)(b[5] + b[7]);
  c[6] = (int16_t)(b[4] - b[6]);
  c[7] = (int16_t)(b[5] - b[7]);
  o[0] = (int16_t)(c[0] + c[4]);
  o[7] = (int16_t)(c[1] + c[5]);
  o[3] = (int16_t)(c[2] + c[6]);
  o[4] = (int16_t)(c[3] + c[7]);
  o[2] = (int16_t)(c[0] - c[4]);
  o[6] = (int16_t)(c[1] - c[5]);
  o[1] = (int16_t)(c[2] - c[6]);
  o[5] = (int16_t)(c[3] - c[7]);
}
__device__ __forceinline__ void had_col4(const int16_t* s, int st, int16_t* o) {
  const int16_t b0 = (int16_t)((s[0] + s[st]) >> 1);
  const int16_t b1 = (int16_t)((s[0] - s[st]) >> 1);
  const int16_t b2 = (int16_t)((s[2 * st] + s[3 * st]) >> 1);
  const int16_t b3 = (int16_t)((s[2 * st] - s[3 * st]) >> 1);
  o[0] = (int16_t)(b0 + b2);
  o[1] = (int16_t)(b1 + b3);
  o[2] = (int16_t)(b0 - b2);
  o[3] = (int16_t)(b1 - b3);
}

// second column pass of aom_highbd_hadamard_8x8_c: int16 in, int32 math
__device__ __forceinline__ void had_col8_i32(const int16_t* s, int st, int32_t* o) {
  int32_t b[8], c[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    b[2 * k] = s[2 * k * st] + s[(2 * k + 1) * st];
    b[2 * k + 1] = s[2 * k * st] - s[(2 * k + 1) * st];
  }
  c[0] = b[0] + b[2];
  c[1] = b[1] + b[3];
  c[2] = b[0] - b[2];
  c[3] = b[1] - b[3];
  c[4] = b[4] + b[6];
  c[5] = b[5] + b[7];
  c[6] = b[4] - b[6];
  c[7] = b[5] - b[7];
  o[0] = c[0] + c[4];
  o[7] = c[1] + c[5];
  o[3] = c[2] + c[6];
  o[4] = c[3] + c[7];
  o[2] = c[0] - c[4];
  o[6] = c[1] - c[5];
  o[1] = c[2] - c[6];
  o[5] = c[3] - c[7];
}

// n x n (n = 4, 8) Hadamard of one block by one lane: two column passes.
// lowbd: int16 throughout and a transposed output (aom_hadamard_{4x4,8x8}_c
// "extra transpose"); highbd 8x8: int32 second pass, no transpose.
template <int n, bool HBD>
__device__ __forceinline__ void had_small(const int16_t* src, int st, int32_t* coeff) {
  int16_t b1[n * n];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    if constexpr (n == 4) had_col4(src + i, st, b1 + 4 * i);
    else had_col8(src + i, st, b1 + 8 * i);
  }
  if constexpr (HBD) {
#pragma unroll
    for (int i = 0; i < 8; ++i) had_col8_i32(b1 + i, 8, coeff + 8 * i);
  } else {
    int16_t b2[n * n];
#pragma unroll
    for (int i = 0; i < n; ++i) {
      if constexpr (n == 4) had_col4(b1 + i, 4, b2 + 4 * i);
      else had_col8(b1 + i, 8, b2 + 8 * i);
    }
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
      for (int j = 0; j < n; ++j) coeff[i * n + j] = b2[j * n + i];
  }
}

// jobs: src_off = element offset of the block, aux_off = coefficient offset.
// coeff16 != nullptr: aom_hadamard_lp_8x8 (avg.c:207-236), the lowbd 8x8
// butterflies and transpose stored as int16.
__global__ __launch_bounds__(64) void hadamard_small_kernel(int n, int highbd, const int16_t* src,
                                                            int stride, const LavishPixJob* jobs,
                                                            int njobs, int32_t* coeff,
                                                            int16_t* coeff16) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= njobs) return;
  const LavishPixJob jb = jobs[j];
  int32_t c[64];
  if (n == 4) had_small<4, false>(src + jb.src_off, stride, c);
  else if (highbd) had_small<8, true>(src + jb.src_off, stride, c);
  else had_small<8, false>(src + jb.src_off, stride, c);
  if (coeff16) {
    for (int i = 0; i < n * n; ++i) coeff16[jb.aux_off + i] = (int16_t)c[i];
  } else {
    for (int i = 0; i < n * n; ++i) coeff[jb.aux_off + i] = c[i];
  }
}

// 16x16 / 32x32: one wave per job; 8x8 sub-blocks by lanes into LDS, then the
// combine stages (avg.c:226-348) over all lanes.  coeff16 != nullptr:
// aom_hadamard_lp_16x16 (avg.c:289-316): every combine value truncated to
// int16 and no AVX2 group swap.
__global__ __launch_bounds__(64) void hadamard_big_kernel(int n, int highbd, const int16_t* src,
                                                          int stride, const LavishPixJob* jobs,
                                                          int32_t* coeff, int16_t* coeff16) {
  const bool lp = coeff16 != nullptr;
  __shared__ int32_t c[1024];
  const LavishPixJob jb = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  const int16_t* s = src + jb.src_off;
  // 16x16 quadrant q of the block at (qy, qx) holds 4 8x8 sub-blocks idx
  const int nq = n == 32 ? 4 : 1;
  if (lane < 4 * nq) {
    const int q = lane >> 2, idx = lane & 3;
    const int qy = (q >> 1) * 16, qx = (q & 1) * 16;
    const int16_t* p = s + (int64_t)(qy + (idx >> 1) * 8) * stride + qx + (idx & 1) * 8;
    if (highbd) had_small<8, true>(p, stride, c + q * 256 + idx * 64);
    else had_small<8, false>(p, stride, c + q * 256 + idx * 64);
  }
  __syncthreads();
  for (int q = 0; q < nq; ++q) {
    int32_t* cq = c + q * 256;
    const int i = lane;  // 64 lanes x one column of 4
    const int32_t a0 = cq[i], a1 = cq[64 + i], a2 = cq[128 + i], a3 = cq[192 + i];
    int32_t b0 = (a0 + a1) >> 1, b1 = (a0 - a1) >> 1;
    int32_t b2 = (a2 + a3) >> 1, b3 = (a2 - a3) >> 1;
    if (lp) {
      b0 = (int16_t)b0;
      b1 = (int16_t)b1;
      b2 = (int16_t)b2;
      b3 = (int16_t)b3;
    }
    __syncthreads();
    cq[i] = lp ? (int16_t)(b0 + b2) : b0 + b2;
    cq[64 + i] = lp ? (int16_t)(b1 + b3) : b1 + b3;
    cq[128 + i] = lp ? (int16_t)(b0 - b2) : b0 - b2;
    cq[192 + i] = lp ? (int16_t)(b1 - b3) : b1 - b3;
    __syncthreads();
    // lowbd only: swap of 4-wide groups to match the AVX2 order (avg.c:281-287)
    if (!highbd && !lp) {
      const int row = lane >> 2, jj = lane & 3;
      const int32_t t = cq[row * 16 + 4 + jj];
      const int32_t u = cq[row * 16 + 8 + jj];
      cq[row * 16 + 4 + jj] = u;
      cq[row * 16 + 8 + jj] = t;
    }
    __syncthreads();
  }
  if (n == 32) {
    for (int i = lane; i < 256; i += 64) {
      const int32_t a0 = c[i], a1 = c[256 + i], a2 = c[512 + i], a3 = c[768 + i];
      const int32_t b0 = (a0 + a1) >> 2, b1 = (a0 - a1) >> 2;
      const int32_t b2 = (a2 + a3) >> 2, b3 = (a2 - a3) >> 2;
      c[i] = b0 + b2;
      c[256 + i] = b1 + b3;
      c[512 + i] = b0 - b2;
      c[768 + i] = b1 - b3;
    }
    __syncthreads();
  }
  if (lp) {
    for (int i = lane; i < n * n; i += 64) coeff16[jb.aux_off + i] = (int16_t)c[i];
  } else {
    for (int i = lane; i < n * n; i += 64) coeff[jb.aux_off + i] = c[i];
  }
}

// ---------------------------------------------------------------- SATD ----
__global__ __launch_bounds__(64) void satd_kernel(const int32_t* coeff, int length, int* out) {
  const int32_t* c = coeff + (int64_t)blockIdx.x * length;
  uint32_t acc = 0;
  for (int i = threadIdx.x; i < length; i += 64) acc += (uint32_t)abs(c[i]);
  acc = wave_sum32(acc);
  if (threadIdx.x == 0) out[blockIdx.x] = (int)acc;
}

__global__ __launch_bounds__(64) void satd_lp_kernel(const int16_t* coeff, int length, int* out) {
  const int16_t* c = coeff + (int64_t)blockIdx.x * length;
  uint32_t acc = 0;
  for (int i = threadIdx.x; i < length; i += 64) acc += (uint32_t)abs((int)c[i]);
  acc = wave_sum32(acc);
  if (threadIdx.x == 0) out[blockIdx.x] = (int)acc;
}

// ------------------------------------------------------- sum and sse ----
// (sum, sse) of an int16 block: aom_sum_sse_2d_i16 (sum_squares.c:75-90) and
// aom_get_blk_sse_sum (blk_sse_sum.c:14-27) -- v * v in int, int64 sums
__global__ __launch_bounds__(64) void sum_sse_kernel(const int16_t* src, int stride, int w, int h,
                                                     const LavishPixJob* jobs, int32_t* sum_out,
                                                     int64_t* sse_out) {
  const LavishPixJob jb = jobs[blockIdx.x];
  int64_t ss = 0, sm = 0;
  for (int i = threadIdx.x; i < w * h; i += 64) {
    const int y = i / w, x = i - y * w;
    const int v = src[jb.src_off + (int64_t)y * stride + x];
    ss += v * v;
    sm += v;
  }
  ss = wave_sum64(ss);
  sm = wave_sum64(sm);
  if (threadIdx.x == 0) {
    if (sum_out) sum_out[blockIdx.x] = (int32_t)sm;
    if (sse_out) sse_out[blockIdx.x] = ss;
  }
}

// --------------------------------------------------------- block error ----
// av1_block_error_lp (rdopt.c:650-660): int16 inputs, diff * diff in int
// (wrapping) arithmetic, int64 sum
__global__ __launch_bounds__(64) void block_error_lp_kernel(const int16_t* coeff,
                                                            const int16_t* dqcoeff, int n,
                                                            int64_t* err_out) {
  const int64_t base = (int64_t)blockIdx.x * n;
  int64_t err = 0;
  for (int i = threadIdx.x; i < n; i += 64) {
    const int32_t df = (int32_t)coeff[base + i] - dqcoeff[base + i];
    err += (int32_t)((uint32_t)df * (uint32_t)df);
  }
  err = wave_sum64(err);
  if (threadIdx.x == 0) err_out[blockIdx.x] = err;
}

__global__ __launch_bounds__(64) void block_error_kernel(const int32_t* coeff,
                                                         const int32_t* dqcoeff, int n, int bd,
                                                         int64_t* err_out, int64_t* ssz_out) {
  const int64_t base = (int64_t)blockIdx.x * n;
  int64_t err = 0, sq = 0;
  for (int i = threadIdx.x; i < n; i += 64) {
    const int32_t c = coeff[base + i], d = dqcoeff[base + i];
    if (bd == 0) {  // lowbd: the reference squares in int (wrapping) arithmetic
      const int32_t df = (int32_t)((uint32_t)c - (uint32_t)d);
      err += (int32_t)((uint32_t)df * (uint32_t)df);
      sq += (int32_t)((uint32_t)c * (uint32_t)c);
    } else {
      const int64_t df = (int64_t)c - d;
      err += df * df;
      sq += (int64_t)c * c;
    }
  }
  err = wave_sum64(err);
  sq = wave_sum64(sq);
  if (threadIdx.x == 0) {
    if (bd > 8) {
      const int shift = 2 * (bd - 8);
      const int64_t rnd = (int64_t)1 << (shift - 1);
      err = (err + rnd) >> shift;
      sq = (sq + rnd) >> shift;
    }
    err_out[blockIdx.x] = err;
    ssz_out[blockIdx.x] = sq;
  }
}

}  // namespace lavish

using namespace lavish;

#define LCHK() LAVISH_CHECK(hipGetLastError())

extern "C" {

int lavish_sad_batch(const void* src, int src_stride, const void* ref, int ref_stride, int w,
                     int h, const LavishPixJob* jobs, int njobs, int nrefs, int mode,
                     const void* second_pred, int highbd, uint32_t* sad_out, void* stream) {
  if (njobs <= 0) return 0;
  if (nrefs < 1 || nrefs > 4 || mode < 0 || mode > 2 || (mode == 2 && !second_pred)) return -1;
  hipStream_t s = (hipStream_t)stream;
  U8Shape sh;
  if (!highbd && u8_shape(w, mode == 1 ? h / 2 : h, sh)) {
    const int blocks = (int)(((int64_t)njobs * sh.lpj + 255) / 256);
    hipLaunchKernelGGL(sad_u8_kernel, dim3(blocks), dim3(256), 0, s, (const uint8_t*)src,
                       src_stride, (const uint8_t*)ref, ref_stride, sh, jobs, njobs, nrefs, mode,
                       (const uint8_t*)second_pred, w, sad_out);
    LCHK();
    return 0;
  }
  if (highbd && u16_shape(w, mode == 1 ? h / 2 : h, sh)) {
    const int blocks = (int)(((int64_t)njobs * sh.lpj + 255) / 256);
    hipLaunchKernelGGL(sad_u16_kernel, dim3(blocks), dim3(256), 0, s, (const uint16_t*)src,
                       src_stride, (const uint16_t*)ref, ref_stride, sh, jobs, njobs, nrefs, mode,
                       (const uint16_t*)second_pred, w, sad_out);
    LCHK();
    return 0;
  }
  if (highbd)
    hipLaunchKernelGGL(sad_kernel<uint16_t>, dim3(njobs), dim3(64), 0, s, (const uint16_t*)src,
                       src_stride, (const uint16_t*)ref, ref_stride, w, h, jobs, nrefs, mode,
                       (const uint16_t*)second_pred, sad_out);
  else
    hipLaunchKernelGGL(sad_kernel<uint8_t>, dim3(njobs), dim3(64), 0, s, (const uint8_t*)src,
                       src_stride, (const uint8_t*)ref, ref_stride, w, h, jobs, nrefs, mode,
                       (const uint8_t*)second_pred, sad_out);
  LCHK();
  return 0;
}

int lavish_variance_batch(const void* a, int a_stride, const void* b, int b_stride, int w, int h,
                          const LavishPixJob* jobs, int njobs, int kind, int bit_depth,
                          int highbd, const void* second_pred, uint32_t* var_out, uint32_t* sse_out, int32_t* sum_out,
                          int64_t* sse64_out, void* stream) {
  if (njobs <= 0) return 0;
  if (kind < 0 || kind > 5 || (kind == 5 && !second_pred)) return -1;
  hipStream_t s = (hipStream_t)stream;
  U8Shape sh;
  if (!highbd && kind != 3 && kind != 5 && u8_shape(w, h, sh)) {
    const int blocks = (int)(((int64_t)njobs * sh.lpj + 255) / 256);
    hipLaunchKernelGGL(var_u8_kernel, dim3(blocks), dim3(256), 0, s, (const uint8_t*)a, a_stride,
                       (const uint8_t*)b, b_stride, sh, w, h, jobs, njobs, kind, var_out,
                       sse_out, sum_out, sse64_out);
    LCHK();
    return 0;
  }
  if (highbd && kind != 3 && kind != 5 && u16_shape(w, h, sh)) {
    const int blocks = (int)(((int64_t)njobs * sh.lpj + 255) / 256);
    hipLaunchKernelGGL(var_u16_kernel, dim3(blocks), dim3(256), 0, s, (const uint16_t*)a,
                       a_stride, (const uint16_t*)b, b_stride, sh, w, h, jobs, njobs, kind,
                       bit_depth, var_out, sse_out, sum_out, sse64_out);
    LCHK();
    return 0;
  }
  if (highbd)
    hipLaunchKernelGGL(var_kernel<uint16_t>, dim3(njobs), dim3(64), 0, s, (const uint16_t*)a,
                       a_stride, (const uint16_t*)b, b_stride, w, h, jobs, kind, bit_depth,
                       (const uint16_t*)second_pred, var_out, sse_out, sum_out, sse64_out);
  else
    hipLaunchKernelGGL(var_kernel<uint8_t>, dim3(njobs), dim3(64), 0, s, (const uint8_t*)a,
                       a_stride, (const uint8_t*)b, b_stride, w, h, jobs, kind, 8,
                       (const uint8_t*)second_pred, var_out,
                       sse_out, sum_out, sse64_out);
  LCHK();
  return 0;
}

int lavish_subtract_batch(int rows, int cols, int16_t* diff, int diff_stride, const void* src,
                          int src_stride, const void* pred, int pred_stride,
                          const LavishPixJob* jobs, int njobs, int highbd, void* stream) {
  if (njobs <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (highbd)
    hipLaunchKernelGGL(subtract_kernel<uint16_t>, dim3(njobs), dim3(256), 0, s, rows, cols, diff,
                       diff_stride, (const uint16_t*)src, src_stride, (const uint16_t*)pred,
                       pred_stride, jobs);
  else
    hipLaunchKernelGGL(subtract_kernel<uint8_t>, dim3(njobs), dim3(256), 0, s, rows, cols, diff,
                       diff_stride, (const uint8_t*)src, src_stride, (const uint8_t*)pred,
                       pred_stride, jobs);
  LCHK();
  return 0;
}

int lavish_sum_squares_batch(const int16_t* src, int stride, int w, int h,
                             const LavishPixJob* jobs, int njobs, uint64_t* out, void* stream) {
  if (njobs <= 0) return 0;
  hipLaunchKernelGGL(sum_squares_kernel, dim3(njobs), dim3(64), 0, (hipStream_t)stream, src,
                     stride, w, h, jobs, out);
  LCHK();
  return 0;
}

int lavish_hadamard_batch(int n, int highbd, const int16_t* src_diff, int stride,
                          const LavishPixJob* jobs, int njobs, int32_t* coeff, void* stream) {
  if (njobs <= 0) return 0;
  if (highbd && n == 4) return -1;  // no aom_highbd_hadamard_4x4 in the reference
  hipStream_t s = (hipStream_t)stream;
  if (n == 4 || n == 8)
    hipLaunchKernelGGL(hadamard_small_kernel, dim3((njobs + 63) / 64), dim3(64), 0, s, n, highbd,
                       src_diff, stride, jobs, njobs, coeff, (int16_t*)nullptr);
  else if (n == 16 || n == 32)
    hipLaunchKernelGGL(hadamard_big_kernel, dim3(njobs), dim3(64), 0, s, n, highbd, src_diff,
                       stride, jobs, coeff, (int16_t*)nullptr);
  else
    return -1;
  LCHK();
  return 0;
}

int lavish_hadamard_lp_batch(int n, const int16_t* src_diff, int stride, const LavishPixJob* jobs,
                             int njobs, int16_t* coeff, void* stream) {
  if (njobs <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (n == 8)
    hipLaunchKernelGGL(hadamard_small_kernel, dim3((njobs + 63) / 64), dim3(64), 0, s, 8, 0,
                       src_diff, stride, jobs, njobs, (int32_t*)nullptr, coeff);
  else if (n == 16)
    hipLaunchKernelGGL(hadamard_big_kernel, dim3(njobs), dim3(64), 0, s, 16, 0, src_diff, stride,
                       jobs, (int32_t*)nullptr, coeff);
  else
    return -1;  // the reference has lp forms for 8x8 and 16x16 only
  LCHK();
  return 0;
}

int lavish_satd_lp_batch(const int16_t* coeff, int length, int nblocks, int* out, void* stream) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(satd_lp_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, coeff,
                     length, out);
  LCHK();
  return 0;
}

int lavish_block_error_lp_batch(const int16_t* coeff, const int16_t* dqcoeff, int n, int nblocks,
                                int64_t* err, void* stream) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(block_error_lp_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream,
                     coeff, dqcoeff, n, err);
  LCHK();
  return 0;
}

int lavish_sum_sse_batch(const int16_t* src, int stride, int w, int h, const LavishPixJob* jobs,
                         int njobs, int32_t* sum, int64_t* sse, void* stream) {
  if (njobs <= 0) return 0;
  if (w <= 0 || h <= 0) return -1;
  hipLaunchKernelGGL(sum_sse_kernel, dim3(njobs), dim3(64), 0, (hipStream_t)stream, src, stride,
                     w, h, jobs, sum, sse);
  LCHK();
  return 0;
}

int lavish_satd_batch(const int32_t* coeff, int length, int nblocks, int* out, void* stream) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(satd_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, coeff, length,
                     out);
  LCHK();
  return 0;
}

int lavish_block_error_batch(const int32_t* coeff, const int32_t* dqcoeff, int n, int nblocks,
                             int bit_depth, int64_t* err, int64_t* ssz, void* stream) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(block_error_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, coeff,
                     dqcoeff, n, bit_depth, err, ssz);
  LCHK();
  return 0;
}

}  // extern "C"
