// subpel.hip -- batched sub-pixel motion refinement for gfx950 (SURVEY.md
// 8(f) rank 2).
//
// Reference (one block, one reference, one CPU thread), subpel_search_method
// SUBPEL_TREE_PRUNED_MORE (speed >= 4) or SUBPEL_TREE_PRUNED:
//   av1_find_best_sub_pixel_tree_pruned_more (av1/encoder/mcomp.c:2907-2990)
//   av1_find_best_sub_pixel_tree_pruned (:2992-3126)
//   -> setup_center_error (:2781-2838, vf at the full-pel start)
//   -> with the full-pel search's cost list: get_cost_surf_min (:2870, one
//      check at the modelled minimum when is_cost_list_wellbehaved) for
//      pruned_more, the whichdir quadrant (3 checks) for pruned
//   -> two_level_checks_fast (:2675) per half / quarter / (hp) eighth step:
//      first_level_check_fast (:2566: left, right, up, down, then the
//      diagonal toward the cheaper sides) and, with iters_per_step > 1,
//      second_level_check_fast (:2608)
//   -> check_better_fast (:2496): in-range test, estimated_pref_error =
//      svf = aom_sub_pixel_variance (bilinear, aom_dsp/variance.c:73-145) +
//      mv_err_cost_ (:290-323, entropy / L1 / none), "strictly better"
//      update.
//
// Here one wave64 owns one (block, reference) job.  Every check of a round
// whose candidates are known in advance (the 4 cardinal points, the 2-3
// second-level points) is evaluated at once: each lane owns 4-pixel row
// segments of the block (source words kept in VGPRs), reads the 5 bytes of
// rows y and y+1 it needs per candidate (two dword loads + v_alignbyte
// each), applies the two bilinear passes with the reference's rounding and
// accumulates (sum, sse); wave sums end in SGPRs and the sequential
// check_better_fast updates run on the scalar unit in the reference's order.
//
// SUBPEL_TREE with subpel_search_type USE_4_TAPS / USE_8_TAPS takes the
// upsampled prediction's error instead (check_better -> upsampled_pref_error,
// mcomp.c:2402-2491,2528-2551 -> aom_upsampled_pred_c, reconinter_enc.c:
// 424-496, unscaled): per candidate the 8-tap-layout kernel row of
// av1_get_filter (filter.h:276-285) at phase 2 * q3, aom_convolve8_horiz_c /
// _vert_c (aom_dsp/aom_convolve.c:36-73: round by FILTER_BITS, clip to 8
// bits; the 2-D case filters rows -3 .. +4 horizontally first), then vf.
// Each lane computes its 4-pixel segments' prediction from the 8 x 12 source
// bytes around them.  USE_2_TAPS is the bilinear kernel through the same
// passes, which is the svf's arithmetic exactly (same weights, same rounding,
// no clipping possible): it takes the svf path.
#include "interp_kernels.h"
#include "lavish_internal.h"

namespace lavish {
namespace {

// [kind][phase][tap] (interp_kernels.h): 0 the 8-tap regular, 4 the 4-tap
// regular kernels (av1_get_filter's USE_8_TAPS / USE_4_TAPS)
__constant__ int16_t kUpK[6][16][8] = LAVISH_K8_INIT;

struct SJob {
  int64_t src_off, ref_off;
  int16_t start_row, start_col, ref_mv_row, ref_mv_col;
  int16_t col_min, col_max, row_min, row_max;
};
static_assert(sizeof(SJob) == sizeof(LavishSubpelJob), "job layout");
static_assert(sizeof(LavishSubpelResult) == 16, "result layout");

__constant__ uint8_t kBil2t[8][2] = {{128, 0}, {112, 16}, {96, 32}, {80, 48},
                                     {64, 64}, {48, 80},  {32, 96}, {16, 112}};

__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// 5 consecutive bytes at p as (dword of bytes 0..3, byte 4) from two
// dword-aligned loads
__device__ __forceinline__ void load5(const uint8_t* p, uint32_t& lo, uint32_t& hi) {
  typedef const __attribute__((address_space(1))) uint32_t* gptr;
  const uintptr_t a = (uintptr_t)p;
  const gptr q = (gptr)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t w0 = q[0], w1 = q[1];
  lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
  hi = (sh == 0 ? w1 : (w1 >> (8 * sh))) & 0xFF;
}

template <int W, int H>
struct Sp {
  static constexpr int SEG = W * H / 4;              // 4-pixel row segments
  static constexpr int NSEG = (SEG + 63) / 64;       // segments per lane
  static constexpr int SPR = W / 4;                  // segments per row
  // source words live in VGPRs up to 8 per lane (32x32 and smaller); larger
  // blocks re-read them with the candidate rows
  static constexpr bool kCache = NSEG <= 8;
  static constexpr int NS = kCache ? NSEG : 1;
};

struct SpCtx {
  const uint8_t* src;
  const uint8_t* ref;
  int ss, rs;
  int ref_mv_row, ref_mv_col;
  int col_min, col_max, row_min, row_max;
  int lambda;  // mv_err_cost_ L1 lambda (0: MV_COST_NONE)
  int up_kind;  // -1: the bilinear svf error; else kUpK kind of the upsampled error
  bool entropy;
  int error_per_bit;
  const int32_t* mvjcost;
  const int32_t* mvcost0;  // centred at MV_MAX
  const int32_t* mvcost1;
};

// mv_err_cost_ (mcomp.c:290-323) at a wave-uniform mv
__device__ __forceinline__ int mv_cost(const SpCtx& c, int row, int col) {
  const int dr = row - c.ref_mv_row, dc = col - c.ref_mv_col;
  if (c.entropy) {
    const int joint = (dc != 0) | ((dr != 0) << 1);  // av1_get_mv_joint
    const int rate = c.mvjcost[joint] + c.mvcost0[dr] + c.mvcost1[dc];
    return (int)(((int64_t)rate * c.error_per_bit + 8192) >> 14);
  }
  return (c.lambda * (abs(dr) + abs(dc))) >> 3;
}
__device__ __forceinline__ bool in_range(const SpCtx& c, int row, int col) {
  return col >= c.col_min && col <= c.col_max && row >= c.row_min && row <= c.row_max;
}

__device__ __forceinline__ void seg4(const SpCtx& c, const uint8_t* base, int y, int x,
                                     uint32_t sw, int f0, int f1, int g0, int g1, int& sum,
                                     uint32_t& sse) {
  uint32_t a0, a4, b0, b4;
  load5(base + (int64_t)y * c.rs + x, a0, a4);
  load5(base + (int64_t)(y + 1) * c.rs + x, b0, b4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p0 = (a0 >> (8 * i)) & 0xFF, p1 = i < 3 ? (a0 >> (8 * i + 8)) & 0xFF : a4;
    const int q0 = (b0 >> (8 * i)) & 0xFF, q1 = i < 3 ? (b0 >> (8 * i + 8)) & 0xFF : b4;
    const int h0 = (p0 * f0 + p1 * f1 + 64) >> 7;  // first pass (FILTER_BITS 7)
    const int h1 = (q0 * f0 + q1 * f1 + 64) >> 7;
    const int v = ((h0 * g0 + h1 * g1 + 64) >> 7) & 0xFF;  // second pass -> uint8
    const int d = v - (int)((sw >> (8 * i)) & 0xFF);
    sum += d;
    sse += (uint32_t)(d * d);
  }
}

// 12 consecutive bytes at p as three dwords (dword-aligned loads + alignbyte)
__device__ __forceinline__ void load12(const uint8_t* p, uint32_t (&d)[3]) {
  typedef const __attribute__((address_space(1))) uint32_t* gptr;
  const uintptr_t a = (uintptr_t)p;
  const gptr q = (gptr)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
  d[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
  d[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
  d[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
}
__device__ __forceinline__ int byte_at(const uint32_t (&d)[3], int i) {
  return (d[i >> 2] >> (8 * (i & 3))) & 0xFF;
}
__device__ __forceinline__ int clip8(int v) { return min(max(v, 0), 255); }

// aom_convolve8_horiz of 4 pixels: src bytes p[-3 .. 7]
__device__ __forceinline__ void hconv4(const uint8_t* p, const int (&k)[8], int (&o)[4]) {
  uint32_t d[3];
  load12(p - 3, d);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int sum = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) sum += byte_at(d, i + t) * k[t];
    o[i] = clip8((sum + 64) >> 7);  // ROUND_POWER_OF_TWO(sum, FILTER_BITS), clip_pixel
  }
}

// (sum, sse) of src - upsampled(ref at mv) over this lane's segments
template <int W, int H>
__device__ __noinline__ void seg_err_up(const SpCtx& c, const uint32_t (&sv)[Sp<W, H>::NS],
                                        int lane, int row, int col, int& sum, uint32_t& sse) {
  using S = Sp<W, H>;
  const int sx = col & 7, sy = row & 7;
  int kx[8], ky[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    kx[t] = kUpK[c.up_kind][2 * sx][t];
    ky[t] = kUpK[c.up_kind][2 * sy][t];
  }
  const uint8_t* base = c.ref + (int64_t)(row >> 3) * c.rs + (col >> 3);
  auto segment = [&](int sg, uint32_t sw) {
    const int y = sg / S::SPR, x = 4 * (sg % S::SPR);
    const uint8_t* p = base + (int64_t)y * c.rs + x;
    int v[4];
    if (sx == 0 && sy == 0) {
      uint32_t d[3];
      load12(p, d);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = byte_at(d, i);
    } else if (sy == 0) {
      hconv4(p, kx, v);
    } else if (sx == 0) {
      int acc[4] = {0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        uint32_t d[3];
        load12(p + (int64_t)(t - 3) * c.rs, d);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] += byte_at(d, i) * ky[t];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = clip8((acc[i] + 64) >> 7);
    } else {
      int acc[4] = {0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        int h[4];
        hconv4(p + (int64_t)(t - 3) * c.rs, kx, h);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] += h[i] * ky[t];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = clip8((acc[i] + 64) >> 7);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = v[i] - (int)((sw >> (8 * i)) & 0xFF);
      sum += d;
      sse += (uint32_t)(d * d);
    }
  };
  if constexpr (S::kCache) {
#pragma unroll
    for (int n = 0; n < S::NS; ++n)
      if (lane + 64 * n < S::SEG) segment(lane + 64 * n, sv[n]);
  } else {
#pragma unroll 1
    for (int sg = lane; sg < S::SEG; sg += 64) {
      uint32_t d[3];
      load12(c.src + (int64_t)(sg / S::SPR) * c.ss + 4 * (sg % S::SPR), d);
      segment(sg, d[0]);
    }
  }
}

// (sum, sse) of src - bilinear(ref at mv) over this lane's segments
template <int W, int H>
__device__ __forceinline__ void seg_err(const SpCtx& c, const uint32_t (&sv)[Sp<W, H>::NS],
                                        int lane, int row, int col, int& sum, uint32_t& sse) {
  using S = Sp<W, H>;
  if (c.up_kind >= 0) {
    seg_err_up<W, H>(c, sv, lane, row, col, sum, sse);
    return;
  }
  const int xo = col & 7, yo = row & 7;
  const int f0 = kBil2t[xo][0], f1 = kBil2t[xo][1];
  const int g0 = kBil2t[yo][0], g1 = kBil2t[yo][1];
  const uint8_t* base = c.ref + (int64_t)(row >> 3) * c.rs + (col >> 3);
  if constexpr (S::kCache) {
#pragma unroll
    for (int n = 0; n < S::NS; ++n) {
      const int sg = lane + 64 * n;
      if (sg < S::SEG)
        seg4(c, base, sg / S::SPR, 4 * (sg % S::SPR), sv[n], f0, f1, g0, g1, sum, sse);
    }
  } else {
#pragma unroll 1
    for (int sg = lane; sg < S::SEG; sg += 64) {
      const int y = sg / S::SPR, x = 4 * (sg % S::SPR);
      uint32_t sw, dummy;
      load5(c.src + (int64_t)y * c.ss + x, sw, dummy);
      seg4(c, base, y, x, sw, f0, f1, g0, g1, sum, sse);
    }
  }
}

// divide_and_round (mcomp.c:2853-2855)
__device__ __forceinline__ int div_round(int n, int d) {
  return ((n < 0) ^ (d < 0)) ? ((n - d / 2) / d) : ((n + d / 2) / d);
}

struct Best {
  int row, col;
  uint32_t besterr, sse1;
  int distortion;
};

// evaluate up to 4 candidates (wave-uniform mvs), then the sequential
// check_better_fast updates; returns each candidate's cost (INT_MAX when out
// of range) through cost[]
template <int W, int H, int N>
__device__ __forceinline__ void check_n(const SpCtx& c, const uint32_t (&sv)[Sp<W, H>::NS],
                                        int lane, const int (&r)[N], const int (&cl)[N],
                                        Best& b, uint32_t (&cost)[N]) {
  int sum[N];
  uint32_t sse[N];
  bool ok[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    sum[k] = 0;
    sse[k] = 0;
    ok[k] = in_range(c, r[k], cl[k]);
    if (ok[k]) seg_err<W, H>(c, sv, lane, r[k], cl[k], sum[k], sse[k]);
  }
#pragma unroll
  for (int k = 0; k < N; ++k) {
    cost[k] = 0x7FFFFFFFu;  // INT_MAX
    if (!ok[k]) continue;
    const int ts = (int)wave_total((uint32_t)sum[k]);
    const uint32_t tq = wave_total(sse[k]);
    const uint32_t var = tq - (uint32_t)(((int64_t)ts * ts) / (W * H));
    cost[k] = (uint32_t)mv_cost(c, r[k], cl[k]) + var;
    if (cost[k] < b.besterr) {
      b.besterr = cost[k];
      b.row = r[k];
      b.col = cl[k];
      b.distortion = (int)var;
      b.sse1 = tq;
    }
  }
}

template <int W, int H>
__device__ void two_level(const SpCtx& c, const uint32_t (&sv)[Sp<W, H>::NS], int lane, int tr,
                          int tc, int hstep, int iters, Best& b) {
  uint32_t cst[4];
  {
    const int r[4] = {tr, tr, tr - hstep, tr + hstep};
    const int cl[4] = {tc - hstep, tc + hstep, tc, tc};
    check_n<W, H, 4>(c, sv, lane, r, cl, b, cst);
  }
  // get_best_diag_step: toward the cheaper of up/down and left/right
  const int dr = cst[2] <= cst[3] ? -hstep : hstep;
  const int dc = cst[0] <= cst[1] ? -hstep : hstep;
  uint32_t d1[1];
  {
    const int r[1] = {tr + dr};
    const int cl[1] = {tc + dc};
    check_n<W, H, 1>(c, sv, lane, r, cl, b, d1);
  }
  if (iters <= 1) return;
  const int br = b.row, bc = b.col;
  if (tr != br && tc != bc) {
    const int r[2] = {br, br + dr};
    const int cl[2] = {bc + dc, bc};
    uint32_t d2[2];
    check_n<W, H, 2>(c, sv, lane, r, cl, b, d2);
  } else if (tr == br && tc != bc) {
    const int r[3] = {br + hstep, br - hstep, br - dr};
    const int cl[3] = {bc + dc, bc + dc, bc};
    uint32_t d3[3];
    check_n<W, H, 3>(c, sv, lane, r, cl, b, d3);
  } else if (tr != br && tc == bc) {
    const int r[3] = {br + dr, br + dr, br};
    const int cl[3] = {bc + hstep, bc - hstep, bc - dc};
    uint32_t d3[3];
    check_n<W, H, 3>(c, sv, lane, r, cl, b, d3);
  }
}

// one SUBPEL_TREE level with the bilinear error (USE_2_TAPS_ORIG):
// first_level_check_fast (mcomp.c:2566-2606) around the current best, then
// with iters_per_step > 1 and a moved best second_level_check_v2
// (:2728-2779): row / column bias points away from a losing diagonal, the
// diagonal bias point only when one of them improved
template <int W, int H>
__device__ void tree_level(const SpCtx& c, const uint32_t (&sv)[Sp<W, H>::NS], int lane,
                           int hstep, int iters, Best& b) {
  const int tr = b.row, tc = b.col;
  uint32_t cst[4];
  {
    const int r[4] = {tr, tr, tr - hstep, tr + hstep};
    const int cl[4] = {tc - hstep, tc + hstep, tc, tc};
    check_n<W, H, 4>(c, sv, lane, r, cl, b, cst);
  }
  int dr = cst[2] <= cst[3] ? -hstep : hstep;
  int dc = cst[0] <= cst[1] ? -hstep : hstep;
  uint32_t d1[1];
  {
    const int r[1] = {tr + dr};
    const int cl[1] = {tc + dc};
    check_n<W, H, 1>(c, sv, lane, r, cl, b, d1);
  }
  if (iters <= 1) return;
  const int br = b.row, bc = b.col;
  if (br == tr && bc == tc) return;
  if (tr == br) dr = -dr;
  else if (tc == bc) dc = -dc;
  const uint32_t before = b.besterr;
  {
    const int r[2] = {br + dr, br};
    const int cl[2] = {bc, bc + dc};
    uint32_t d2[2];
    check_n<W, H, 2>(c, sv, lane, r, cl, b, d2);
  }
  if (b.besterr != before) {
    const int r[1] = {br + dr};
    const int cl[1] = {bc + dc};
    check_n<W, H, 1>(c, sv, lane, r, cl, b, d1);
  }
}

template <int W, int H>
__global__ __launch_bounds__(256) void subpel_kernel(const uint8_t* __restrict__ src, int ss,
                                                     const uint8_t* __restrict__ ref, int rs,
                                                     const SJob* __restrict__ jobs, int njobs,
                                                     const LavishDiamondResult* __restrict__ fp,
                                                     int method, int up_kind,
                                                     int forced_stop, int allow_hp,
                                                     int iters, LavishMvCostParams cost,
                                                     const int32_t* __restrict__ cost_lists,
                                                     LavishSubpelResult* out) {
  using S = Sp<W, H>;
  // XCD-aware: consecutive job quads share an XCD's L2
  const int nwg = gridDim.x;  // multiple of 8
  const int wg = (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  const int lane = threadIdx.x & 63;
  const int j = wg * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (j >= njobs) return;
  const SJob jb = jobs[j];
  SpCtx c;
  c.src = src + jb.src_off;
  c.ref = ref + jb.ref_off;
  c.ss = ss;
  c.rs = rs;
  c.ref_mv_row = jb.ref_mv_row;
  c.ref_mv_col = jb.ref_mv_col;
  c.col_min = jb.col_min;
  c.col_max = jb.col_max;
  c.row_min = jb.row_min;
  c.row_max = jb.row_max;
  // mv_err_cost_ lambdas: SSE_LAMBDA_LOWRES 2, MIDRES 0, HDRES 1; NONE 0
  c.lambda = cost.mv_cost_type == 1 ? 2 : cost.mv_cost_type == 3 ? 1 : 0;
  c.up_kind = method == 0 ? up_kind : -1;  // only SUBPEL_TREE takes the upsampled error
  c.entropy = cost.mv_cost_type == 0;
  c.error_per_bit = cost.error_per_bit;
  c.mvjcost = cost.mvjcost;
  c.mvcost0 = cost.mvcost[0];
  c.mvcost1 = cost.mvcost[1];
  // source words of this lane's segments
  uint32_t sv[S::NS];
#pragma unroll
  for (int n = 0; n < S::NS; ++n) {
    const int sg = lane + 64 * n;
    sv[n] = 0;
    if (S::kCache && sg < S::SEG) {
      const int y = sg / S::SPR, x = 4 * (sg % S::SPR);
      uint32_t lo, hi;
      load5(c.src + (int64_t)y * ss + x, lo, hi);
      sv[n] = lo;
    }
  }
  // setup_center_error: vf at the full-pel start (the bilinear passes with
  // zero offsets reproduce the plain pixels exactly)
  // start: the job's, or the full-pel search result of the same job index
  const int start_row = fp ? 8 * fp[j].best_row : jb.start_row;
  const int start_col = fp ? 8 * fp[j].best_col : jb.start_col;
  Best b;
  b.row = start_row;
  b.col = start_col;
  {
    int sum = 0;
    uint32_t sse = 0;
    seg_err<W, H>(c, sv, lane, b.row, b.col, sum, sse);
    const int ts = (int)wave_total((uint32_t)sum);
    const uint32_t tq = wave_total(sse);
    const uint32_t var = tq - (uint32_t)(((int64_t)ts * ts) / (W * H));
    b.distortion = (int)var;
    b.sse1 = tq;
    b.besterr = var + (uint32_t)mv_cost(c, b.row, b.col);
  }
  if (method == 0) {  // av1_find_best_sub_pixel_tree (mcomp.c:3128-3194), no repeat list
    const int round = min(3 - forced_stop, 3 - (allow_hp ? 0 : 1));
    int hstep = 4;
    for (int it = 0; it < round; ++it, hstep >>= 1) tree_level<W, H>(c, sv, lane, hstep, iters, b);
  } else if (forced_stop != 3) {  // FULL_PEL
    int hstep = 4;         // INIT_SUBPEL_STEP_SIZE: half pel
    int cl[5] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX, INT_MAX};
    if (cost_lists) {
#pragma unroll
      for (int i = 0; i < 5; ++i) cl[i] = cost_lists[5 * (int64_t)j + i];
    }
    const bool cl_ok = cl[0] != INT_MAX && cl[1] != INT_MAX && cl[2] != INT_MAX &&
                       cl[3] != INT_MAX && cl[4] != INT_MAX;
    if (method == 2 && cl_ok && cl[0] < cl[1] && cl[0] < cl[2] && cl[0] < cl[3] &&
        cl[0] < cl[4]) {
      // get_cost_surf_min (bits 1): |ic|, |ir| <= 1
      const int ic = div_round(cl[1] - cl[3], cl[1] - 2 * cl[0] + cl[3]);
      const int ir = div_round(cl[4] - cl[2], cl[4] - 2 * cl[0] + cl[2]);
      if (ir != 0 || ic != 0) {
        const int r[1] = {start_row + ir * hstep};
        const int cc[1] = {start_col + ic * hstep};
        uint32_t d1[1];
        check_n<W, H, 1>(c, sv, lane, r, cc, b, d1);
      }
    } else if (method == 1 && cl_ok) {
      // whichdir: left / right by cl[1] < cl[3], bottom / top by cl[2] < cl[4]
      const int dc = cl[1] < cl[3] ? -hstep : hstep;
      const int dr = cl[2] < cl[4] ? hstep : -hstep;
      const int r[3] = {start_row, start_row + dr, start_row + dr};
      const int cc[3] = {start_col + dc, start_col, start_col + dc};
      uint32_t d3[3];
      check_n<W, H, 3>(c, sv, lane, r, cc, b, d3);
    } else {
      two_level<W, H>(c, sv, lane, start_row, start_col, hstep, iters, b);
    }
    if (forced_stop < 2) {  // below HALF_PEL
      hstep >>= 1;
      two_level<W, H>(c, sv, lane, b.row, b.col, hstep, iters, b);
    }
    if (allow_hp && forced_stop == 0) {  // EIGHTH_PEL
      hstep >>= 1;
      two_level<W, H>(c, sv, lane, b.row, b.col, hstep, iters, b);
    }
  }
  if (lane == 0) {
    LavishSubpelResult r;
    r.best_row = (int16_t)b.row;
    r.best_col = (int16_t)b.col;
    r.besterr = b.besterr;
    r.distortion = b.distortion;
    r.sse = b.sse1;
    out[j] = r;
  }
}

template <int W, int H>
void launch(const uint8_t* src, int ss, const uint8_t* ref, int rs, const LavishSubpelJob* jobs,
            int njobs, const LavishDiamondResult* fp, int method, int up_kind, int forced_stop,
            int allow_hp, int iters, const LavishMvCostParams& cost, const int32_t* cost_lists,
            LavishSubpelResult* out, hipStream_t s) {
  int nwg = (njobs + 3) / 4;
  nwg = (nwg + 7) & ~7;
  hipLaunchKernelGGL((subpel_kernel<W, H>), dim3(nwg), dim3(256), 0, s, src, ss, ref, rs,
                     (const SJob*)jobs, njobs, fp, method, up_kind, forced_stop, allow_hp, iters,
                     cost, cost_lists, out);
}

int subpel_batch(const uint8_t* src, int src_stride, const uint8_t* ref, int ref_stride, int w,
                 int h, const LavishSubpelJob* jobs, int njobs, const LavishDiamondResult* fp,
                 int method, int forced_stop, int allow_hp, int iters_per_step,
                 const LavishMvCostParams* cost, const int32_t* cost_lists,
                 LavishSubpelResult* out, hipStream_t s, int search_type = 0) {
  if (njobs <= 0) return 0;
  if (search_type < 0 || search_type > 3) return -7;
  // USE_2_TAPS_ORIG / USE_2_TAPS: the svf; USE_4_TAPS / USE_8_TAPS: kUpK kind
  const int up_kind = search_type == 2 ? 4 : search_type == 3 ? 0 : -1;
  if (forced_stop < 0 || forced_stop > 3) return -1;
  if (cost == nullptr || cost->mv_cost_type < 0 || cost->mv_cost_type > 4) return -2;
  if (cost->mv_cost_type == 0 &&
      (cost->mvjcost == nullptr || cost->mvcost[0] == nullptr || cost->mvcost[1] == nullptr))
    return -2;
  if (iters_per_step < 1 || iters_per_step > 2) return -4;
  if (method < 0 || method > 2) return -6;  // SUBPEL_TREE (bilinear) / _PRUNED / _PRUNED_MORE
#define LAVISH_SP_CASE(W, H)                                                                   \
  if (w == W && h == H) {                                                                      \
    launch<W, H>(src, src_stride, ref, ref_stride, jobs, njobs, fp, method, up_kind,          \
                 forced_stop, allow_hp, iters_per_step, *cost, cost_lists, out, s);            \
    LAVISH_CHECK(hipGetLastError());                                                           \
    return 0;                                                                                  \
  }
  LAVISH_ENCODER_BLOCK_SIZES(LAVISH_SP_CASE)
#undef LAVISH_SP_CASE
  return -3;
}

LavishMvCostParams l1_cost(int mv_cost_type) {
  LavishMvCostParams c = {};
  // the L1 entry points never took MV_COST_ENTROPY (it needs the tables)
  c.mv_cost_type = mv_cost_type == 0 ? -1 : mv_cost_type;
  return c;
}

}  // namespace
}  // namespace lavish

using namespace lavish;

extern "C" int lavish_subpel_search_batch(const uint8_t* src, int src_stride, const uint8_t* ref,
                                          int ref_stride, int w, int h,
                                          const LavishSubpelJob* jobs, int njobs,
                                          int forced_stop, int allow_hp, int iters_per_step,
                                          int mv_cost_type, LavishSubpelResult* out,
                                          void* stream) {
  const LavishMvCostParams c = l1_cost(mv_cost_type);
  return subpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, nullptr, 2,
                      forced_stop, allow_hp, iters_per_step, &c, nullptr, out,
                      (hipStream_t)stream);
}

extern "C" int lavish_subpel_search_after_diamond(const uint8_t* src, int src_stride,
                                                  const uint8_t* ref, int ref_stride, int w,
                                                  int h, const LavishSubpelJob* jobs,
                                                  const LavishDiamondResult* fullpel, int njobs,
                                                  int forced_stop, int allow_hp,
                                                  int iters_per_step, int mv_cost_type,
                                                  LavishSubpelResult* out, void* stream) {
  if (fullpel == nullptr) return -5;
  const LavishMvCostParams c = l1_cost(mv_cost_type);
  return subpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, fullpel, 2,
                      forced_stop, allow_hp, iters_per_step, &c, nullptr, out,
                      (hipStream_t)stream);
}

extern "C" int lavish_find_best_sub_pixel_tree_batch(
    const uint8_t* src, int src_stride, const uint8_t* ref, int ref_stride, int w, int h,
    const LavishSubpelJob* jobs, const LavishDiamondResult* fullpel, int njobs,
    int subpel_search_method, int forced_stop, int allow_hp, int iters_per_step,
    const LavishMvCostParams* cost, const int32_t* cost_lists, LavishSubpelResult* out,
    void* stream) {
  return subpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, fullpel,
                      subpel_search_method, forced_stop, allow_hp, iters_per_step, cost,
                      cost_lists, out, (hipStream_t)stream);
}

extern "C" int lavish_find_best_sub_pixel_tree_batch_ex(
    const uint8_t* src, int src_stride, const uint8_t* ref, int ref_stride, int w, int h,
    const LavishSubpelJob* jobs, const LavishDiamondResult* fullpel, int njobs,
    int subpel_search_method, int subpel_search_type, int forced_stop, int allow_hp,
    int iters_per_step, const LavishMvCostParams* cost, const int32_t* cost_lists,
    LavishSubpelResult* out, void* stream) {
  return subpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, fullpel,
                      subpel_search_method, forced_stop, allow_hp, iters_per_step, cost,
                      cost_lists, out, (hipStream_t)stream, subpel_search_type);
}
