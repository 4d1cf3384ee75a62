// mcomp.hip -- batched DIAMOND full-pixel motion search for gfx950 (C3).
//
// Reference (one block, one reference frame, one CPU thread):
//   av1_full_pixel_search (av1/encoder/mcomp.c:1755-1895, method DIAMOND)
//   -> full_pixel_diamond (:1479-1526) -> diamond_search_sad (:1318-1477)
//   sites of av1_init_dsmotion_compensation (:369-404, level 0: radius
//   1024 >> k, 8 sites per step), mvsad_err_cost / mv_err_cost (:257-360),
//   sdf / sdx4df = aom_sad{W}x{H}[x4d] or the _skip variants when
//   use_downsampled_sad (:132-142) with the quality recheck (:1840-1867),
//   vf = aom_variance{W}x{H}.
//
// Here one wave64 owns one (block, reference) job and runs that sequential
// walk.  A step's 8 candidate sites are evaluated at once: lane group
// g = lane / 8 takes site g + 1, its 8 lanes split the block's rows, each
// lane accumulates v_sad_u8 over 4-byte words (each row one byte-addressed
// 16-byte load), and three DPP adds leave the
// group's SAD in every lane.  Each group then forms the key
// (sad + mvsad_cost) * 8 + site for its site and the wave takes the minimum
// over the 8 groups (8 readlanes + s_min): the reference's sequential
// "strictly better" scan in site order keeps exactly the first site of
// minimal cost (its sad < bestsad prefilter never rejects a site whose cost
// is lower, since the mv cost is >= 0), so the walk and every tie are the
// reference's.  The source block stays in VGPRs for the whole search;
// reference pixels come from L2 / MALL (a 1080p padded reference is ~2.5 MB).
#include <type_traits>

#include <atomic>

#include "lavish_internal.h"
#include "txq_dev.h"

namespace lavish {
namespace {

constexpr int kMaxSteps = 11;  // MAX_MVSEARCH_STEPS (mcomp_structs.h:19)

__device__ __forceinline__ uint32_t sad4(uint32_t a, uint32_t b, uint32_t acc) {
  return __builtin_amdgcn_sad_u8(a, b, acc);
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// DW consecutive 4-byte words starting at an arbitrary byte address.  The
// queues run with unaligned access enabled (SH_MEM_CONFIG alignment mode;
// probed on the box by tools/microbench/unaligned.hip), so one dwordx4 /
// dwordx2 load per 16 / 8 bytes at the byte address returns the row
// directly: one vector-memory instruction per 16-byte row instead of a
// dwordx4 + dword pair and four v_alignbyte.
template <int DW>
__device__ __forceinline__ void load_row(const uint8_t* p, uint32_t (&out)[DW]) {
  // global address space: global_load (not flat: no LDS-aperture check and
  // no lgkmcnt dependency)
  if constexpr (DW % 4 == 0) {
    typedef const __attribute__((address_space(1))) u32x4u* gptr4;
    const gptr4 q = (gptr4)p;
#pragma unroll
    for (int i = 0; i < DW / 4; ++i) {
      const u32x4u v = q[i];
      out[4 * i] = v.x;
      out[4 * i + 1] = v.y;
      out[4 * i + 2] = v.z;
      out[4 * i + 3] = v.w;
    }
  } else if constexpr (DW == 2) {
    typedef const __attribute__((address_space(1))) u32x2u* gptr2;
    const u32x2u v = *(gptr2)p;
    out[0] = v.x;
    out[1] = v.y;
  } else {
    typedef const __attribute__((address_space(1))) u32u* gptr;
#pragma unroll
    for (int i = 0; i < DW; ++i) out[i] = ((gptr)p)[i];
  }
}

// The same DW words from dword-aligned loads (DW words + one more, merged into
// dwordx4 loads) and v_alignbyte: the pattern searches keep this form -- their
// candidates sit a few pixels apart, so a wave's lanes hit the same lines at
// different byte offsets, the shape where byte-addressed 16-byte loads cost
// the address path most (profiles/r02_ta_rate.txt, "grp8"); measured on the
// TPL FAST_BIGDIA leg: 0.191 ms aligned vs 0.218 ms byte-addressed.
template <int DW>
__device__ __forceinline__ void load_row_aligned(const uint8_t* p, uint32_t (&out)[DW]) {
  const uintptr_t a = (uintptr_t)p;
  typedef const __attribute__((address_space(1))) uint32_t* gptr;
  const gptr q = (gptr)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  uint32_t w[DW + 1];
#pragma unroll
  for (int i = 0; i < DW; ++i) w[i] = q[i];
  // the next word only matters when the row is unaligned; an aligned row
  // re-reads its last word instead (no branch, no byte past the row)
  w[DW] = q[sh ? DW : DW - 1];
#pragma unroll
  for (int i = 0; i < DW; ++i) out[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}

// sum over the 8-lane group (every lane of the group gets it): quad_perm
// [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror
__device__ __forceinline__ uint32_t group_sum8(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
  return v;
}

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// Minimum / sum over the 8 lane groups of a value uniform within each group,
// returned as a scalar: row_ror:8 pairs the two groups of a 16-lane row, the
// gfx950 permlane16 / permlane32 swaps the rows -- 3 VALU steps instead of 8
// readlanes and a scalar chain.
__device__ __forceinline__ uint32_t groups_min(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false));
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = min((uint32_t)p[0], (uint32_t)p[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  v = min((uint32_t)q[0], (uint32_t)q[1]);
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint32_t groups_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = (uint32_t)p[0] + (uint32_t)p[1];
  const auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  v = (uint32_t)q[0] + (uint32_t)q[1];
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

struct Job {
  int64_t src_off, ref_off;
  int16_t start_row, start_col, ref_mv_row, ref_mv_col;
  int16_t col_min, col_max, row_min, row_max;
};
static_assert(sizeof(Job) == sizeof(LavishDiamondJob), "job layout");

struct Ctx {
  const uint8_t* src;
  const uint8_t* ref;  // block origin at mv (0,0)
  int ss, rs;
  int col_min, col_max, row_min, row_max;
  int ref_mv_row, ref_mv_col, full_ref_row, full_ref_col;
  int cost_type;
  int sad_lambda, sse_lambda;  // per cost_type, hoisted out of the walk
  int sad_per_bit, error_per_bit;  // MV_COST_ENTROPY
  const int32_t* mvjcost;
  const int32_t* mvcost0;  // centred at MV_MAX
  const int32_t* mvcost1;
  // tiled copy of the reference buffer (LavishRefTiles): the block origin's
  // row / column in the whole buffer, strip-column height, field size
  const uint8_t* tiles;
  int oy, ox, fh, fsz;
};

// byte offset of buffer pixel (y, x) in the tiled copy: field y & 1, strip
// x >> 4 (bytes [16k, 16k + 32) of each field row), field row y >> 1
__device__ __forceinline__ uint32_t tile_off(const Ctx& c, int y, int x) {
  return (uint32_t)((y & 1) * c.fsz) +
         ((uint32_t)(__mul24(x >> 4, c.fh) + (y >> 1)) << 5) + (uint32_t)(x & 15);
}

__device__ const int32_t kZeroRate[1] = {0};

__device__ __forceinline__ int sad_lambda(int t) { return t == 1 ? 32 : t == 2 ? 15 : t == 3 ? 8 : 0; }
__device__ __forceinline__ int sse_lambda(int t) { return t == 1 ? 2 : t == 2 ? 0 : t == 3 ? 1 : 0; }

// mv_cost (mcomp.c:269-273) of a 1/8-pel diff: joint + row + col rates
__device__ __forceinline__ int mv_rate(const Ctx& c, int dr, int dc) {
  const int joint = (dc != 0) | ((dr != 0) << 1);  // av1_get_mv_joint
  return c.mvjcost[joint] + c.mvcost0[dr] + c.mvcost1[dc];
}

// mvsad_err_cost (mcomp.c:329-350); the L1 lambdas are 0 for MV_COST_NONE.
// In two parts so a search step can put the table loads in flight before
// its candidate's SAD load and consume them after (one L2 round trip per
// step, not two): mvsad_rate() issues the three loads -- branch-free: for
// the L1 / none cost types the kernel points the tables at kZeroRate and
// the indices are 0 -- and mvsad_finish() forms the cost.
struct MvRate {
  int32_t j, r, c;
};
__device__ __forceinline__ MvRate mvsad_rate(const Ctx& c, int row, int col) {
  const int dr = (row - c.full_ref_row) * 8, dc = (col - c.full_ref_col) * 8;
  const bool ent = c.cost_type == 0;
  const int joint = ent ? ((dc != 0) | ((dr != 0) << 1)) : 0;  // av1_get_mv_joint
  typedef const __attribute__((address_space(1))) int32_t* gi32;
  return MvRate{((gi32)c.mvjcost)[joint], ((gi32)c.mvcost0)[ent ? dr : 0],
                ((gi32)c.mvcost1)[ent ? dc : 0]};
}
__device__ __forceinline__ uint32_t mvsad_finish(const Ctx& c, const MvRate& m, int row, int col) {
  const int dr = (row - c.full_ref_row) * 8, dc = (col - c.full_ref_col) * 8;
  // ROUND_POWER_OF_TWO(., AV1_PROB_COST_SHIFT); rates < 2^24
  const uint32_t e = (__umul24((uint32_t)(m.j + m.r + m.c), (uint32_t)c.sad_per_bit) + 256u) >> 9;
  const uint32_t l1 = (uint32_t)((c.sad_lambda * (abs(dr) + abs(dc))) >> 3);
  return c.cost_type == 0 ? e : l1;
}
__device__ __forceinline__ uint32_t mvsad_cost(const Ctx& c, int row, int col) {
  return mvsad_finish(c, mvsad_rate(c, row, col), row, col);
}
// mv_err_cost (mcomp.c:290-314)
__device__ __forceinline__ int mv_cost(const Ctx& c, int row, int col) {
  const int dr = row * 8 - c.ref_mv_row, dc = col * 8 - c.ref_mv_col;
  if (c.cost_type == 0)  // RDDIV_BITS + AV1_PROB_COST_SHIFT - RD_EPB_SHIFT + 4 = 14
    return (int)(((int64_t)mv_rate(c, dr, dc) * c.error_per_bit + 8192) >> 14);
  return (c.sse_lambda * (abs(dr) + abs(dc))) >> 3;
}

// Row split of a block inside one 8-lane group.
template <int W, int H, bool SKIP>
struct Geo {
  static constexpr int RH = SKIP ? H / 2 : H;        // rows the SAD reads
  static constexpr int RPL = RH >= 8 ? RH / 8 : 1;   // rows per lane
  static constexpr int DW = W / 4;                   // words per row
  static constexpr int YS = SKIP ? 2 : 1;            // row step
};

// vf (aom_variance{W}x{H}) + mv_err_cost at a full-pel mv, in two parts:
// per-lane (sum, sse) of src/ref words, then the wave reduction.
__device__ __forceinline__ void var_acc(uint32_t a, uint32_t b, int& sum, uint32_t& sse) {
  sum += (int)sad4(a, 0, 0) - (int)sad4(b, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = (int)((a >> (8 * j)) & 255) - (int)((b >> (8 * j)) & 255);
    sse += (uint32_t)(d * d);
  }
}

template <int W, int H>
__device__ __forceinline__ int var_finish(const Ctx& c, int sum, uint32_t sse, int row, int col,
                                          uint32_t* vout = nullptr) {
  const uint32_t ts = groups_sum(group_sum8((uint32_t)sum)), tq = groups_sum(group_sum8(sse));
  const uint32_t var = tq - (uint32_t)(((int64_t)(int)ts * (int)ts) / (W * H));
  if (vout) *vout = var;
  return (int)var + mv_cost(c, row, col);
}

// the whole wave walks the W*H pixels one word per lane, from global memory
template <int W, int H>
__device__ int var_cost(const Ctx& c, int lane, int row, int col, uint32_t* vout = nullptr) {
  constexpr int DW = W / 4;
  int sum = 0;
  uint32_t sse = 0;
  const uint8_t* rb = c.ref + (int64_t)row * c.rs + col;
  for (int i = lane; i < H * DW; i += 64) {
    const int y = i / DW, x = i - y * DW;
    uint32_t a[1], b[1];
    load_row<1>(c.src + (int64_t)y * c.ss + 4 * x, a);
    load_row<1>(rb + (int64_t)y * c.rs + 4 * x, b);
    var_acc(a[0], b[0], sum, sse);
  }
  return var_finish<W, H>(c, sum, sse, row, col, vout);
}

// sdf and sdsf (aom_sad / aom_sad_skip) at a full-pel mv in one pass: the
// whole wave walks the block one word per lane; the skip SAD is twice the
// SAD of the even rows
template <int W, int H>
__device__ void sad_and_skip(const Ctx& c, int lane, int row, int col, int& sad, int& ssad) {
  constexpr int DW = W / 4;
  uint32_t all = 0, even = 0;
  const uint8_t* rb = c.ref + (int64_t)row * c.rs + col;
  for (int i = lane; i < H * DW; i += 64) {
    const int y = i / DW, x = i - y * DW;
    uint32_t a[1], b[1];
    load_row<1>(c.src + (int64_t)y * c.ss + 4 * x, a);
    load_row<1>(rb + (int64_t)y * c.rs + 4 * x, b);
    const uint32_t d = sad4(a[0], b[0], 0);
    all += d;
    even += (y & 1) ? 0u : d;
  }
  const uint32_t ta = groups_sum(group_sum8(all)), te = groups_sum(group_sum8(even));
  sad = (int)ta;
  ssad = (int)(2 * te);
}

// sdf (full-row SAD) of a 16x16 block at up to 4 full-pel positions (r[k],
// cc[k]) for k in [from, to): one source word and four reference words per
// lane, every load in flight before the first SAD (a call per position
// waited one memory latency each)
__device__ __forceinline__ void sad16_multi(const Ctx& c, int lane, const int (&r)[4],
                                            const int (&cc)[4], int from, int to, int (&out)[4]) {
  const int y = lane >> 2, x = 4 * (lane & 3);
  uint32_t sa[1], rb[4][1];
  load_row<1>(c.src + (int64_t)y * c.ss + x, sa);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = min(max(k, from), to - 1);  // (surplus slots repeat a valid position)
    const int rr = k == kk ? r[k] : (kk == 0 ? r[0] : kk == 1 ? r[1] : kk == 2 ? r[2] : r[3]);
    const int cq = k == kk ? cc[k] : (kk == 0 ? cc[0] : kk == 1 ? cc[1] : kk == 2 ? cc[2] : cc[3]);
    load_row<1>(c.ref + (int64_t)(rr + y) * c.rs + cq + x, rb[k]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t t = groups_sum(group_sum8(sad4(sa[0], rb[k][0], 0)));
    if (k >= from && k < to) out[k] = (int)t;
  }
}

// sad16_multi in two halves: the loads (a caller can issue them before a
// wait and use them after it), then the SADs
struct Sad16Loads {
  uint32_t sa, rb[4];
};
__device__ __forceinline__ Sad16Loads sad16_load(const Ctx& c, int lane, const int (&r)[4],
                                                 const int (&cc)[4], int from, int to) {
  const int y = lane >> 2, x = 4 * (lane & 3);
  Sad16Loads L;
  uint32_t t[1];
  load_row<1>(c.src + (int64_t)y * c.ss + x, t);
  L.sa = t[0];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = min(max(k, from), to - 1);
    const int rr = k == kk ? r[k] : (kk == 0 ? r[0] : kk == 1 ? r[1] : kk == 2 ? r[2] : r[3]);
    const int cq = k == kk ? cc[k] : (kk == 0 ? cc[0] : kk == 1 ? cc[1] : kk == 2 ? cc[2] : cc[3]);
    load_row<1>(c.ref + (int64_t)(rr + y) * c.rs + cq + x, t);
    L.rb[k] = t[0];
  }
  return L;
}
__device__ __forceinline__ void sad16_finish(const Sad16Loads& L, int from, int to,
                                             int (&out)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t t = groups_sum(group_sum8(sad4(L.sa, L.rb[k], 0)));
    if (k >= from && k < to) out[k] = (int)t;
  }
}

typedef __attribute__((address_space(3))) uint32_t* lds_u32;
typedef __attribute__((address_space(3))) uint8_t* lds_u8;

// LDS window of the reference for the small-radius tail of a search: once the
// radius drops to <= 8 the walk can move at most 8+4+2+1 = 15 pixels, so every
// later candidate lies in (H + 30) x (W + 30) pixels around the centre at that
// point.  The wave copies that window once (whole rows: one cache line access
// per row instead of one per candidate row per step) and the remaining steps
// read their candidates from LDS.
template <int W, int H>
struct Win {
  static constexpr int R = 15;                  // displacement bound after the fill
  static constexpr int MAXRAD = 8;              // fill at the first step with rad <= 8
  static constexpr bool kOn = W <= 32 && H <= 32;
  static constexpr int ROWS = H + 2 * R;
  // dwords per row: W + 30 bytes + misalignment, filled by 16-byte loads
  static constexpr int Q = (W + 2 * R + 3 + 15) / 16;
  static constexpr int DW = 4 * Q;
  static constexpr int SIZE = kOn ? ROWS * DW : 1;
};

// diamond site i + 1 (i = 0..7) of av1_init_dsmotion_compensation in units
// of the radius: (-1,0) (1,0) (0,-1) (0,1) (-1,-1) (1,1) (-1,1) (1,-1),
// packed as 2-bit (d + 1) fields
__device__ __forceinline__ int site_dr(int i) { return ((0x8858 >> (2 * i)) & 3) - 1; }
__device__ __forceinline__ int site_dc(int i) { return ((0x2885 >> (2 * i)) & 3) - 1; }

// av1_init_motion_compensation_nstep (mcomp.c:452-494): radius of step st
// (1, 2, 3, 5, 8, 12, 18, 27, 41, 62, 93, 140, then 210: the radius grows
// to max((int)(1.5 r + 0.5), r + 1) after each of the first 12 stages) and
// the step count (NSTEP 15, NSTEP_8PT 16)
__device__ __forceinline__ int nstep_radius(int st) {
  constexpr uint32_t kLo[4] = {0x05030201u, 0x1b120c08u, 0x8c5d3e29u, 0xd2d2d2d2u};
  const int w = st >> 2, b = (st & 3) * 8;
  const uint32_t v = w == 0 ? kLo[0] : w == 1 ? kLo[1] : w == 2 ? kLo[2] : kLo[3];
  return (int)((v >> b) & 0xFF);
}
// tan_radius = max((int)(0.41 * r), 1) of the 12-point steps (r > 5; in
// double, as the reference computes it: 3, 4, 7, 11, 16, 25, 38, 57, 86)
__device__ __forceinline__ int nstep_tan(int st) {
  const int w = st >> 2, b = (st & 3) * 8;  // (st 0..3: 8-point steps, unused)
  const uint32_t v = w == 1 ? 0x0b070403u : w == 2 ? 0x39261910u : w == 3 ? 0x56565656u : 0u;
  return (int)((v >> b) & 0xFF);
}
__device__ __forceinline__ int nstep_steps(int level) { return level > 0 ? 16 : 15; }
// site i + 1 (i = 0..11) at radius r, tangent t: (-r,0) (r,0) (0,-r) (0,r)
// (-r,-t) (r,t) (-t,r) (t,-r) (-r,t) (r,-t) (t,r) (-t,-r)
__device__ __forceinline__ void nstep_site(int i, int r, int t, int& dr, int& dc) {
  // per site: row and column as (sign, r-or-t) codes, 3 bits each: 0 zero,
  // 1 +r, 2 -r, 3 +t, 4 -t
  constexpr uint64_t kR = 0x0ull | (2ull << 0) | (1ull << 3) | (0ull << 6) | (0ull << 9) |
                          (2ull << 12) | (1ull << 15) | (4ull << 18) | (3ull << 21) |
                          (2ull << 24) | (1ull << 27) | (3ull << 30) | (4ull << 33);
  constexpr uint64_t kC = 0x0ull | (0ull << 0) | (0ull << 3) | (2ull << 6) | (1ull << 9) |
                          (4ull << 12) | (3ull << 15) | (1ull << 18) | (2ull << 21) |
                          (3ull << 24) | (4ull << 27) | (1ull << 30) | (2ull << 33);
  const int a = (int)((kR >> (3 * i)) & 7), b = (int)((kC >> (3 * i)) & 7);
  auto val = [&](int code) {
    return code == 1 ? r : code == 2 ? -r : code == 3 ? t : code == 4 ? -t : 0;
  };
  dr = val(a);
  dc = val(b);
}

// UA: candidate rows as byte-addressed loads (DIAMOND: its global-memory
// steps are the large-radius ones) or aligned loads + v_alignbyte (the
// pattern searches, see load_row_aligned).  TL: candidate rows from the
// tiled copy (c.tiles), byte-addressed inside one 32-byte strip row.
template <int W, int H, bool SKIP, bool UA = true, bool TL = false>
struct Search {
  static_assert(!TL || W <= 16, "tiled candidate rows: w <= 16");
  using G = Geo<W, H, SKIP>;
  using WN = Win<W, H>;
  // source rows live in VGPRs up to 32 words per lane (32x32 and smaller);
  // larger blocks re-read them through L2 with the candidate rows
  static constexpr bool kCache = G::RPL * G::DW <= 32;
  uint32_t s[kCache ? G::RPL : 1][kCache ? G::DW : 1];
  // source words of the variance (one per lane per 64 words), for the
  // window-served var cost
  static constexpr int VN = (H * (W / 4) + 63) / 64;
  static constexpr bool kVarWin = WN::kOn && VN <= 4;
  uint32_t sv[kVarWin ? VN : 1];
  bool inwin;               // the last diamond() ended inside its window
  bool wfilled;             // win holds the window at (wr0, wc0)
  // every diamond_search_sad run of a full_pixel_diamond starts at the same
  // clamped start_mv: its SAD is read once
  bool have_c0;
  int c0row, c0col;
  uint32_t c0sad;
  int l;  // lane within the group
  lds_u32 win;              // this wave's window (WN::SIZE dwords), or null
  int wr0, wc0;             // window origin (mv units: block top-left at ref + wr0*rs + wc0)
  uintptr_t wbase;          // byte address of the window origin

  __device__ __forceinline__ void load_src(const Ctx& c, int lane, lds_u32 w = nullptr) {
    l = lane & 7;
    win = w;
    inwin = false;
    wfilled = false;
    have_c0 = false;
    if constexpr (kVarWin) {
#pragma unroll
      for (int v = 0; v < VN; ++v) {
        const int i = lane + 64 * v;
        if (i < H * (W / 4)) {
          uint32_t t[1];
          load_row<1>(c.src + (int64_t)(i / (W / 4)) * c.ss + 4 * (i % (W / 4)), t);
          sv[v] = t[0];
        }
      }
    }
    if constexpr (kCache) {
#pragma unroll
      for (int k = 0; k < G::RPL; ++k) {
        const int row = l + 8 * k;
        if (row < G::RH) load_row<G::DW>(c.src + (int64_t)row * G::YS * c.ss, s[k]);
      }
    }
  }

  // group-partial SAD of the candidate at mv (r, cc), reduced over the 8
  // lanes.  Lanes whose candidate is not valid read the block at (sr, sc)
  // (in range) instead: no divergent branch around the loads; callers mask
  // the result.
  __device__ __forceinline__ uint32_t group_sad(const Ctx& c, int r, int cc, bool valid, int sr,
                                                int sc) const {
    r = valid ? r : sr;
    cc = valid ? cc : sc;
    const int64_t off = (int64_t)__mul24(r, c.rs) + cc;
    uint32_t acc = 0;
    if constexpr (TL) {
      // lane l's rows: field rows (oy + r + row * YS) of strip (ox + cc) >> 4;
      // with the downsampled SAD a group's 8 rows are consecutive rows of one
      // field: 256 contiguous bytes (2-3 cache lines) per candidate
      const int x = c.ox + cc;
#pragma unroll
      for (int k = 0; k < G::RPL; ++k) {
        const int row = l + 8 * k;
        if (row < G::RH) {
          uint32_t t[G::DW];
          load_row<G::DW>(c.tiles + tile_off(c, c.oy + r + row * G::YS, x), t);
#pragma unroll
          for (int i = 0; i < G::DW; ++i) acc = sad4(s[k][i], t[i], acc);
        }
      }
    } else if constexpr (kCache) {
#pragma unroll
      for (int k = 0; k < G::RPL; ++k) {
        const int row = l + 8 * k;
        if (row < G::RH) {
          uint32_t r[G::DW];
          if constexpr (UA) load_row<G::DW>(c.ref + off + (int64_t)row * G::YS * c.rs, r);
          else load_row_aligned<G::DW>(c.ref + off + (int64_t)row * G::YS * c.rs, r);
#pragma unroll
          for (int i = 0; i < G::DW; ++i) acc = sad4(s[k][i], r[i], acc);
        }
      }
    } else {
      // rows in 32-byte chunks, not unrolled (keeps code and VGPRs small)
      constexpr int CH = G::DW < 8 ? G::DW : 8;
#pragma unroll 1
      for (int k = 0; k < G::RPL; ++k) {
        const int row = l + 8 * k;
        const uint8_t* rp = c.ref + off + (int64_t)row * G::YS * c.rs;
        const uint8_t* sp = c.src + (int64_t)row * G::YS * c.ss;
#pragma unroll 1
        for (int x = 0; x < G::DW; x += CH) {
          uint32_t r[CH], q[CH];
          load_row<CH>(rp + 4 * x, r);
          load_row<CH>(sp + 4 * x, q);
#pragma unroll
          for (int i = 0; i < CH; ++i) acc = sad4(q[i], r[i], acc);
        }
      }
    }
    acc = group_sum8(acc);
    return SKIP ? 2 * acc : acc;
  }
  __device__ __forceinline__ uint32_t group_sad(const Ctx& c, int r, int cc) const {
    return group_sad(c, r, cc, true, r, cc);
  }

  // copy the window around (row, col): rows outside [row_min, row_max + H)
  // (never touched by a valid candidate) repeat the nearest row inside; all
  // loads are issued before the first store
  static constexpr int kFillN = WN::ROWS * WN::Q, kFillNI = (kFillN + 63) / 64;
  typedef uint32_t fill_v __attribute__((ext_vector_type(4)));
  // fill() in two halves, so a caller can keep several windows' loads in
  // flight: the loads (and the window origin), then the LDS stores
  __device__ __forceinline__ void fill_load(const Ctx& c, int lane, int row, int col,
                                            fill_v (&v)[kFillNI]) {
    typedef const __attribute__((address_space(1))) uint32_t* gptr;
    wr0 = row - WN::R;
    wc0 = col - WN::R;
    wbase = (uintptr_t)(c.ref + (int64_t)wr0 * c.rs + wc0);
    const int rlo = max(0, c.row_min - wr0), rhi = min(WN::ROWS, c.row_max + H - wr0);
#pragma unroll
    for (int it = 0; it < kFillNI; ++it) {
      const int i = min(64 * it + lane, kFillN - 1);
      const int wr = i / WN::Q, d = i - wr * WN::Q;
      const int sr = min(max(wr, rlo), rhi - 1);
      // dword-aligned 16-byte load (any dword alignment is a single access)
      const uintptr_t ra = ((wbase + (int64_t)sr * c.rs) & ~(uintptr_t)3) + 16 * d;
      const gptr q = (gptr)ra;
      v[it] = fill_v{q[0], q[1], q[2], q[3]};
    }
  }
  __device__ __forceinline__ void fill_store(int lane, const fill_v (&v)[kFillNI]) const {
    typedef __attribute__((address_space(3))) fill_v* lptr4;
#pragma unroll
    for (int it = 0; it < kFillNI; ++it) {
      const int i = 64 * it + lane;
      if (i < kFillN) ((lptr4)win)[i] = v[it];
    }
  }
  __device__ __forceinline__ void fill(const Ctx& c, int lane, int row, int col) {
    fill_v v[kFillNI];
    fill_load(c, lane, row, col, v);
    fill_store(lane, v);
    wave_sync();
  }

  // group SAD of the candidate at (r, cc) from the window
  // (lanes whose candidate is not valid read the window centre instead)
  __device__ __forceinline__ uint32_t group_sad_win(const Ctx& c, int r, int cc,
                                                    bool valid) const {
    r = valid ? r : wr0 + WN::R;
    cc = valid ? cc : wc0 + WN::R;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < G::RPL; ++k) {
      const int row = l + 8 * k;
      if (row < G::RH) {
        const int wr = r - wr0 + row * G::YS;  // >= 0
        const int x = cc - wc0 + (int)(((uint32_t)wbase + __umul24(wr, c.rs & 3)) & 3);
        // byte-addressed (unaligned) LDS reads, 16 / 8 / 4 bytes at a time
        const lds_u8 p = (lds_u8)win + (wr * WN::DW * 4 + x);
        uint32_t w[G::DW];
        if constexpr (G::DW % 4 == 0) {
#pragma unroll
          for (int i = 0; i < G::DW / 4; ++i) {
            const u32x4u v = ((const __attribute__((address_space(3))) u32x4u*)p)[i];
            w[4 * i] = v.x;
            w[4 * i + 1] = v.y;
            w[4 * i + 2] = v.z;
            w[4 * i + 3] = v.w;
          }
        } else if constexpr (G::DW == 2) {
          const u32x2u v = *(const __attribute__((address_space(3))) u32x2u*)p;
          w[0] = v.x;
          w[1] = v.y;
        } else {
          w[0] = *(const __attribute__((address_space(3))) u32u*)p;
        }
#pragma unroll
        for (int i = 0; i < G::DW; ++i) acc = sad4(s[k][i], w[i], acc);
      }
    }
    acc = group_sum8(acc);
    return SKIP ? 2 * acc : acc;
  }

  // var cost at (row, col): from the window when the last search filled one
  // (its result lies within 15 pixels of the fill centre)
  __device__ __forceinline__ int var_cost_at(const Ctx& c, int lane, int row, int col,
                                             uint32_t* vout = nullptr) const {
    if constexpr (kVarWin) {
      if (inwin) {
        int sum = 0;
        uint32_t sse = 0;
#pragma unroll
        for (int v = 0; v < VN; ++v) {
          const int i = lane + 64 * v;
          if (i < H * (W / 4)) {
            const int y = i / (W / 4), x4 = i % (W / 4);
            const int wr = row - wr0 + y;
            const int xb = col - wc0 + 4 * x4 + (int)(((uint32_t)wbase + __umul24(wr, c.rs & 3)) & 3);
            const lds_u8 p = (lds_u8)win + (wr * WN::DW * 4 + xb);
            var_acc(sv[v], *(const __attribute__((address_space(3))) u32u*)p, sum, sse);
          }
        }
        return var_finish<W, H>(c, sum, sse, row, col, vout);
      }
    }
    return var_cost<W, H>(c, lane, row, col, vout);
  }

  // diamond_search_sad (no second_pred): returns bestsad
  __device__ __forceinline__ uint32_t diamond(const Ctx& c, int lane, int srow, int scol,
                                              int search_step, int& brow, int& bcol,
                                              int& num00, int& steps) {
    const int g = lane >> 3;
    // site g + 1 of av1_init_dsmotion_compensation (row, col) in units of radius
    const int sdr = site_dr(g), sdc = site_dc(g);
    srow = min(max(srow, c.row_min), c.row_max);
    scol = min(max(scol, c.col_min), c.col_max);
    int row = srow, col = scol, off_center = 0, center = 0;
    if (!have_c0 || c0row != srow || c0col != scol) {
      c0sad = rdlane(group_sad(c, srow, scol), 0);
      have_c0 = true;
      c0row = srow;
      c0col = scol;
    }
    uint32_t best = mvsad_cost(c, row, col) + c0sad;
    const int tot = kMaxSteps - search_step;
    inwin = false;
    // one step: the 8 sites at radius rad around (row, col), straight-line
    // (the candidate's SAD load and the mv-cost table loads issue together)
    auto step_at = [&](int rad, auto win_tag) {
      constexpr bool INW = decltype(win_tag)::value;
      // (all_in of the reference only skips this test when it holds)
      const int r = row + sdr * rad, cc = col + sdc * rad;
      const bool valid = cc >= c.col_min && cc <= c.col_max && r >= c.row_min && r <= c.row_max;
      // the mv-cost table loads first, consumed after the SAD: both L2
      // round trips overlap (|r|, |cc| < 2048 keep every index inside the
      // cost tables, valid or not)
      const MvRate mr = mvsad_rate(c, r, cc);
      uint32_t mine;
      if constexpr (INW) mine = group_sad_win(c, r, cc, valid);
      else mine = group_sad(c, r, cc, valid, row, col);
      const uint32_t mvs = mvsad_finish(c, mr, r, cc);
      // key = cost * 8 + site (costs < 2^26 for blocks <= 128x128); ~0 for
      // an invalid site -- an OR, not a select, so the cost (and its loads)
      // is computed unconditionally, in the SAD's basic block
      const uint32_t key = (((mine + mvs) << 3) | (uint32_t)g) | (valid ? 0u : ~0u);
      const uint32_t kmin = groups_min(key);
      ++steps;
      if (kmin < (best << 3)) {
        best = kmin >> 3;
        const int i = (int)(kmin & 7);
        row += site_dr(i) * rad;
        col += site_dc(i) * rad;
        off_center = 1;
      }
      if (!off_center) ++center;
    };
    int step = tot - 1;
    constexpr bool kWin = WN::kOn && kCache;
    // large radii: candidates from global memory (L2)
    for (; step >= 0 && (!kWin || win == nullptr || (1 << step) > WN::MAXRAD); --step)
      step_at(1 << step, std::false_type{});
    if constexpr (kWin) {
      if (step >= 0) {
        // radius <= 8: the walk stays inside the LDS window around (row, col)
        // (a later run reaching radius 8 at the same point finds its window)
        if (!wfilled || wr0 != row - WN::R || wc0 != col - WN::R) fill(c, lane, row, col);
        wfilled = true;
        inwin = true;
        for (; step >= 0; --step) step_at(1 << step, std::true_type{});
      }
    }
    brow = row;
    bcol = col;
    num00 = center;
    return best;
  }

  // diamond_search_sad over the site configuration of
  // av1_init_motion_compensation_nstep (mcomp.c:452-494; level 0: NSTEP, 15
  // steps, 12 points once the radius passes 5; level 1: NSTEP_8PT, 16 steps
  // of 8 points), candidates from global memory.  12 points take two rounds
  // (sites 1..8, then 9..12); key = cost * 16 + site index, so the minimum
  // over both rounds is the reference's sequential strict-< scan.  The steps
  // of an equal radius below an unmoved step are skipped and counted as
  // centre steps (UPDATE_SEARCH_STEP, mcomp.c:1334-1341).
  __device__ __forceinline__ uint32_t nstep_diamond(const Ctx& c, int lane, int level, int srow,
                                                    int scol, int search_step, int& brow,
                                                    int& bcol, int& num00, int& steps) {
    const int g = lane >> 3;
    srow = min(max(srow, c.row_min), c.row_max);
    scol = min(max(scol, c.col_min), c.col_max);
    int row = srow, col = scol, off_center = 0, center = 0;
    if (!have_c0 || c0row != srow || c0col != scol) {
      c0sad = rdlane(group_sad(c, srow, scol), 0);
      have_c0 = true;
      c0row = srow;
      c0col = scol;
    }
    uint32_t best = mvsad_cost(c, row, col) + c0sad;
    const int tot = nstep_steps(level) - search_step;
    inwin = false;
    // one round: site (first + g) of the step at radius rad / tangent tan
    auto round = [&](int rad, int tan, int first, int cnt) -> uint32_t {
      const int i = first + g;  // 0-based site index (site i + 1)
      int dr, dc;
      nstep_site(i, rad, tan, dr, dc);
      const int r = row + dr, cc = col + dc;
      const bool valid = g < cnt && cc >= c.col_min && cc <= c.col_max && r >= c.row_min &&
                         r <= c.row_max;
      const MvRate mr = mvsad_rate(c, r, cc);
      const uint32_t mine = group_sad(c, r, cc, valid, row, col);
      const uint32_t mvs = mvsad_finish(c, mr, r, cc);
      return groups_min((((mine + mvs) << 4) | (uint32_t)i) | (valid ? 0u : ~0u));
    };
    for (int step = tot - 1; step >= 0; --step) {
      const int rad = nstep_radius(step);
      const int npts = (rad <= 5 || level > 0) ? 8 : 12;
      const int tan = npts == 8 ? rad : nstep_tan(step);
      uint32_t kmin = round(rad, tan, 0, 8);
      if (npts == 12) kmin = min(kmin, round(rad, tan, 8, 4));
      ++steps;
      bool moved = false;
      if (kmin < (best << 4)) {
        best = kmin >> 4;
        int dr, dc;
        nstep_site((int)(kmin & 15), rad, tan, dr, dc);
        row += dr;
        col += dc;
        off_center = 1;
        moved = true;
      }
      if (!off_center) ++center;
      if (!moved && step > 2) {
        while (nstep_radius(step - 1) == rad && step > 2) {
          ++center;
          --step;
        }
      }
    }
    brow = row;
    bcol = col;
    num00 = center;
    return best;
  }
};

// cl[i] = v for a wave-uniform but dynamic i, without a private-array index
__device__ __forceinline__ void set_cl(int (&cl)[5], int i, int v) {
#pragma unroll
  for (int t = 0; t < 5; ++t) cl[t] = i == t ? v : cl[t];
}

// calc_int_sad_list (mcomp.c:789-841): cost list around (br, bc) -- centre,
// left, bottom, right, top -- raw SADs (recomputed unless the pattern search
// left them in cl) plus mvsad_err_cost; INT_MAX for out-of-range neighbours.
// Groups 0..4 evaluate the five points at once.
template <class S_t>
__device__ void int_sad_list(const S_t& S, const Ctx& c, int lane, int br, int bc,
                             bool has_sad, int (&cl)[5]) {
  const int g = lane >> 3;
  if (!has_sad) {
    const int dr = g == 2 ? 1 : g == 4 ? -1 : 0;
    const int dc = g == 1 ? -1 : g == 3 ? 1 : 0;
    const int r = br + dr, cc = bc + dc;
    // (check_bounds of the reference only skips this test when it holds)
    const bool valid =
        g < 5 && cc >= c.col_min && cc <= c.col_max && r >= c.row_min && r <= c.row_max;
    const uint32_t sad = S.group_sad(c, r, cc, valid, br, bc);
    const uint32_t v = valid ? sad : 0x7FFFFFFFu;
#pragma unroll
    for (int i = 0; i < 5; ++i) cl[i] = (int)rdlane(v, 8 * i);
  }
  cl[0] += (int)mvsad_cost(c, br, bc);
  if (cl[1] != INT_MAX) cl[1] += (int)mvsad_cost(c, br, bc - 1);
  if (cl[2] != INT_MAX) cl[2] += (int)mvsad_cost(c, br + 1, bc);
  if (cl[3] != INT_MAX) cl[3] += (int)mvsad_cost(c, br, bc + 1);
  if (cl[4] != INT_MAX) cl[4] += (int)mvsad_cost(c, br - 1, bc);
}

// full_pixel_diamond (mcomp.c:1479-1526)
// level -1: DIAMOND (av1_init_dsmotion_compensation); 0 / 1: NSTEP /
// NSTEP_8PT (no LDS window: their radii do not shrink by halves)
template <int W, int H, bool SKIP, bool TL>
__device__ int full_pixel_diamond(const Ctx& c, int lane, int srow, int scol, int step_param,
                                  int& brow, int& bcol, int& steps, int& searches, lds_u32 win,
                                  bool want_cl, int (&cl)[5], int level = -1) {
  Search<W, H, SKIP, true, TL> S;
  S.load_src(c, lane, level < 0 ? win : nullptr);
  int n, num00 = 0;
  auto run = [&](int sp, int& r, int& cc, int& n00) {
    if (level < 0) S.diamond(c, lane, srow, scol, sp, r, cc, n00, steps);
    else S.nstep_diamond(c, lane, level, srow, scol, sp, r, cc, n00, steps);
  };
  run(step_param, brow, bcol, n);
  ++searches;
  int bestsme = S.var_cost_at(c, lane, brow, bcol);
  const int further = (level < 0 ? kMaxSteps : nstep_steps(level)) - 1 - step_param;
  while (n < further) {
    ++n;
    int tr, tc;
    run(step_param + n, tr, tc, num00);
    ++searches;
    const int sme = S.var_cost_at(c, lane, tr, tc);
    if (sme < bestsme) {
      bestsme = sme;
      brow = tr;
      bcol = tc;
    }
    if (num00) {
      n += num00;
      num00 = 0;
    }
  }
  if (want_cl) int_sad_list(S, c, lane, brow, bcol, false, cl);
  return bestsme;
}

__device__ __forceinline__ int rawpel(int x) { return (x + 3 + (x >= 0)) >> 3; }  // mv.h:28

// ---------------------------------------------------------------- BIGDIA --
// av1_init_motion_compensation_bigdia (mcomp.c:498-550): scale 0 has the 4
// nearest points, scale s >= 1 8 points of radius r = 2^(s-1) / 2r.
// Offsets as 3-bit fields of (d + 2) in units of the scale's r, read by a
// shift per lane (the select chains over i compiled to exec-mask branches):
// scale 0 (0,-1) (1,0) (0,1) (-1,0); scale s >= 1, r = 2^(s-1):
// (-r,-r) (0,-2r) (r,-r) (2r,0) (r,r) (0,2r) (-r,r) (-2r,0)
constexpr uint32_t bigdia_pack(const int (&d)[8]) {
  uint32_t p = 0;
  for (int i = 0; i < 8; ++i) p |= (uint32_t)(d[i] + 2) << (3 * i);
  return p;
}
constexpr int kBdR0[8] = {0, 1, 0, -1, 0, 0, 0, 0}, kBdC0[8] = {-1, 0, 1, 0, 0, 0, 0, 0};
constexpr int kBdR1[8] = {-1, 0, 1, 2, 1, 0, -1, -2}, kBdC1[8] = {-1, -2, -1, 0, 1, 2, 1, 0};
constexpr uint32_t kBdPR0 = bigdia_pack(kBdR0), kBdPC0 = bigdia_pack(kBdC0);
constexpr uint32_t kBdPR1 = bigdia_pack(kBdR1), kBdPC1 = bigdia_pack(kBdC1);
__device__ __forceinline__ void bigdia_site(int s, int i, int& dr, int& dc) {
  const uint32_t pr = s == 0 ? kBdPR0 : kBdPR1, pc = s == 0 ? kBdPC0 : kBdPC1;
  const int sh = s == 0 ? 0 : s - 1;
  dr = ((int)((pr >> (3 * i)) & 7) - 2) * (1 << sh);
  dc = ((int)((pc >> (3 * i)) & 7) - 2) * (1 << sh);
}
// The other pattern_search site sets: av1_init_motion_compensation_square
// (mcomp.c:553-604: 8 points of r = 2^s, (-1,-1) (0,-1) (1,-1) (1,0) (1,1)
// (0,1) (-1,1) (-1,0) x r) and _hex (:607-653: scale 0 the square's 8,
// scale s >= 1 6 points (-1,-2) (1,-2) (2,0) (1,2) (-1,2) (-2,0) x 2^(s-1))
enum { kPatBigdia = 0, kPatSquare = 1, kPatHex = 2 };
constexpr int kSqR[8] = {-1, 0, 1, 1, 1, 0, -1, -1}, kSqC[8] = {-1, -1, -1, 0, 1, 1, 1, 0};
constexpr int kHxR[8] = {-1, 1, 2, 1, -1, -2, 0, 0}, kHxC[8] = {-2, -2, 0, 2, 2, 0, 0, 0};
constexpr uint32_t kSqPR = bigdia_pack(kSqR), kSqPC = bigdia_pack(kSqC);
constexpr uint32_t kHxPR = bigdia_pack(kHxR), kHxPC = bigdia_pack(kHxC);
__device__ __forceinline__ void pat_site(int kind, int s, int i, int& dr, int& dc) {
  if (kind == kPatBigdia) {
    bigdia_site(s, i, dr, dc);
    return;
  }
  const bool sq = kind == kPatSquare || s == 0;
  const uint32_t pr = sq ? kSqPR : kHxPR, pc = sq ? kSqPC : kHxPC;
  const int sh = sq ? s : s - 1;
  dr = ((int)((pr >> (3 * i)) & 7) - 2) * (1 << sh);
  dc = ((int)((pc >> (3 * i)) & 7) - 2) * (1 << sh);
}
// searches_per_step of scale s
__device__ __forceinline__ int pat_n(int kind, int s) {
  return kind == kPatBigdia ? (s == 0 ? 4 : 8) : (kind == kPatHex && s > 0 ? 6 : 8);
}

// pattern_search (mcomp.c:1017-1245) over the BIGDIA sites: with
// do_init_search every scale up to the start scale around the start point
// first (bigdia_search), else straight from the start scale (fast_bigdia /
// fast_dia / vfast_dia); per scale all candidates, then the 3 points around
// the winning direction until none improves.  With a cost list the last
// scale runs in the reference's separate block that keeps the raw SADs of
// the final neighbourhood (:1166-1221), then calc_int_sad_list.
// Lane group g evaluates candidate g; the keyed minimum is the reference's
// sequential update order (update_mvs_and_sad, mcomp.c:858-877), whose raw
// SAD is kept as raw_bestsad.
// WINP (a wave-serial caller, the TPL wavefront): the search first copies the
// (H + 30) x (W + 30) reference window around its clamped start into LDS
// (win: Win<W, H>::SIZE dwords, then 4 + 2 x 31 ints of mv-cost rates: the
// joint costs and the mvcost rows / columns of the window's 31 full-pel
// rows / columns), and every round whose candidates all lie inside it reads
// SADs and mv costs from LDS: one memory latency per search instead of one
// per round.  Rounds that reach outside read global memory as before.  vout:
// the plain variance at the result (the sub-pel step's FULL_PEL error).
typedef __attribute__((address_space(3))) int32_t* lds_i32;

// the window's mv-cost rates (after the window in LDS): the joint costs and
// the mvcost rows / columns of its 31 full-pel rows / columns around the
// clamped start (br, bc); lane l's three values
template <int W, int H>
__device__ __forceinline__ void win_rates_load(const Ctx& c, int lane, int br, int bc,
                                               int (&r)[3]) {
  using WN = Win<W, H>;
  constexpr int NR = 2 * WN::R + 1;
  const bool ent = c.cost_type == 0;
  typedef const __attribute__((address_space(1))) int32_t* gi32;
  const int wr0 = br - WN::R, wc0 = bc - WN::R;
  const int l = min(lane, NR - 1);
  // |row - full_ref| <= 1023 + 15 inside the window: inside the tables
  r[0] = ent ? ((gi32)c.mvjcost)[lane & 3] : 0;
  r[1] = ent ? ((gi32)c.mvcost0)[(wr0 + l - c.full_ref_row) * 8] : 0;
  r[2] = ent ? ((gi32)c.mvcost1)[(wc0 + l - c.full_ref_col) * 8] : 0;
}
template <int W, int H>
__device__ __forceinline__ void win_rates_store(lds_u32 win, int lane, const int (&r)[3]) {
  using WN = Win<W, H>;
  constexpr int NR = 2 * WN::R + 1;
  const lds_i32 rates = (lds_i32)(win + WN::SIZE);
  if (lane < 4) rates[lane] = r[0];
  if (lane < NR) {
    rates[4 + lane] = r[1];
    rates[4 + NR + lane] = r[2];
  }
}

// pattern()'s LDS window around the clamped start (br, bc): the reference
// window, then the mv-cost rates of its 31 full-pel rows / columns; S (any
// Search over this window) gets the window's origin
template <int W, int H, class S_t>
__device__ __forceinline__ void win_prefill(S_t& S, const Ctx& c, int lane, lds_u32 win, int br,
                                            int bc, bool filled) {
  using WN = Win<W, H>;
  S.win = win;
  if (filled) {  // the same window, already in LDS (S.fill without the copy)
    S.wr0 = br - WN::R;
    S.wc0 = bc - WN::R;
    S.wbase = (uintptr_t)(c.ref + (int64_t)S.wr0 * c.rs + S.wc0);
    return;
  }
  int r[3];
  win_rates_load<W, H>(c, lane, br, bc, r);
  win_rates_store<W, H>(win, lane, r);
  S.fill(c, lane, br, bc);  // (its wave_sync covers the rate stores)
}

// prefilled (WINP): the caller already copied this search's window
// (win_prefill at the same clamped start and limits)
template <int W, int H, bool SKIP, bool TL, bool WINP = false>
__device__ int pattern(const Ctx& c, int lane, int srow, int scol, int search_step, bool do_init,
                       bool want_cl, int (&cl)[5], int& brow, int& bcol, int& steps,
                       int& nsad, lds_u32 win = nullptr, uint32_t* vout = nullptr,
                       bool prefilled = false, int kind = kPatBigdia) {
  static_assert(!WINP || (Win<W, H>::kOn && !TL), "window: w, h <= 32, linear layout");
  using WN = Win<W, H>;
  constexpr int NR = 2 * WN::R + 1;  // full-pel rows / columns a window spans
  Search<W, H, SKIP, false, TL> S;
  S.load_src(c, lane, WINP ? win : nullptr);
  const int g = lane >> 3;
  search_step = min(search_step, kMaxSteps - 1);
  int best_init_s = kMaxSteps - 1 - search_step;  // search_steps[] = {10, 9, ..., 0}
  int br = min(max(srow, c.row_min), c.row_max);
  int bc = min(max(scol, c.col_min), c.col_max);
  if (want_cl) cl[0] = cl[1] = cl[2] = cl[3] = cl[4] = INT_MAX;
  bool has_sad = false;
  lds_i32 rates = nullptr;
  if constexpr (WINP) {
    rates = (lds_i32)(win + WN::SIZE);
    win_prefill<W, H>(S, c, lane, win, br, bc, prefilled);
  }
  // every candidate within d pixels of (r0, c0) inside the window
  auto in_win = [&](int r0, int c0, int d) {
    return WINP && r0 - d >= S.wr0 && r0 + d <= S.wr0 + 2 * WN::R && c0 - d >= S.wc0 &&
           c0 + d <= S.wc0 + 2 * WN::R;
  };
  auto rate_win = [&](int r, int cc) {
    const int dr = (r - c.full_ref_row) * 8, dc = (cc - c.full_ref_col) * 8;
    const int joint = c.cost_type == 0 ? ((dc != 0) | ((dr != 0) << 1)) : 0;
    const int ir = min(max(r - S.wr0, 0), NR - 1), ic = min(max(cc - S.wc0, 0), NR - 1);
    return MvRate{rates[joint], rates[4 + ir], rates[4 + NR + ic]};
  };
  uint32_t raw, best;
  if (in_win(br, bc, 0)) {
    raw = rdlane(S.group_sad_win(c, br, bc, true), 0);
    best = raw + mvsad_finish(c, rate_win(br, bc), br, bc);
  } else {
    raw = rdlane(S.group_sad(c, br, bc), 0);
    best = raw + mvsad_cost(c, br, bc);
  }
  ++nsad;
  // one round: candidate idx (groups g < cnt) of scale s around (br, bc);
  // returns the winning group or -1.  clmode 1: raw SADs of the valid
  // candidates into cl (calc_sad4 / calc_sad_update_bestmv); 2: also INT_MAX
  // for invalid ones (calc_sad3 / _with_indices)
  auto check = [&](int s, int cnt, int idx, int clmode) -> int {
    int dr, dc;
    pat_site(kind, s, idx, dr, dc);
    const int r = br + dr, cc = bc + dc;
    // (check_bounds only skips this test when it holds)
    const bool valid =
        g < cnt && cc >= c.col_min && cc <= c.col_max && r >= c.row_min && r <= c.row_max;
    MvRate mr;
    uint32_t mine;
    if (in_win(br, bc, 1 << s)) {  // scale s moves at most 2^s (4 points of 1 at s = 0)
      mr = rate_win(r, cc);
      mine = S.group_sad_win(c, r, cc, valid);
    } else {
      mr = mvsad_rate(c, r, cc);  // in flight with the SAD's loads
      mine = S.group_sad(c, r, cc, valid, br, bc);
    }
    const uint32_t key =
        (((mine + mvsad_finish(c, mr, r, cc)) << 3) | (uint32_t)g) | (valid ? 0u : ~0u);
    uint32_t kmin = groups_min(key);
    ++steps;
    nsad += __popcll(__ballot(valid)) >> 3;  // candidate blocks read this round
    if (clmode) {
      const uint32_t tag = valid ? (mine << 1) | 1u : 0u;  // SADs < 2^22
      for (int i = 0; i < cnt; ++i) {
        const uint32_t t = rdlane(tag, 8 * i);
        const int ix = (int)rdlane((uint32_t)idx, 8 * i);
        if (t & 1u) set_cl(cl, ix + 1, (int)(t >> 1));
        else if (clmode == 2) set_cl(cl, ix + 1, INT_MAX);
      }
    }
    if (kmin >= (best << 3)) return -1;
    best = kmin >> 3;
    raw = rdlane(mine, 8 * (int)(kmin & 7));
    return (int)(kmin & 7);
  };
  auto move = [&](int s, int k) {
    int dr, dc;
    pat_site(kind, s, k, dr, dc);
    br += dr;
    bc += dc;
  };
  // next_chkpts_indices: k - 1, k, k + 1 (cyclic over n)
  // (n is 4 or 8: a mask, no per-lane select chain -- those compiled to
  // exec-mask branches; HEX's 6: two compares)
  auto around = [](int j, int k, int n) {
    if ((n & (n - 1)) == 0) return (k + j - 1 + n) & (n - 1);
    int v = k + j - 1;
    v += v < 0 ? n : 0;
    return v >= n ? v - n : v;
  };
  // candidates a full scan of scale s evaluates: with every candidate in
  // bounds the reference's calc_sad4 groups of four and then
  // calc_sad_update_bestmv(num_candidates = n % 4, cand_start = n & ~3),
  // whose loop never runs -- HEX's 6-point scales evaluate their first four
  // (mcomp.c:1064-1077,1108-1122,964)
  auto scan_n = [&](int s) {
    const int n = pat_n(kind, s), d = 1 << s;
    const bool all = br - d >= c.row_min && br + d <= c.row_max && bc - d >= c.col_min &&
                     bc + d <= c.col_max;
    return all ? (n & ~3) : n;
  };
  int k = -1;
  if (do_init) {
    const int smax = best_init_s;
    best_init_s = -1;
    for (int t = 0; t <= smax; ++t) {
      const int w = check(t, scan_n(t), g, 0);
      if (w < 0) continue;
      best_init_s = t;
      k = w;
    }
    if (best_init_s != -1) move(best_init_s, k);
  }
  if (best_init_s != -1) {
    // last_is_4 && cost_list: num_candidates[0] == 4 (BIGDIA only)
    const int last_s = want_cl && kind == kPatBigdia ? 1 : 0;
    int best_site = -1;
    int s = best_init_s;
    for (; s >= last_s; --s) {
      const int n = pat_n(kind, s);
      if (!do_init || s != best_init_s) {
        best_site = check(s, scan_n(s), g, 0);
        if (best_site < 0) continue;
        move(s, best_site);
        k = best_site;
      }
      do {
        best_site = check(s, 3, around(g, k, n), 0);
        if (best_site >= 0) {
          k = around(best_site, k, n);
          move(s, k);
        }
      } while (best_site >= 0);
    }
    if (s == 0 && want_cl && kind == kPatBigdia) {
      cl[0] = (int)raw;
      has_sad = true;
      if (!do_init || s != best_init_s) {
        best_site = check(0, 4, g, 1);
        if (best_site >= 0) {
          move(0, best_site);
          k = best_site;
        }
      }
      while (best_site >= 0) {
        cl[1] = cl[2] = cl[3] = cl[4] = INT_MAX;
        set_cl(cl, ((k + 2) & 3) + 1, cl[0]);
        cl[0] = (int)raw;
        best_site = check(0, 3, around(g, k, 4), 2);
        if (best_site >= 0) {
          k = around(best_site, k, 4);
          move(0, k);
        }
      }
    }
  }
  brow = br;
  bcol = bc;
  if (want_cl) {
    if (in_win(br, bc, 1)) {
      // calc_int_sad_list (int_sad_list) with the window's SADs and rates
      if (!has_sad) {
        const int dr = g == 2 ? 1 : g == 4 ? -1 : 0, dc = g == 1 ? -1 : g == 3 ? 1 : 0;
        const int r = br + dr, cc = bc + dc;
        const bool valid =
            g < 5 && cc >= c.col_min && cc <= c.col_max && r >= c.row_min && r <= c.row_max;
        const uint32_t sad = S.group_sad_win(c, r, cc, valid);
        const uint32_t v = valid ? sad : 0x7FFFFFFFu;
#pragma unroll
        for (int i = 0; i < 5; ++i) cl[i] = (int)rdlane(v, 8 * i);
      }
      cl[0] += (int)mvsad_finish(c, rate_win(br, bc), br, bc);
      if (cl[1] != INT_MAX) cl[1] += (int)mvsad_finish(c, rate_win(br, bc - 1), br, bc - 1);
      if (cl[2] != INT_MAX) cl[2] += (int)mvsad_finish(c, rate_win(br + 1, bc), br + 1, bc);
      if (cl[3] != INT_MAX) cl[3] += (int)mvsad_finish(c, rate_win(br, bc + 1), br, bc + 1);
      if (cl[4] != INT_MAX) cl[4] += (int)mvsad_finish(c, rate_win(br - 1, bc), br - 1, bc);
    } else {
      int_sad_list(S, c, lane, br, bc, has_sad, cl);
    }
    if (!has_sad) nsad += 1 + (cl[1] != INT_MAX) + (cl[2] != INT_MAX) + (cl[3] != INT_MAX) +
                          (cl[4] != INT_MAX);
  }
  if constexpr (WINP) {
    S.inwin = in_win(br, bc, 0);
    return S.var_cost_at(c, lane, br, bc, vout);  // get_mvpred_var_cost
  }
  return var_cost<W, H>(c, lane, br, bc, vout);  // get_mvpred_var_cost
}

// waves (jobs) per workgroup of the search kernels
#ifndef LAVISH_DK_WAVES
#define LAVISH_DK_WAVES 4
#endif
constexpr int kDkWaves = LAVISH_DK_WAVES;

// search_method values of SEARCH_METHODS (av1/encoder/mcomp_structs.h:56-86)
enum {
  kDiamond = 0, kNstep = 1, kNstep8 = 2, kHex = 4, kBigdia = 5, kSquare = 6, kFastHex = 7,
  kFastDiamond = 8, kFastBigdia = 9, kVfastDiamond = 10
};
// the diamond_search_sad walks (full_pixel_diamond); the others are pattern searches
__host__ __device__ __forceinline__ bool diamond_method(int m) {
  return m == kDiamond || m == kNstep || m == kNstep8;
}
__host__ __device__ __forceinline__ int method_steps(int m) {
  return m == kNstep ? 15 : m == kNstep8 ? 16 : kMaxSteps;
}

// search context of one job: its buffers, FullMvLimits, ref_mv and mv costs
__device__ __forceinline__ Ctx job_ctx(const uint8_t* src, int ss, const uint8_t* ref, int rs,
                                       const Job& jb, const LavishMvCostParams& cost) {
  Ctx c;
  c.src = src + jb.src_off;
  c.ref = ref + jb.ref_off;
  c.ss = ss;
  c.rs = rs;
  c.col_min = jb.col_min;
  c.col_max = jb.col_max;
  c.row_min = jb.row_min;
  c.row_max = jb.row_max;
  c.ref_mv_row = jb.ref_mv_row;
  c.ref_mv_col = jb.ref_mv_col;
  c.full_ref_row = rawpel(jb.ref_mv_row);
  c.full_ref_col = rawpel(jb.ref_mv_col);
  c.cost_type = cost.mv_cost_type;
  c.sad_lambda = sad_lambda(cost.mv_cost_type);
  c.sse_lambda = sse_lambda(cost.mv_cost_type);
  c.sad_per_bit = cost.sad_per_bit;
  c.error_per_bit = cost.error_per_bit;
  const bool ent = cost.mv_cost_type == 0;  // (mvsad_cost: zero tables otherwise)
  c.mvjcost = ent ? cost.mvjcost : kZeroRate;
  c.mvcost0 = ent ? cost.mvcost[0] : kZeroRate;
  c.mvcost1 = ent ? cost.mvcost[1] : kZeroRate;
  return c;
}

// av1_full_pixel_search (mcomp.c:1755-1873, no mesh) of one job by one wave:
// DIAMOND (PAT false) or the BIGDIA-site pattern searches (method 5 / 8 /
// 9 / 10), the downsampled-SAD quality check and its full-SAD redo.
// searches: DIAMOND runs / the SAD blocks read by a pattern search.
template <int W, int H, bool PAT, bool TL, bool WINP = false>
__device__ __forceinline__ int job_search(const Ctx& c, int lane, int start_row, int start_col,
                                          int step_param, int skip, int method, lds_u32 win,
                                          bool want_cl, int (&cl)[5], int& br, int& bc,
                                          int& steps, int& searches, uint32_t* vout = nullptr,
                                          bool prefilled = false, bool* skip_used = nullptr) {
  int sme;
  auto search = [&](auto skip_tag) {
    constexpr bool SK = decltype(skip_tag)::value;
    if constexpr (!PAT) {
      return full_pixel_diamond<W, H, SK, TL>(c, lane, start_row, start_col, step_param, br, bc,
                                              steps, searches, win, want_cl, cl,
                                              method == kNstep ? 0 : method == kNstep8 ? 1 : -1);
    } else {
      // bigdia / hex / square (do_init 1), fast_dia / vfast_dia / fast_bigdia
      // / fast_hex (do_init 0) (mcomp.c:1258-1316)
      const bool init = method == kBigdia || method == kHex || method == kSquare;
      const int step = init                     ? step_param
                       : method == kFastDiamond || method == kFastHex ? max(kMaxSteps - 2, step_param)
                       : method == kVfastDiamond ? max(kMaxSteps - 1, step_param)
                                                 : max(kMaxSteps - 3, step_param);
      // (WINP: the TPL wavefront, whose methods are the BIGDIA family only)
      const int kind = WINP                                 ? kPatBigdia
                       : method == kHex || method == kFastHex ? kPatHex
                       : method == kSquare                  ? kPatSquare
                                                            : kPatBigdia;
      return pattern<W, H, SK, TL, WINP>(c, lane, start_row, start_col, step, init, want_cl, cl,
                                         br, bc, steps, searches, win, vout, prefilled, kind);
    }
  };
  // use_downsampled_sad applies to blocks at least 16 high (mcomp.c:132-133)
  if (skip && H >= 16) {
    sme = search(std::true_type{});
    // quality check of the row-skipping search (mcomp.c:1840-1867)
    int sad, ssad;
    sad_and_skip<W, H>(c, lane, br, bc, sad, ssad);
    const int thresh = (W >> 2) * (H >> 2);
    const bool redo = sad > thresh && abs(ssad - sad) * 10 >= max(sad, 1) * 9;
    if (redo) sme = search(std::false_type{});
    if (skip_used) *skip_used = !redo;
  } else {
    sme = search(std::false_type{});
    if (skip_used) *skip_used = false;
  }
  return sme;
}

// PAT: the BIGDIA-site pattern searches (method 5 / 8 / 9 / 10), else DIAMOND
template <int W, int H, bool PAT, bool TL>
__global__ __launch_bounds__(64 * kDkWaves, (W <= 16 && H <= 16) ? 8 : 7) void diamond_kernel(const uint8_t* __restrict__ src, int ss,
                                                      const uint8_t* __restrict__ ref, int rs,
                                                      LavishRefTiles tiles,
                                                      const Job* __restrict__ jobs, int njobs,
                                                      int step_param, LavishMvCostParams cost,
                                                      int skip, int method,
                                                      LavishDiamondResult* __restrict__ out,
                                                      int32_t* __restrict__ cost_lists,
                                                      uint8_t* __restrict__ sdf_kind) {
  // XCD-aware: consecutive job quads (neighbouring blocks) share an XCD's L2
  const int nwg = gridDim.x;  // multiple of 8
  const int wg = (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = wg * kDkWaves + wave;
  if (j >= njobs) return;
  constexpr int WS = PAT ? 1 : Win<W, H>::SIZE;  // the window serves DIAMOND only
  __shared__ uint32_t win_s[kDkWaves * WS];
  const lds_u32 win = (!PAT && Win<W, H>::kOn) ? (lds_u32)(win_s + wave * WS) : nullptr;
  const Job jb = jobs[j];
  Ctx c = job_ctx(src, ss, ref, rs, jb, cost);
  if constexpr (TL) {
    c.tiles = tiles.data;
    c.fh = tiles.field_rows;
    c.fsz = (int)tiles.field_bytes;
    // the job's block origin as (row, column) of the whole buffer (uniform)
    const int oy = (int)(jb.ref_off / rs);
    c.oy = __builtin_amdgcn_readfirstlane(oy);
    c.ox = __builtin_amdgcn_readfirstlane((int)(jb.ref_off - (int64_t)oy * rs));
  }
  const bool want_cl = cost_lists != nullptr;
  int cl[5] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX, INT_MAX};
  int br, bc, steps = 0, searches = 0;
  bool skip_used = false;
  const int sme = job_search<W, H, PAT, TL>(c, lane, jb.start_row, jb.start_col, step_param, skip,
                                            method, win, want_cl, cl, br, bc, steps, searches,
                                            nullptr, false, &skip_used);
  if (lane == 0) {
    LavishDiamondResult r;
    r.best_row = (int16_t)br;
    r.best_col = (int16_t)bc;
    r.bestsme = sme;
    r.steps = steps;
    r.searches = searches;
    out[j] = r;
    if (sdf_kind) sdf_kind[j] = skip_used;
  }
  if (want_cl && lane < 5) {
    const int v = lane == 0 ? cl[0] : lane == 1 ? cl[1] : lane == 2 ? cl[2] : lane == 3 ? cl[3] : cl[4];
    cost_lists[5 * (int64_t)j + lane] = v;
  }
}

// ---------------------------------------------------------------------------
// The exhaustive mesh refinement of av1_full_pixel_search (mcomp.c:1818-1838,
// 1875-1893 -> full_pixel_exhaustive :1603-1680 -> exhaustive_mesh_search
// :1529-1601), after the search kernel, one wave per job: forced when the
// search's variance passes force_mesh_thresh scaled to the block (NSTEP /
// NSTEP_8PT), or run_mesh_search; pruned when the search moved by at most
// mesh_search_mv_diff_threshold.  Each pass scans every step-th row and column
// of the range around its clamped start (column step 4 at step 1, the
// reference's 4-at-a-time calls, whose last partial group of a row stops one
// short of end_col) with the search's sdf (sdf_kind: the downsampled SAD when
// the search kept it); lane group g takes candidate base + g, and the keyed
// minimum (cost * 8 + g) over 8 candidates against the running best is the
// reference's sequential strict-< update.  The pass's best is the next pass's
// centre; the var cost at the end replaces the search's result only when
// smaller; the cost list is recomputed around the mesh's best either way (the
// reference's full_pixel_exhaustive writes it).
struct MeshArgs {
  int run, nstep, thr, prune, diff, intra, fine;
  int range[4], interval[4];
};

template <int W, int H, bool SK>
__device__ int mesh_refine(const Ctx& c, int lane, const MeshArgs& m, int srow, int scol,
                           bool want_cl, int (&cl)[5], int& br, int& bc) {
  Search<W, H, SK> S;
  S.load_src(c, lane);
  const int g = lane >> 3;
  int range = m.range[0], interval = m.interval[0];
  const int div = range / interval;  // (the host checked the first pattern)
  const int mag = max(abs(srow), abs(scol));
  range = min(max(range, 5 * mag / 4), 256);
  interval = max(interval, range / div);
  if (m.fine) interval = min(interval, 4);
  br = srow;
  bc = scol;
  auto pass = [&](int rng, int step) {
    const int r0c = min(max(br, c.row_min), c.row_max), c0c = min(max(bc, c.col_min), c.col_max);
    const int r0 = max(-rng, c.row_min - r0c), r1 = min(rng, c.row_max - r0c);
    const int q0 = max(-rng, c.col_min - c0c), q1 = min(rng, c.col_max - c0c);
    br = r0c;
    bc = c0c;
    uint32_t best = rdlane(S.group_sad(c, r0c, c0c), 0) + mvsad_cost(c, r0c, c0c);
    if (r1 < r0 || q1 < q0) return;
    const int nrows = (r1 - r0) / step + 1;
    int ncols;
    if (step > 1) {
      ncols = (q1 - q0) / step + 1;
    } else {
      const int n = q1 - q0 + 1;
      ncols = 4 * (n >> 2) + max((n & 3) - 1, 0);
    }
    if (ncols <= 0) return;
    const int total = nrows * ncols;
    for (int base = 0; base < total; base += 8) {
      const int idx = base + g;
      const bool valid = idx < total;
      const int ri = idx / ncols, ci = idx - ri * ncols;
      const int r = r0c + r0 + ri * step, cc = c0c + q0 + ci * step;
      const MvRate mr = mvsad_rate(c, valid ? r : r0c, valid ? cc : c0c);
      const uint32_t sad = S.group_sad(c, r, cc, valid, r0c, c0c);
      const uint32_t key = (((sad + mvsad_finish(c, mr, r, cc)) << 3) | (uint32_t)g) |
                           (valid ? 0u : ~0u);
      const uint32_t kmin = groups_min(key);
      if (kmin < (best << 3)) {
        best = kmin >> 3;
        const int bi = base + (int)(kmin & 7);
        const int bri = bi / ncols;
        br = r0c + r0 + bri * step;
        bc = c0c + q0 + (bi - bri * ncols) * step;
      }
    }
  };
  pass(range, interval);
  if (interval > 1 && range > 7) {
    for (int i = 1; i < 4; ++i) {
      pass(m.range[i], m.interval[i]);
      if (m.interval[i] == 1) break;
    }
  }
  if (want_cl) int_sad_list(S, c, lane, br, bc, false, cl);
  return var_cost<W, H>(c, lane, br, bc);
}

template <int W, int H>
__global__ __launch_bounds__(64 * kDkWaves) void mesh_kernel(
    const uint8_t* __restrict__ src, int ss, const uint8_t* __restrict__ ref, int rs,
    const Job* __restrict__ jobs, int njobs, LavishMvCostParams cost, MeshArgs m,
    const uint8_t* __restrict__ sdf_kind, LavishDiamondResult* __restrict__ out,
    int32_t* __restrict__ cost_lists) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = blockIdx.x * kDkWaves + wave;
  if (j >= njobs) return;
  const Job jb = jobs[j];
  const Ctx c = job_ctx(src, ss, ref, rs, jb, cost);
  LavishDiamondResult r = out[j];
  const int var = r.bestsme;
  bool run = m.run;
  if (!run && m.nstep && var > m.thr) run = true;
  if (!m.intra && m.prune &&
      max(abs(jb.start_row - r.best_row), abs(jb.start_col - r.best_col)) <= m.diff)
    run = false;
  if (!run) return;
  const bool want_cl = cost_lists != nullptr;
  int cl[5];
  int br, bc;
  const int var_ex = sdf_kind[j] ? mesh_refine<W, H, true>(c, lane, m, r.best_row, r.best_col,
                                                           want_cl, cl, br, bc)
                                 : mesh_refine<W, H, false>(c, lane, m, r.best_row, r.best_col,
                                                            want_cl, cl, br, bc);
  if (lane == 0 && var_ex < var) {
    r.best_row = (int16_t)br;
    r.best_col = (int16_t)bc;
    r.bestsme = var_ex;
    out[j] = r;
  }
  if (want_cl && lane < 5) {
    const int v = lane == 0 ? cl[0] : lane == 1 ? cl[1] : lane == 2 ? cl[2] : lane == 3 ? cl[3] : cl[4];
    cost_lists[5 * (int64_t)j + lane] = v;
  }
}

// ---------------------------------------------------------------------------
// TPL motion search with the reference's start-mv candidates (mode_estimation,
// av1/encoder/tpl_model.c:640-743): for every (reference, block) in raster
// order the centre mvs are the zero mv plus the above, left and above-right
// blocks' finished tpl mvs of the same reference that are not is_alike_mv
// (:319-333) to the ones already taken, the optional third-pass mv replacing
// centre 0 (:687-703); with prune_starting_mv their full SADs at the clamped
// full-pel centres rank them (qsort by compare_sad, :310-317, stable for
// these <= 4 entries), the list is cut to 4 - prune_starting_mv and by the
// SAD-gap rule (:720-727); motion_estimation (:249-303) runs per centre with
// ref_mv = the centre (mv cost, av1_set_mv_search_range) and the smallest
// sub-pel error wins (strict <).  With tpl_sf.subpel_force_stop FULL_PEL
// (speed >= 5) the sub-pel step returns setup_center_error: the variance at
// the full-pel best (MV_COST_NONE adds nothing) and the tpl mv is that best
// x 8.
//
// The dependency on finished neighbours makes this a wavefront: one wave per
// (reference, block row) walks its row left to right, a second wave of its
// workgroup does the walk's global stores (below).  A block's tpl mv is
// published by one device-scope atomic store into the mv array, which the
// call first fills with INVALID_MV; a wave waits for the above-right block by
// polling that slot (the mv itself is the ready flag: no separate progress
// counter and no second round trip), keeps the above mv from the previous
// step and the left mv in registers.  Rows are dealt out by an atomic ticket
// in (row, reference) order, so a waiting wave's producer already runs (no
// dependence on dispatch order); every wait is bounded, and a wave that gives
// up counts the failure in sync[1] and stops waiting, so the grid always
// drains.  Device-scope atomics bypass the per-XCD L2s, which are not
// coherent with each other.  The FAST_BIGDIA-family searches run with the
// LDS window of pattern() (one memory latency per search).
struct TplMvArgs {
  const uint8_t* src;
  const uint8_t* ref;
  int ss, rs;
  const Job* jobs;  // [nrefs][rows * cols]: offsets and x->mv_limits
  int cols, rows, nrefs;
  int step_param, skip, method, prune, alike_thr;
  LavishMvCostParams cost;
  const int32_t* third;  // [nrefs][rows * cols] int_mv or null
  int32_t* mvs;          // out: tpl mv (int_mv) per job; INVALID_MV until published
  LavishDiamondResult* out;
  int32_t* cost_lists;
  int32_t* centers;      // out: the winning centre (int_mv) per job, or null
  int32_t* sync;         // [0] ticket, [1] failed waits
};

constexpr int kTplMaxSpins = 1 << 22;  // ~0.3 s of s_sleep 2 per wait
#ifndef LAVISH_TPL_PREFILL
#define LAVISH_TPL_PREFILL 0  // 1: every centre's window copied at once, ranking SADs from them (A/B)
#endif
// LAVISH_TPL_SPEC=1: the speculative row walk (below).  Measured slower
// than the plain walk once the search got cheaper (2.04-2.12 vs 1.90 ms per
// 1080p x 7 refs, profiles/r04_v8_tpl_runs.jsonl): its extra per-block work
// (every kept centre's search before the wait, the bookkeeping of results
// per centre) costs more than the dependency latency it hides.
#ifndef LAVISH_TPL_SPEC
#define LAVISH_TPL_SPEC 0
#endif
constexpr int32_t kInvalidMv = (int32_t)0x80008000;  // INVALID_MV (mv.h)

__device__ __forceinline__ int mv_row(int32_t m) { return (int16_t)(m & 0xFFFF); }
__device__ __forceinline__ int mv_col(int32_t m) { return (int16_t)((uint32_t)m >> 16); }
__device__ __forceinline__ int32_t mv_pack(int row, int col) {
  return (int32_t)(((uint32_t)(uint16_t)col << 16) | (uint16_t)row);
}

// a[i] of a 4-entry register array for a dynamic i (select chains, no
// private-memory indexing)
__device__ __forceinline__ int get4(const int (&v)[4], int i) {
  return i == 0 ? v[0] : i == 1 ? v[1] : i == 2 ? v[2] : v[3];
}
__device__ __forceinline__ void set4(int (&v)[4], int i, int x) {
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = i == k ? x : v[k];
}

// LAVISH_TPL_PROF=1 (a diagnostic build, never the product): the wave's
// clock per step phase, summed over the grid into g_tpl_prof: [0] awaits,
// [1] centres + windows + ranking + searches after the await (speculative
// walk: the new-centre redo), [2] the same before the await (speculative
// walk), [3] new centres after the await, [4] publish, [5] the whole walk,
// [6] awaits that slept, [7] blocks, [9..12] steps with 1..4 centres before
// the ranking (non-speculative walk)
#ifndef LAVISH_TPL_PROF
#define LAVISH_TPL_PROF 0
#endif
#if LAVISH_TPL_PROF
__device__ unsigned long long g_tpl_prof[16];
#define TPL_PROF(...) __VA_ARGS__
__device__ __forceinline__ void tpl_lap(unsigned long long& acc, uint64_t& t) {
  const uint64_t now = clock64();
  acc += now - t;
  t = now;
}
#else
#define TPL_PROF(...)
#endif

// A block's results, handed from the searching wave to the publishing wave
struct TplBox {
  int seq;  // block index + 1 once the payload below is written
  int mv, br, bc, sme, steps, searches, center, cl[5];
};

template <bool PAT>
__global__ __launch_bounds__(128) void tpl_mv_kernel(TplMvArgs a) {
  constexpr int W = 16, H = 16;
  using WN = Win<W, H>;
  constexpr int WSZ = WN::SIZE + (PAT ? 4 + 2 * (2 * WN::R + 1) : 0);
  // PAT: one window per centre, all copied at once; DIAMOND: one
  constexpr bool kPrefill = PAT && LAVISH_TPL_PREFILL;
  constexpr bool kSpec = PAT && LAVISH_TPL_SPEC;
  using SW = Search<W, H, false, false, false>;
  const int lane = threadIdx.x & 63;
  // reference windows (+ the pattern searches' mv-cost rates)
  __shared__ uint32_t win_s[kPrefill ? 4 : 1][WSZ];
  __shared__ int res_s[kSpec ? 4 : 1][11];  // the speculative walk's search results
  __shared__ TplBox box_s[2];               // results by block parity
  __shared__ int ack_s, ticket_s;           // blocks published; the row ticket
  if (threadIdx.x == 0) {
    ticket_s = __hip_atomic_fetch_add(a.sync, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ack_s = 0;
    box_s[0].seq = box_s[1].seq = 0;
  }
  __syncthreads();
  const int t = __builtin_amdgcn_readfirstlane(ticket_s);
  TPL_PROF(unsigned long long prof[16] = {});
  const int ref = t % a.nrefs, row = t / a.nrefs;
  if (row >= a.rows) return;
  const int64_t nb = (int64_t)a.rows * a.cols;
  int32_t* const mvs = a.mvs + ref * nb;
  // Wave 1 publishes: the searching wave (0) hands each block's results over
  // in LDS and goes on.  On gfx9 a wave's stores and loads share one
  // completion counter, so a wave that stored its block's mv (a device-scope
  // store, ~2 us to complete) waited for that store at its next load; with
  // the stores on another wave the walk's loads wait for themselves only.
  if (threadIdx.x >= 64) {
    // The publisher's wait covers the searching wave's own waits on the row
    // above (each bounded by kTplMaxSpins x s_sleep 2), so it gets twice that
    // budget.  On a timeout the box holds no valid payload (col - 2's, or
    // nothing for col 0 / 1): the block and the rest of the row publish
    // INVALID_MV, which neighbours skip like an unavailable mv, the failure is
    // counted in sync[1] (TplFrame.check raises) and every block is
    // acknowledged so the searching wave never waits on this wave again.
    bool dead = false;
    for (int col = 0; col < a.cols; ++col) {
      TplBox& b = box_s[col & 1];
      int spins = 0;
      while (!dead &&
             __hip_atomic_load(&b.seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != col + 1) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins >= 2 * kTplMaxSpins) {  // (bounded: the grid always drains)
          if (lane == 0)
            __hip_atomic_fetch_add(a.sync + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          dead = true;
          __hip_atomic_store(&ack_s, a.cols, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      const int64_t bi = (int64_t)row * a.cols + col, j = ref * nb + bi;
      if (dead) {
        if (lane == 0) __hip_atomic_store(mvs + bi, kInvalidMv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      if (lane == 0) {
        __hip_atomic_store(mvs + bi, b.mv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        LavishDiamondResult best;
        best.best_row = (int16_t)b.br;
        best.best_col = (int16_t)b.bc;
        best.bestsme = b.sme;
        best.steps = b.steps;
        best.searches = b.searches;
        a.out[j] = best;
        if (a.centers) a.centers[j] = b.center;
      }
      if (a.cost_lists != nullptr && lane < 5) a.cost_lists[5 * j + lane] = b.cl[lane];
      __hip_atomic_store(&ack_s, col + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return;
  }
  // block col's results to the publishing wave (box reused every 2 blocks)
  auto publish = [&](int col, int32_t mv, int br, int bc, int sme, int steps, int searches,
                     int32_t center, const int* cl5) {
    TplBox& b = box_s[col & 1];
    int spins = 0;
    while (col >= 2 &&
           __hip_atomic_load(&ack_s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < col - 1) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins >= kTplMaxSpins) break;
    }
    if (lane == 0) {
      b.mv = mv;
      b.br = br;
      b.bc = bc;
      b.sme = sme;
      b.steps = steps;
      b.searches = searches;
      b.center = center;
#pragma unroll
      for (int q = 0; q < 5; ++q) b.cl[q] = cl5[q];
      __hip_atomic_store(&b.seq, col + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };
  bool waiting = true;
  // poll a published mv of the row above (uniform)
  auto await_mv = [&](int64_t k) -> int32_t {
    int32_t m = __hip_atomic_load(mvs + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (m == kInvalidMv && waiting) {
      __builtin_amdgcn_s_sleep(2);
      m = __hip_atomic_load(mvs + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      TPL_PROF(prof[6] += spins == 0);
      if (++spins >= kTplMaxSpins) {
        if (lane == 0)
          __hip_atomic_fetch_add(a.sync + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        waiting = false;
      }
    }
    return __builtin_amdgcn_readfirstlane(m);
  };
  const bool want_cl = a.cost_lists != nullptr;
  int32_t above = 0, left = 0;
  // the next block's job, loaded a step ahead as one dword per lane (lanes
  // 0..7) and kept in a vector register until the step that uses it: loaded
  // straight into scalars, the compiler waited for it at the load (one
  // exposed memory latency per block)
  auto job_load = [&](int64_t k) -> uint32_t {
    return ((const uint32_t*)(a.jobs + k))[min(lane, 7)];
  };
  auto job_get = [&](uint32_t w) {
    uint32_t d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = (uint32_t)__builtin_amdgcn_readlane((int)w, q);
    Job jb;
    __builtin_memcpy(&jb, d, sizeof(Job));
    return jb;
  };
  static_assert(sizeof(Job) == 32, "job: 8 dwords");
  uint32_t jw = job_load(ref * nb + (int64_t)row * a.cols);
  TPL_PROF(const uint64_t tk0 = clock64());
  if constexpr (kSpec) {
    // The row walk with speculation: everything a block needs but the
    // above-right neighbour (the job, the source, the centres from the zero
    // / above / left mvs, their windows and ranking SADs, and the searches of
    // the ranking's top centres) is done before waiting for that neighbour.
    // When it arrives it either adds no centre (is_alike_mv to one taken) --
    // the speculative result is the block's -- or a new last centre, which
    // gets its window and SAD; the ranking reruns over all centres and only
    // searches not yet run are added.  The searches' results are kept per
    // centre, so the outcome is the sequential one's (tpl_model.c:640-743).
    // With a third-pass mv (it replaces centre 0 unless alike to any
    // neighbour centre, the above-right one included) there is no
    // speculation.
    SW P;
    for (int col = 0; col < a.cols; ++col) {
      const int64_t bi = (int64_t)row * a.cols + col;
      TPL_PROF(uint64_t tp = clock64());
      if (row > 0 && col == 0) above = await_mv(bi - a.cols);
      const int64_t j = ref * nb + bi;
      const Job jb = job_get(jw);
      if (col + 1 < a.cols) jw = job_load(j + 1);
      const bool has_ar = row > 0 && col + 1 < a.cols;
      const bool spec = a.third == nullptr;
      int cr[4] = {0, 0, 0, 0}, cc[4] = {0, 0, 0, 0}, cs[4] = {0, 0, 0, 0};
      int n = 1;
      auto alike = [&](int r, int c, int from) {
        bool al = false;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          al |= i >= from && i < n && abs(cc[i] - c) < a.alike_thr && abs(cr[i] - r) < a.alike_thr;
        return al;
      };
      auto add = [&](int32_t m) {
        if (m == kInvalidMv) return;  // a timed-out wait never yields a centre
        const int r = mv_row(m), c = mv_col(m);
        if (!alike(r, c, 0)) {
          set4(cr, n, r);
          set4(cc, n, c);
          ++n;
        }
      };
      const Ctx c = job_ctx(a.src, a.ss, a.ref, a.rs, jb, a.cost);
      auto centre_ctx = [&](int i) {
        const int mr = get4(cr, i), mc = get4(cc, i);
        Ctx ci = c;
        ci.ref_mv_row = mr;
        ci.ref_mv_col = mc;
        ci.full_ref_row = rawpel(mr);
        ci.full_ref_col = rawpel(mc);
        // av1_set_mv_search_range (mcomp.c:206-234)
        ci.col_min = max((int)jb.col_min, max(((mc + 7) >> 3) - 1023, -2047));
        ci.row_min = max((int)jb.row_min, max(((mr + 7) >> 3) - 1023, -2047));
        ci.col_max = max(ci.col_min, min((int)jb.col_max, min((mc >> 3) + 1023, 2047)));
        ci.row_max = max(ci.row_min, min((int)jb.row_max, min((mr >> 3) + 1023, 2047)));
        return ci;
      };
      if constexpr (kPrefill) P.load_src(c, lane, (lds_u32)win_s[0]);  // (the window SADs' source rows)
      // per centre (original index): its search's results once run, in LDS
      // (res_s[k]: var, row, col, sme, steps, searches, cost list) -- in
      // registers they were 44 live scalars across every search
      int have = 0;
      int ix[4] = {0, 1, 2, 3}, np = 1, nf = 0;
      int32_t above_right = 0;
      for (int phase = spec ? 0 : 1; phase < 2; ++phase) {
        if (phase == 0) {
          if (row > 0) add(above);
          if (col > 0) add(left);
        } else {
          if (has_ar) above_right = await_mv(bi - a.cols + 1);
          TPL_PROF(tpl_lap(prof[0], tp));
          if (spec) {
            const int n0 = n;
            if (has_ar) add(above_right);
            if (n == n0) break;  // nothing new: the speculative result stands
            TPL_PROF(prof[3] += 1);
          } else {
            if (row > 0) add(above);
            if (col > 0) add(left);
            if (has_ar) add(above_right);
            const int32_t m = a.third[j];
            if (m != kInvalidMv && !alike(mv_row(m), mv_col(m), 1)) {
              cr[0] = mv_row(m);
              cc[0] = mv_col(m);
            }
          }
        }
        TPL_PROF(tpl_lap(prof[8], tp));
        // windows (pattern's own fill at the start clamped to the centre's
        // limits, all loads in flight together) and ranking SADs of the
        // centres [nf, n)
        if constexpr (!kPrefill) {  // ranking SADs from global memory, all in flight
          if (a.prune) {
            // get_fullmv_from_mv + clamp_fullmv to x->mv_limits, then sdf
            int fr[4], fc[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              fr[k] = min(max(rawpel(cr[k]), (int)jb.row_min), (int)jb.row_max);
              fc[k] = min(max(rawpel(cc[k]), (int)jb.col_min), (int)jb.col_max);
            }
            sad16_multi(c, lane, fr, fc, nf, n, cs);
          }
          nf = n;
          TPL_PROF(tpl_lap(prof[10], tp));
        } else {
          typename SW::fill_v v[4][SW::kFillNI];
          int rt[4][3];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (k >= nf && k < n) {
              const Ctx ci = centre_ctx(k);
              const int sr = min(max(rawpel(get4(cr, k)), ci.row_min), ci.row_max);
              const int sc = min(max(rawpel(get4(cc, k)), ci.col_min), ci.col_max);
              P.fill_load(ci, lane, sr, sc, v[k]);
              win_rates_load<W, H>(ci, lane, sr, sc, rt[k]);
            }
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (k >= nf && k < n) {
              P.win = (lds_u32)win_s[k];
              P.fill_store(lane, v[k]);
              win_rates_store<W, H>(P.win, lane, rt[k]);
            }
          }
          wave_sync();
          TPL_PROF(tpl_lap(prof[9], tp));
          if (a.prune) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              if (k >= nf && k < n) {
                const Ctx ci = centre_ctx(k);
                const int sr = min(max(rawpel(get4(cr, k)), ci.row_min), ci.row_max);
                const int sc = min(max(rawpel(get4(cc, k)), ci.col_min), ci.col_max);
                const int fr = min(max(rawpel(get4(cr, k)), (int)jb.row_min), (int)jb.row_max);
                const int fc = min(max(rawpel(get4(cc, k)), (int)jb.col_min), (int)jb.col_max);
                int sad;
                if (fr == sr && fc == sc) {
                  win_prefill<W, H>(P, ci, lane, (lds_u32)win_s[k], sr, sc, true);  // (origin only)
                  sad = (int)rdlane(P.group_sad_win(ci, fr, fc, true), 0);
                } else {  // off the window centre: from global memory
                  int ssad;
                  sad_and_skip<W, H>(c, lane, fr, fc, sad, ssad);
                }
                set4(cs, k, sad);
              }
            }
          }
          nf = n;
          TPL_PROF(tpl_lap(prof[10], tp));
        }
        // the ranking: stable insertion sort of the centres by SAD (glibc's
        // qsort on <= 4 entries), cut to 4 - prune_starting_mv and by the
        // SAD-gap rule
        ix[0] = 0;
        ix[1] = 1;
        ix[2] = 2;
        ix[3] = 3;
        np = n;
        if (a.prune && n > 1) {
          int sc4[4] = {cs[0], cs[1], cs[2], cs[3]};
#pragma unroll
          for (int i = 1; i < 4; ++i) {
#pragma unroll
            for (int k = i; k > 0; --k) {
              if (i < n && sc4[k - 1] > sc4[k]) {
                const int x = sc4[k], o = ix[k];
                sc4[k] = sc4[k - 1];
                ix[k] = ix[k - 1];
                sc4[k - 1] = x;
                ix[k - 1] = o;
              }
            }
          }
          np = min(4 - a.prune, n);
          if (np > 1 && (get4(sc4, np - 1) - get4(sc4, np - 2)) * 5 > get4(sc4, np - 2)) --np;
        }
        TPL_PROF(tpl_lap(prof[11], tp));
        // the searches of the kept centres not yet run
#pragma unroll 1
        for (int i = 0; i < np; ++i) {
          const int k = get4(ix, i);
          if ((have >> k) & 1) continue;
          TPL_PROF(prof[13] += 1);
          const int mr = get4(cr, k), mc = get4(cc, k);
          const Ctx ci = centre_ctx(k);
          int cl[5] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX, INT_MAX};
          int br, bc, steps = 0, searches = 0;
          uint32_t var = 0;
          const int sme = job_search<W, H, PAT, false, PAT>(
              ci, lane, rawpel(mr), rawpel(mc), a.step_param, a.skip, a.method,
              (lds_u32)win_s[kPrefill ? k : 0], want_cl, cl, br, bc, steps, searches, &var,
              kPrefill);
          have |= 1 << k;
          if (lane == 0) {
            int* o = res_s[k];
            o[0] = (int)var;
            o[1] = br;
            o[2] = bc;
            o[3] = sme;
            o[4] = steps;
            o[5] = searches;
#pragma unroll
            for (int q = 0; q < 5; ++q) o[6 + q] = cl[q];
          }
        }
        TPL_PROF(tpl_lap(prof[12], tp));
      }
      // the kept centres in ranking order: the smallest error wins (strict <)
      wave_sync();
      int win_k = get4(ix, 0);
      uint32_t bestsme = (uint32_t)res_s[win_k][0];
      for (int i = 1; i < np; ++i) {
        const int k = get4(ix, i);
        if ((uint32_t)res_s[k][0] < bestsme) {
          bestsme = (uint32_t)res_s[k][0];
          win_k = k;
        }
      }
      const int* w = res_s[win_k];
      const int best_r = w[1], best_c = w[2];
      const int32_t mine = mv_pack(8 * best_r, 8 * best_c);
      publish(col, mine, best_r, best_c, w[3], w[4], w[5],
              mv_pack(get4(cr, win_k), get4(cc, win_k)), w + 6);
      (void)j;
      left = mine;
      above = above_right;
      TPL_PROF(tpl_lap(prof[4], tp));
    }
  } else {
  for (int col = 0; col < a.cols; ++col) {
    const int64_t bi = (int64_t)row * a.cols + col;
    int32_t above_right = 0;
    TPL_PROF(uint64_t tp = clock64());
    if (row > 0 && col == 0) above = await_mv(bi - a.cols);
    const int64_t j = ref * nb + bi;
    const Job jb = job_get(jw);
    if (col + 1 < a.cols) jw = job_load(j + 1);
    // centre candidates (row, col in 1/8 pel) and their SADs
    int cr[4] = {0, 0, 0, 0}, cc[4] = {0, 0, 0, 0}, cs[4] = {0, 0, 0, 0};
    int n = 1;
    // is_alike_mv against centres [from, n)
    auto alike = [&](int r, int c, int from) {
      bool al = false;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        al |= i >= from && i < n && abs(cc[i] - c) < a.alike_thr && abs(cr[i] - r) < a.alike_thr;
      return al;
    };
    auto add = [&](int32_t m) {
      // a slot still holding INVALID_MV is a neighbour whose wait timed out
      // (counted in sync[1], the caller raises): never a centre
      if (m == kInvalidMv) return;
      const int r = mv_row(m), c = mv_col(m);
      if (!alike(r, c, 0)) {
        set4(cr, n, r);
        set4(cc, n, c);
        ++n;
      }
    };
    if (row > 0) add(above);
    if (col > 0) add(left);
    Ctx c = job_ctx(a.src, a.ss, a.ref, a.rs, jb, a.cost);
    // get_fullmv_from_mv + clamp_fullmv to x->mv_limits: the ranking's point
    int fr[4], fc[4];
    auto rank_points = [&]() {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fr[i] = min(max(rawpel(cr[i]), (int)jb.row_min), (int)jb.row_max);
        fc[i] = min(max(rawpel(cc[i]), (int)jb.col_min), (int)jb.col_max);
      }
    };
    // the ranking loads of the centres known before the above-right block
    // (zero / above / left) go out before its wait; their SADs are taken
    // after it (without prune_starting_mv nothing is ranked)
    const int n0 = n;
    Sad16Loads pre{};
    if (!kPrefill && a.prune) {
      rank_points();
      pre = sad16_load(c, lane, fr, fc, 0, n0);
    }
    if (row > 0 && col + 1 < a.cols) {
      above_right = await_mv(bi - a.cols + 1);
      add(above_right);
    }
    TPL_PROF(tpl_lap(prof[0], tp));
    bool c0_new = false;
    if (a.third) {
      const int32_t m = a.third[j];
      if (m != kInvalidMv && !alike(mv_row(m), mv_col(m), 1)) {
        cr[0] = mv_row(m);
        cc[0] = mv_col(m);
        c0_new = true;
      }
    }
    if (!kPrefill && a.prune && n > 1) {
      if (n > n0 || c0_new) {  // the above-right centre / a third-pass centre 0: after the wait
        rank_points();
        const Sad16Loads post = sad16_load(c, lane, fr, fc, c0_new ? 0 : n0, n);
        if (!c0_new) sad16_finish(pre, 0, n0, cs);
        sad16_finish(post, c0_new ? 0 : n0, n, cs);
      } else {
        sad16_finish(pre, 0, n, cs);
      }
    }
    TPL_PROF(prof[8 + n] += 1);  // centres before the ranking
    // av1_make_default_fullpel_ms_params with ref_mv = centre i
    auto centre_ctx = [&](int i) {
      const int mr = get4(cr, i), mc = get4(cc, i);
      Ctx ci = c;
      ci.ref_mv_row = mr;
      ci.ref_mv_col = mc;
      ci.full_ref_row = rawpel(mr);
      ci.full_ref_col = rawpel(mc);
      // av1_set_mv_search_range (mcomp.c:206-234): MAX_FULL_PEL_VAL 1023,
      // MV_LOW / MV_UPP = -/+ (1 << 14)
      ci.col_min = max((int)jb.col_min, max(((mc + 7) >> 3) - 1023, -2047));
      ci.row_min = max((int)jb.row_min, max(((mr + 7) >> 3) - 1023, -2047));
      ci.col_max = max(ci.col_min, min((int)jb.col_max, min((mc >> 3) + 1023, 2047)));
      ci.row_max = max(ci.row_min, min((int)jb.row_max, min((mr >> 3) + 1023, 2047)));
      return ci;
    };
    // the search's start: the centre clamped to its own limits
    auto centre_start = [&](const Ctx& ci, int i, int& sr, int& sc) {
      sr = min(max(rawpel(get4(cr, i)), ci.row_min), ci.row_max);
      sc = min(max(rawpel(get4(cc, i)), ci.col_min), ci.col_max);
    };
    const bool rank = a.prune && n > 1;  // one centre: the ranking and both cuts change nothing
    int ix[4] = {0, 1, 2, 3};            // original centre of each sorted position
    if constexpr (kPrefill) {
      // every centre's search window (pattern's own fill: the start clamped
      // to the centre's limits) with all loads in flight together; the
      // ranking SADs then come from the windows wherever the ranking's clamp
      // (x->mv_limits) lands on the window centre: the ranking and the
      // windows share one memory latency
      SW P;
      P.load_src(c, lane, (lds_u32)win_s[0]);
      typename SW::fill_v v[4][SW::kFillNI];
      int rt[4][3];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = min(i, n - 1);  // (surplus slots repeat the last centre, never stored)
        const Ctx ci = centre_ctx(k);
        int sr, sc;
        centre_start(ci, k, sr, sc);
        P.fill_load(ci, lane, sr, sc, v[i]);
        win_rates_load<W, H>(ci, lane, sr, sc, rt[i]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i < n) {
          P.win = (lds_u32)win_s[i];
          P.fill_store(lane, v[i]);
          win_rates_store<W, H>(P.win, lane, rt[i]);
        }
      }
      wave_sync();
      if (rank) {
        uint32_t part[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = min(i, n - 1);
          const Ctx ci = centre_ctx(k);
          int sr, sc;
          centre_start(ci, k, sr, sc);
          const int fr = min(max(rawpel(get4(cr, k)), (int)jb.row_min), (int)jb.row_max);
          const int fc = min(max(rawpel(get4(cc, k)), (int)jb.col_min), (int)jb.col_max);
          P.win = (lds_u32)win_s[k];
          win_prefill<W, H>(P, ci, lane, P.win, sr, sc, true);  // (origin only)
          part[i] = P.group_sad_win(ci, fr, fc, fr == sr && fc == sc);
          cs[i] = (int)rdlane(part[i], 0);
          if (fr != sr || fc != sc) {  // off the window centre: from global memory
            int sad, ssad;
            sad_and_skip<W, H>(c, lane, fr, fc, sad, ssad);
            cs[i] = sad;
          }
        }
      }
    }
    if (rank) {
      // insertion sort: stable, like glibc's qsort on <= 4 entries; as
      // compare-exchanges of neighbours (i from 1, each sinking left)
#pragma unroll
      for (int i = 1; i < 4; ++i) {
#pragma unroll
        for (int k = i; k > 0; --k) {
          if (i < n && cs[k - 1] > cs[k]) {
            const int r = cr[k], q = cc[k], x = cs[k], o = ix[k];
            cr[k] = cr[k - 1];
            cc[k] = cc[k - 1];
            cs[k] = cs[k - 1];
            ix[k] = ix[k - 1];
            cr[k - 1] = r;
            cc[k - 1] = q;
            cs[k - 1] = x;
            ix[k - 1] = o;
          }
        }
      }
      n = min(4 - a.prune, n);
      if (n > 1 && (get4(cs, n - 1) - get4(cs, n - 2)) * 5 > get4(cs, n - 2)) --n;
    }
    TPL_PROF(tpl_lap(prof[1], tp));
    uint32_t bestsme = 0xFFFFFFFFu;
    int best_r = 0, best_c = 0, win_i = 0;
    int bcl[5] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX, INT_MAX};
    LavishDiamondResult best{};
    for (int i = 0; i < n; ++i) {
      const int mr = get4(cr, i), mc = get4(cc, i);
      const Ctx ci = centre_ctx(i);
      int cl[5] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX, INT_MAX};
      int br, bc, steps = 0, searches = 0;
      uint32_t var = 0;
      const lds_u32 win = (lds_u32)win_s[kPrefill ? get4(ix, i) : 0];
      const int sme = job_search<W, H, PAT, false, PAT>(ci, lane, rawpel(mr), rawpel(mc),
                                                        a.step_param, a.skip, a.method, win,
                                                        want_cl, cl, br, bc, steps, searches,
                                                        &var, kPrefill);
      // find_fractional_mv_step at FULL_PEL: setup_center_error, the plain
      // variance at the full-pel best (MV_COST_NONE); the pattern searches
      // return it with their var cost
      if constexpr (!PAT) {
        Ctx cv = ci;
        cv.cost_type = 4;
        cv.sse_lambda = 0;
        var = (uint32_t)var_cost<W, H>(cv, lane, br, bc);
      }
      if (var < bestsme) {
        bestsme = var;
        best_r = br;
        best_c = bc;
        win_i = i;
        best.best_row = (int16_t)br;
        best.best_col = (int16_t)bc;
        best.bestsme = sme;
        best.steps = steps;
        best.searches = searches;
#pragma unroll
        for (int k = 0; k < 5; ++k) bcl[k] = cl[k];
      }
    }
    TPL_PROF(tpl_lap(prof[2], tp));
    const int32_t mine = mv_pack(8 * best_r, 8 * best_c);
    publish(col, mine, best_r, best_c, best.bestsme, best.steps, best.searches,
            mv_pack(get4(cr, win_i), get4(cc, win_i)), bcl);
    left = mine;
    above = above_right;
    TPL_PROF(tpl_lap(prof[4], tp));
  }
  }
#if LAVISH_TPL_PROF
  prof[5] = clock64() - tk0;
  prof[7] = a.cols;
  if (lane == 0)
    for (int k = 0; k < 16; ++k)
      __hip_atomic_fetch_add(&g_tpl_prof[k], prof[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// ---------------------------------------------------------------------------
// DIAMOND, 16x16 blocks, tiled references: eight jobs per wave.
//
// The one-job-per-wave kernel spends ~70 VALU + ~60 SALU instructions per
// 8-site step on one job: its time goes to instruction issue and to the
// per-step dependency chain, not to memory (halving its address-path work
// with the tiled layout changed nothing, profiles/r03_*).  Here lane
// (j = lane >> 3, l = lane & 7) works for job j of eight: a step evaluates
// the job's 8 sites one after the other, lane l reading row 2l (downsampled
// SAD; rows l and l + 8 otherwise) of each candidate from the tiled copy, so
// one load instruction covers one site of all eight jobs (8 x 256 contiguous
// bytes) and one step's bookkeeping serves eight jobs.  Each job carries its
// own walk in the lanes of its group (row, col, radius, search index, num00
// state): jobs at different radii / searches step together, branch-free.
// full_pixel_diamond's var costs do not steer the search sequence (n and
// num00 come from the walks alone), so each search's result is recorded and
// the var costs are evaluated once the job's walks are done, in the
// reference's order with its strict "sme < bestsme".  Then the cost list,
// the downsampled-SAD quality check (mcomp.c:1840-1867) and, for the jobs it
// fails, a second pass with full-row SADs.  Bit-exact with diamond_kernel.
constexpr int kLjJobs = 8;  // jobs per wave
constexpr int kMvDecHalf = 2047;          // MV_MAX / 8: full-pel reach of the cost tables
constexpr int kMvDecN = 2 * kMvDecHalf + 1;

__device__ __forceinline__ uint32_t group_min8(uint32_t v) {  // min over the 8-lane group
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
  return v;
}

// source rows of lane l: sk = row 2l (downsampled SAD), fr[k] = row l + 8k
struct LjSrc {
  uint32_t sk[4], fr[2][4];
};

// group SAD of the job's candidate at (r, cc) (in range), from the tiles
template <bool SKIP>
__device__ __forceinline__ uint32_t lj_sad(const Ctx& c, const LjSrc& s, int l, int r, int cc) {
  const int x = c.ox + cc;
  uint32_t acc = 0;
  if constexpr (SKIP) {
    uint32_t t[4];
    load_row<4>(c.tiles + tile_off(c, c.oy + r + 2 * l, x), t);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = sad4(s.sk[i], t[i], acc);
  } else {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint32_t t[4];
      load_row<4>(c.tiles + tile_off(c, c.oy + r + l + 8 * k, x), t);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = sad4(s.fr[k][i], t[i], acc);
    }
  }
  acc = group_sum8(acc);
  return SKIP ? 2 * acc : acc;
}

// aom_variance16x16 + mv_err_cost at (r, cc), the linear reference; lane l
// takes rows l and l + 8
__device__ __forceinline__ int lj_var(const Ctx& c, const LjSrc& s, int l, int r, int cc) {
  int sum = 0;
  uint32_t sse = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    uint32_t t[4];
    load_row<4>(c.ref + (int64_t)(r + l + 8 * k) * c.rs + cc, t);
#pragma unroll
    for (int i = 0; i < 4; ++i) var_acc(s.fr[k][i], t[i], sum, sse);
  }
  const uint32_t ts = group_sum8((uint32_t)sum), tq = group_sum8(sse);
  const uint32_t var = tq - (uint32_t)(((int64_t)(int)ts * (int)ts) / 256);
  return (int)var + mv_cost(c, r, cc);
}

// N candidates' group SADs with every load in flight before the first SAD:
// (r[i], cc[i]) in range where v[i]; an invalid candidate's rows are read at
// an offset past the tiled buffer's end, which the buffer descriptor's range
// check drops (no memory request, the value 0; its SAD is masked by the
// caller).  Loads through a branch per candidate were serialised by the
// compiler, one memory round trip per candidate (profiles/r04_c3_isa_*).
template <bool SKIP, int N>
__device__ __forceinline__ void lj_sads(const Ctx& c, const LjSrc& s, int l,
                                        __amdgpu_buffer_rsrc_t trs, int oob, const int (&r)[N],
                                        const int (&cc)[N], const bool (&v)[N],
                                        uint32_t (&out)[N]) {
  constexpr int RW = SKIP ? 1 : 2;  // rows per lane
  u32x4 t[N][RW];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      const int y = c.oy + r[i] + (SKIP ? 2 * l : l + 8 * k);
      t[i][k] = __builtin_amdgcn_raw_buffer_load_b128(
          trs, v[i] ? (int)tile_off(c, y, c.ox + cc[i]) : oob, 0, 0);
    }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      const uint32_t* q = SKIP ? s.sk : s.fr[k];
      acc = sad4(q[0], t[i][k].x, acc);
      acc = sad4(q[1], t[i][k].y, acc);
      acc = sad4(q[2], t[i][k].z, acc);
      acc = sad4(q[3], t[i][k].w, acc);
    }
    acc = group_sum8(acc);
    out[i] = SKIP ? 2 * acc : acc;
  }
}

// The 8 candidates' group SADs of a diamond step, lane l of each 8-lane
// group keeping the one of site l: a reduce-scatter over the group instead
// of 8 full group sums and a select.  Stage 1 pairs lane l with its mirror
// 7 - l (row_half_mirror): the lane keeps the half of the sites it will end
// with (0-3 below lane 4, 4-7 above), adds its partner's partial sums of
// that half and hands over the other; stages 2 and 3 do the same with lane
// l ^ 2 and l ^ 1 (quad_perm), so lane l ends with site 4 b2 + 2 b1 + b0 =
// l summed over all 8 lanes: 21 DPP adds / selects per step instead of 24
// DPP adds + 8 selects.  The same sums as group_sum8 (integer adds).
__device__ __forceinline__ uint32_t scatter_sum8(const uint32_t (&p)[8], int l) {
  const bool hi = l & 4, m1 = l & 2, m0 = l & 1;
  uint32_t q[4], r[2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t send = hi ? p[k] : p[k + 4];
    const uint32_t keep = hi ? p[k + 4] : p[k];
    q[k] = keep + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0x141, 0xF, 0xF, false);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t send = m1 ? q[k] : q[k + 2];
    const uint32_t keep = m1 ? q[k + 2] : q[k];
    r[k] = keep + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0x4E, 0xF, 0xF, false);
  }
  const uint32_t send = m0 ? r[0] : r[1];
  const uint32_t keep = m0 ? r[1] : r[0];
  return keep + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0xB1, 0xF, 0xF, false);
}

// the 8-site step (downsampled rows) at offsets into the tiled copy computed
// by the caller, lane l reading row 2l of each candidate: lane l gets site
// l's group SAD
__device__ __forceinline__ uint32_t lj_step_sad(const LjSrc& s, __amdgpu_buffer_rsrc_t trs,
                                                int oob, const uint32_t (&off)[8],
                                                const bool (&v)[8], int l) {
  u32x4 t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    t[i] = __builtin_amdgcn_raw_buffer_load_b128(trs, v[i] ? (int)off[i] : oob, 0, 0);
  uint32_t p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t acc = sad4(s.sk[0], t[i].x, 0);
    acc = sad4(s.sk[1], t[i].y, acc);
    acc = sad4(s.sk[2], t[i].z, acc);
    p[i] = sad4(s.sk[3], t[i].w, acc);
  }
  return 2 * scatter_sum8(p, l);
}

// mvsad_err_cost's table reads for the entropy cost through the decimated
// copy of the caller's row / column tables (dec[0..4094] = mvcost0[8 k],
// dec[4095..] = mvcost1[8 k], k = -2047 .. 2047, built per call by
// mvcost_dec_kernel): a full-pel search only ever indexes multiples of 8,
// so the copy is contiguous in what a step reads (a job's 8 sites differ by
// +-rad full pels) and the site costs of a step share cache lines.
__device__ __forceinline__ MvRate mvsad_rate_dec(const Ctx& c, const int32_t* dec, int row,
                                                 int col) {
  if (dec == nullptr) return mvsad_rate(c, row, col);
  const int kr = row - c.full_ref_row, kc = col - c.full_ref_col;
  const int joint = (kc != 0) | ((kr != 0) << 1);  // av1_get_mv_joint
  typedef const __attribute__((address_space(1))) int32_t* gi32;
  return MvRate{((gi32)c.mvjcost)[joint], ((gi32)dec)[kr + kMvDecHalf],
                ((gi32)dec)[kc + kMvDecHalf + kMvDecN]};
}

// one pass of full_pixel_diamond (+ its cost list) for the wave's jobs whose
// `run` is set; accumulates steps / searches, leaves the pass's best mv, var
// cost and cost list
template <bool SKIP>
__device__ void lj_pass(const Ctx& c, const LjSrc& s, int l, __amdgpu_buffer_rsrc_t trs, int oob,
                        const int32_t* dec, bool run, int step_param, bool want_cl,
                        uint32_t* res, int& steps,
                        int& searches, int& br, int& bc, int& sme, int (&cl)[5]) {
  // (br / bc carry the start mv on entry; diamond_search_sad clamps it)
  const int srow = min(max(br, c.row_min), c.row_max);
  const int scol = min(max(bc, c.col_min), c.col_max);
  const int sdr = site_dr(l), sdc = site_dc(l);
  // the start: its SAD once per pass (every run restarts there)
  uint32_t c0;
  {
    const int r1[1] = {srow}, c1[1] = {scol};
    const bool v1[1] = {true};
    uint32_t o1[1];
    lj_sads<SKIP, 1>(c, s, l, trs, oob, r1, c1, v1, o1);
    c0 = o1[0] + mvsad_finish(c, mvsad_rate_dec(c, dec, srow, scol), srow, scol);
  }
  const int further = kMaxSteps - 1 - step_param;
  bool active = run;
  bool first = true;
  int n = 0, row = srow, col = scol, stp = kMaxSteps - step_param - 1, center = 0, nres = 0;
  bool offc = false;
  uint32_t best = c0;
  while (__builtin_amdgcn_ballot_w64(active) != 0) {
    const int rad = 1 << stp;
    // lane l: site l's cost (its loads in flight with the SAD loads below)
    const int rl = row + sdr * rad, cl_ = col + sdc * rad;
    const bool vl = cl_ >= c.col_min && cl_ <= c.col_max && rl >= c.row_min && rl <= c.row_max;
    // loads only for in-range sites of jobs still walking: out-of-range
    // sites (most of the large radii) and finished jobs issue no memory
    // requests (the range-checked offset); a job's 8 lanes share both
    // conditions, so each group's DPP sum stays whole
    MvRate mr = {0, 0, 0};
    if (vl && active) mr = mvsad_rate_dec(c, dec, rl, cl_);
    uint32_t mine = 0;
    // the 8 sites: all loads issued, then the SADs (SKIP: 8 x 1 row per
    // lane; full rows: two halves of 4 sites x 2 rows)
    constexpr int NS = SKIP ? 8 : 4;
    if constexpr (SKIP) {
      // the sites' tile offsets and range checks from per-step parts: the
      // walk's position is in range, so a site is valid iff its row and
      // column moves stay inside; with an even radius the site rows keep
      // the field of row y and move its row half linearly (rad / 2 strip
      // rows), so an offset is one add of a row part (3 per step) and a
      // column part (3 per step) instead of a tile_off per site
      const bool up = row - rad >= c.row_min, dn = row + rad <= c.row_max;
      const bool lf = col - rad >= c.col_min, rt = col + rad <= c.col_max;
      const int y0 = c.oy + row + 2 * l, x0 = c.ox + col;
      uint32_t off[8];
      bool vv[8];
      if (stp > 0) {
        const int yb = (y0 & 1) * c.fsz + ((y0 >> 1) << 5), d16 = rad << 4;
        const int f32 = c.fh << 5;
        auto xo = [&](int x) { return __mul24(x >> 4, f32) + (x & 15); };
        const int xm = xo(x0 - rad), xc = xo(x0), xp = xo(x0 + rad);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int dr = site_dr(t), dc = site_dc(t);
          off[t] = (uint32_t)((dr < 0 ? yb - d16 : dr > 0 ? yb + d16 : yb) +
                              (dc < 0 ? xm : dc > 0 ? xp : xc));
        }
      } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) off[t] = tile_off(c, y0 + site_dr(t), x0 + site_dc(t));
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int dr = site_dr(t), dc = site_dc(t);
        vv[t] = active && (dr < 0 ? up : dr > 0 ? dn : true) && (dc < 0 ? lf : dc > 0 ? rt : true);
      }
      if (active) mine = lj_step_sad(s, trs, oob, off, vv, l);
    } else
    if (active)  // finished jobs' lanes off for the whole step (one branch; measured neutral, r04_v6)
#pragma unroll
    for (int h = 0; h < 8 / NS; ++h) {
      int rr[NS], cc[NS];
      bool vv[NS];
      uint32_t sd[NS];
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const int t = h * NS + i;
        rr[i] = row + site_dr(t) * rad;
        cc[i] = col + site_dc(t) * rad;
        vv[i] = active && cc[i] >= c.col_min && cc[i] <= c.col_max && rr[i] >= c.row_min &&
                rr[i] <= c.row_max;
      }
      lj_sads<SKIP, NS>(c, s, l, trs, oob, rr, cc, vv, sd);
#pragma unroll
      for (int i = 0; i < NS; ++i) mine = l == h * NS + i ? sd[i] : mine;
    }
    const uint32_t key =
        (((mine + mvsad_finish(c, mr, rl, cl_)) << 3) | (uint32_t)l) | (vl ? 0u : ~0u);
    const uint32_t kmin = group_min8(key);
    if (active) {
      ++steps;
      if (kmin < (best << 3)) {
        best = kmin >> 3;
        const int i = (int)(kmin & 7);
        row += site_dr(i) * rad;
        col += site_dc(i) * rad;
        offc = true;
      }
      if (!offc) ++center;
      if (--stp < 0) {  // this diamond_search_sad run is over
        if (l == 0) res[nres] = ((uint32_t)(uint16_t)row << 16) | (uint16_t)col;
        ++nres;
        ++searches;
        if (first) n = center;       // the first run's num00
        else if (center) n += center;
        first = false;
        if (n < further) {           // the next run, one step shorter
          ++n;
          row = srow;
          col = scol;
          best = c0;
          stp = kMaxSteps - (step_param + n) - 1;
          center = 0;
          offc = false;
        } else {
          active = false;
          stp = 0;  // a finished job keeps stepping in place at radius 1 (masked)
        }
      }
    }
  }
  wave_sync();
  if (!run) return;
  // var costs of the runs' results in order, strict "<" (full_pixel_diamond)
  for (int i = 0; i < nres; ++i) {
    const uint32_t p = res[i];
    const int r = (int16_t)(p >> 16), cc = (int16_t)(p & 0xFFFF);
    const int v = lj_var(c, s, l, r, cc);
    if (i == 0 || v < sme) {
      sme = v;
      br = r;
      bc = cc;
    }
  }
  if (want_cl) {  // calc_int_sad_list around (br, bc): centre, left, bottom, right, top
    int rr[5], cc[5];
    bool vv[5];
    uint32_t sd[5];
    MvRate m[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      rr[t] = br + (t == 2 ? 1 : t == 4 ? -1 : 0);
      cc[t] = bc + (t == 1 ? -1 : t == 3 ? 1 : 0);
      vv[t] = t == 0 ||
              (cc[t] >= c.col_min && cc[t] <= c.col_max && rr[t] >= c.row_min && rr[t] <= c.row_max);
      m[t] = mvsad_rate_dec(c, dec, vv[t] ? rr[t] : br, vv[t] ? cc[t] : bc);  // (in-range indices)
    }
    lj_sads<SKIP, 5>(c, s, l, trs, oob, rr, cc, vv, sd);
#pragma unroll
    for (int t = 0; t < 5; ++t)
      cl[t] = vv[t] ? (int)(sd[t] + mvsad_finish(c, m[t], rr[t], cc[t])) : INT_MAX;
  }
}

__device__ __forceinline__ void lj_jobs(
    const uint8_t* __restrict__ src, int ss, const uint8_t* __restrict__ ref, int rs,
    const LavishRefTiles& tiles, const Job* __restrict__ jobs, int njobs, int step_param,
    const LavishMvCostParams& cost, const int32_t* dec, int skip,
    LavishDiamondResult* __restrict__ out, int32_t* __restrict__ cost_lists, int j0,
    uint32_t* res);

// one group of WPG x 8 jobs: virtual workgroup vwg of nvwg (a multiple of 8)
template <int WPG>
__device__ __forceinline__ void lj_group(
    const uint8_t* __restrict__ src, int ss, const uint8_t* __restrict__ ref, int rs,
    const LavishRefTiles& tiles, const Job* __restrict__ jobs, int njobs, int step_param,
    const LavishMvCostParams& cost, const int32_t* dec, int skip,
    LavishDiamondResult* __restrict__ out, int32_t* __restrict__ cost_lists, int vwg, int nvwg) {
  __shared__ uint32_t res_s[WPG][kLjJobs][kMaxSteps];  // (LDS-addressed, not through a pointer)
  // XCD-aware: consecutive job groups (neighbouring blocks) share an XCD's L2
  const int wg = (vwg & 7) * (nvwg >> 3) + (vwg >> 3);
  const int lane = threadIdx.x & 63;
  const int wave = WPG == 1 ? 0 : threadIdx.x >> 6;
  const int j0 = (wg * WPG + wave) * kLjJobs;
  if (j0 >= njobs) return;
  lj_jobs(src, ss, ref, rs, tiles, jobs, njobs, step_param, cost, dec, skip, out, cost_lists, j0,
          res_s[wave][lane >> 3]);
}

// the eight jobs j0 .. j0 + 7 of one wave (res: this lane group's LDS slot
// for the runs' results)
__device__ __forceinline__ void lj_jobs(
    const uint8_t* __restrict__ src, int ss, const uint8_t* __restrict__ ref, int rs,
    const LavishRefTiles& tiles, const Job* __restrict__ jobs, int njobs, int step_param,
    const LavishMvCostParams& cost, const int32_t* dec, int skip,
    LavishDiamondResult* __restrict__ out, int32_t* __restrict__ cost_lists, int j0,
    uint32_t* res) {
  const int lane = threadIdx.x & 63;
  const int jg = lane >> 3, l = lane & 7;
  const int j = min(j0 + jg, njobs - 1);  // a surplus group repeats the last job, never stores
  const bool mine_job = j0 + jg < njobs;
  const Job jb = jobs[j];
  Ctx c;
  c.src = src + jb.src_off;
  c.ref = ref + jb.ref_off;
  c.ss = ss;
  c.rs = rs;
  c.col_min = jb.col_min;
  c.col_max = jb.col_max;
  c.row_min = jb.row_min;
  c.row_max = jb.row_max;
  c.ref_mv_row = jb.ref_mv_row;
  c.ref_mv_col = jb.ref_mv_col;
  c.full_ref_row = rawpel(jb.ref_mv_row);
  c.full_ref_col = rawpel(jb.ref_mv_col);
  c.cost_type = cost.mv_cost_type;
  c.sad_lambda = sad_lambda(cost.mv_cost_type);
  c.sse_lambda = sse_lambda(cost.mv_cost_type);
  c.sad_per_bit = cost.sad_per_bit;
  c.error_per_bit = cost.error_per_bit;
  const bool ent = cost.mv_cost_type == 0;
  c.mvjcost = ent ? cost.mvjcost : kZeroRate;
  c.mvcost0 = ent ? cost.mvcost[0] : kZeroRate;
  c.mvcost1 = ent ? cost.mvcost[1] : kZeroRate;
  c.tiles = tiles.data;
  c.fh = tiles.field_rows;
  c.fsz = (int)tiles.field_bytes;
  c.oy = (int)(jb.ref_off / rs);
  c.ox = (int)(jb.ref_off - (int64_t)c.oy * rs);
  // the tiled copy through a range-checked buffer descriptor (uniform:
  // kernel arguments only); `oob` = an offset past its end
  const int oob = (int)(2 * tiles.field_bytes);
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc((void*)tiles.data, 0, oob, 0x00020000);
  LjSrc s;
  load_row<4>(c.src + (int64_t)(2 * l) * ss, s.sk);
  load_row<4>(c.src + (int64_t)l * ss, s.fr[0]);
  load_row<4>(c.src + (int64_t)(l + 8) * ss, s.fr[1]);
  const bool want_cl = cost_lists != nullptr;
  int cl[5] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX, INT_MAX};
  int steps = 0, searches = 0, sme = 0;
  int br = jb.start_row, bc = jb.start_col;
  bool full = true;
  if (skip) {
    lj_pass<true>(c, s, l, trs, oob, dec, true, step_param, want_cl, res, steps, searches, br, bc,
                  sme, cl);
    // quality check of the row-skipping search (mcomp.c:1840-1867): sad and
    // sad_skip at the result, rows l and l + 8 of lane l (same parity as l)
    uint32_t all = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint32_t t[4];
      load_row<4>(c.ref + (int64_t)(br + l + 8 * k) * rs + bc, t);
#pragma unroll
      for (int i = 0; i < 4; ++i) all = sad4(s.fr[k][i], t[i], all);
    }
    const int sad = (int)group_sum8(all);
    const int ssad = (int)(2 * group_sum8((l & 1) ? 0u : all));
    full = sad > 16 && abs(ssad - sad) * 10 >= max(sad, 1) * 9;
    if (full) {
      br = jb.start_row;
      bc = jb.start_col;
    }
  }
  if (__builtin_amdgcn_ballot_w64(full) != 0)
    lj_pass<false>(c, s, l, trs, oob, dec, full, step_param, want_cl, res, steps, searches, br, bc,
                   sme, cl);
  if (!mine_job) return;
  if (l == 0) {
    LavishDiamondResult r;
    r.best_row = (int16_t)br;
    r.best_col = (int16_t)bc;
    r.bestsme = sme;
    r.steps = steps;
    r.searches = searches;
    out[j] = r;
  }
  if (want_cl && l < 5) {
    const int v = l == 0 ? cl[0] : l == 1 ? cl[1] : l == 2 ? cl[2] : l == 3 ? cl[3] : cl[4];
    cost_lists[5 * (int64_t)j + l] = v;
  }
}

// nvwg virtual workgroups over gridDim.x (<= nvwg, both multiples of 8, so a
// virtual workgroup runs on the XCD of its first): with a smaller grid the
// search holds fewer CU slots while a concurrent leg runs beside it
// WPG waves per workgroup.  1 would let the dispatcher refill a SIMD slot as
// soon as one wave's eight jobs are done; measured, four-wave workgroups are
// faster (0.294 vs 0.303 ms, profiles/r04_v5_c3_wpg_ab.txt): the four waves
// of a workgroup are consecutive job groups on one CU, sharing its L1
#ifndef LAVISH_LJ_WAVES
#define LAVISH_LJ_WAVES 4  // minimum waves per SIMD requested (VGPR budget 512 / this)
#endif
template <int WPG>
__global__ __launch_bounds__(64 * WPG, LAVISH_LJ_WAVES) void diamond_lj_kernel(
    const uint8_t* __restrict__ src, int ss, const uint8_t* __restrict__ ref, int rs,
    LavishRefTiles tiles, const Job* __restrict__ jobs, int njobs, int step_param,
    LavishMvCostParams cost, const int32_t* dec, int skip, LavishDiamondResult* __restrict__ out,
    int32_t* __restrict__ cost_lists, int nvwg) {
  for (int v = blockIdx.x; v < nvwg; v += gridDim.x)
    lj_group<WPG>(src, ss, ref, rs, tiles, jobs, njobs, step_param, cost, dec, skip, out,
                  cost_lists, v, nvwg);
}

// The capped grid with work pulled from queues: beside C2 the search runs in
// `cap` workgroups (lavish_set_search_workgroup_cap) that each process many
// 8-job wave units.  Dealt statically (grid-stride over virtual workgroups),
// ceil(groups / cap) rounds set the leg's length while most workgroups sit
// idle in the last round (1760 groups over 512 workgroups: 223 do 4, 289 do
// 3) and every wave of a workgroup waits for its slowest unit.  Here every
// wave pulls its next unit from a queue with one returning atomic: the
// units of XCD label x = blockIdx % 8 (blocks b and b + 8 share an XCD, so
// neighbouring blocks' reference tiles stay in one L2, as with the static
// mapping) are the contiguous range [units x / 8, units (x + 1) / 8); a
// label's workgroups drain it together.  queue: 8 counters 16 ints apart,
// zero at launch (mvcost_dec_kernel or lj_queue_zero clears them on the
// same stream).  The order of the units changes no result.
constexpr int kLjQueueStride = 16;  // ints between two labels' counters (64 B)

template <int WPG>
__global__ __launch_bounds__(64 * WPG, LAVISH_LJ_WAVES) void diamond_lj_dyn_kernel(
    const uint8_t* __restrict__ src, int ss, const uint8_t* __restrict__ ref, int rs,
    LavishRefTiles tiles, const Job* __restrict__ jobs, int njobs, int step_param,
    LavishMvCostParams cost, const int32_t* dec, int skip, LavishDiamondResult* __restrict__ out,
    int32_t* __restrict__ cost_lists, int* __restrict__ queue) {
  __shared__ uint32_t res_s[WPG][kLjJobs][kMaxSteps];
  const int units = (njobs + kLjJobs - 1) / kLjJobs;
  const int x = blockIdx.x & 7;
  const int u0 = units * x / 8, u1 = units * (x + 1) / 8;
  const int lane = threadIdx.x & 63;
  const int wave = WPG == 1 ? 0 : threadIdx.x >> 6;
  uint32_t* res = res_s[wave][lane >> 3];
  int* q = queue + x * kLjQueueStride;
  for (;;) {
    int t = 0;
    if (lane == 0) t = __hip_atomic_fetch_add(q, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __builtin_amdgcn_readfirstlane(t);
    if (u0 + t >= u1) break;  // every wave of the label ends here once the range is drained
    lj_jobs(src, ss, ref, rs, tiles, jobs, njobs, step_param, cost, dec, skip, out, cost_lists,
            (u0 + t) * kLjJobs, res);
  }
}

__global__ void lj_queue_zero(int* __restrict__ queue) {
  if (threadIdx.x < 8 * kLjQueueStride) queue[threadIdx.x] = 0;
}

// ---------------------------------------------------------------------------
// C2 + C3 in one launch (lavish_txq_frame_search): the <= 16-point class of
// lavish_txq_frame (txq_multi_body<0>) and the 16x16 DIAMOND search's job
// groups (lj_group) in one grid.  The dispatch order -- units of 8
// consecutive workgroups, so a unit keeps the XCD congruence both mappings
// rely on -- places a search unit every `every` units from the start and the
// transform workgroups around them: the long-lived search waves (a dependent
// chain of L2 round trips per job) take a bounded share of the CU slots while
// the transform's write stream keeps the rest, instead of two streams'
// workgroups racing for the slots.  VGPRs: the larger of the two bodies
// (both 115), LDS: the class's 37 KB + the search's result slots.
struct LjLaunch {
  const uint8_t* src;
  int ss;
  const uint8_t* ref;
  int rs;
  LavishRefTiles tiles;
  const Job* jobs;
  int njobs, step_param;
  LavishMvCostParams cost;
  const int32_t* dec;
  int skip;
  LavishDiamondResult* out;
  int32_t* cost_lists;
  int nvwg;   // the search's virtual workgroups (a multiple of 8)
  int units;  // nvwg / 8
  int every;  // a search unit every `every` units of the dispatch order
};

__global__ __launch_bounds__(256, 4) void txq_search_kernel(TxqDispatch d, TxqArgs a0, TxqArgs a1,
                                                            TxqArgs a2, TxqArgs a3, TxqArgs a4,
                                                            TxqArgs a5, TxqArgs a6, TxqArgs a7,
                                                            TxqArgs a8, LjLaunch c) {
  __shared__ __attribute__((aligned(16))) char lds[class_lds(0)];
  const int u = blockIdx.x >> 3, x = blockIdx.x & 7;
  const int k = u / c.every;
  if (u - k * c.every == 0 && k < c.units) {
    lj_group<4>(c.src, c.ss, c.ref, c.rs, c.tiles, c.jobs, c.njobs, c.step_param, c.cost, c.dec,
                c.skip, c.out, c.cost_lists, k * 8 + x, c.nvwg);
    return;
  }
  const int before = min((u + c.every - 1) / c.every, c.units);  // search units in 0 .. u - 1
  txq_multi_body<0>(d, a0, a1, a2, a3, a4, a5, a6, a7, a8, (u - before) * 8 + x, lds);
}

// the decimated entropy cost tables of mvsad_rate_dec
// (+ the search queue's counters zeroed, when given)
__global__ __launch_bounds__(256) void mvcost_dec_kernel(const int32_t* __restrict__ mvcost0,
                                                         const int32_t* __restrict__ mvcost1,
                                                         int32_t* __restrict__ dec,
                                                         int* __restrict__ queue) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (queue != nullptr && i < 8 * kLjQueueStride) queue[i] = 0;
  if (i >= 2 * kMvDecN) return;
  const int k = (i % kMvDecN) - kMvDecHalf;
  dec[i] = (i < kMvDecN ? mvcost0 : mvcost1)[8 * k];
}

thread_local StreamScratch t_mvdec;

// at most this many workgroups for the 16x16 DIAMOND search (rounded to 8;
// 0: one per 32 jobs): lavish_set_search_workgroup_cap
static std::atomic<int> g_lj_cap{0};
static int lj_grid_cap() { return g_lj_cap.load(std::memory_order_relaxed); }
// a capped grid: 1 = units pulled from queues (default), 0 = the static
// grid-stride (lavish_set_search_schedule, A/B)
static std::atomic<int> g_lj_queue{1};

template <int W, int H, bool TL>
void launch_tl(const uint8_t* src, int ss, const uint8_t* ref, int rs, const LavishRefTiles& t,
               const LavishDiamondJob* jobs, int njobs, int step_param,
               const LavishMvCostParams& cost, int skip, int method, LavishDiamondResult* out,
               int32_t* cost_lists, hipStream_t s, uint8_t* sdf_kind = nullptr) {
  int nwg = (njobs + kDkWaves - 1) / kDkWaves;
  nwg = (nwg + 7) & ~7;
  if (diamond_method(method))
    hipLaunchKernelGGL((diamond_kernel<W, H, false, TL>), dim3(nwg), dim3(64 * kDkWaves), 0, s, src, ss,
                       ref, rs, t, (const Job*)jobs, njobs, step_param, cost, skip, method, out,
                       cost_lists, sdf_kind);
  else
    hipLaunchKernelGGL((diamond_kernel<W, H, true, TL>), dim3(nwg), dim3(64 * kDkWaves), 0, s, src, ss,
                       ref, rs, t, (const Job*)jobs, njobs, step_param, cost, skip, method, out,
                       cost_lists, sdf_kind);
}

thread_local StreamScratch t_mesh;

// the search (diamond_kernel, recording each job's sdf) then mesh_kernel
template <int W, int H>
void launch_mesh(const uint8_t* src, int ss, const uint8_t* ref, int rs, const LavishRefTiles* t,
                 const LavishDiamondJob* jobs, int njobs, int step_param,
                 const LavishMvCostParams& cost, int skip, int method, LavishDiamondResult* out,
                 int32_t* cost_lists, const MeshArgs& m, hipStream_t s) {
  uint8_t* kind = (uint8_t*)t_mesh.acquire((size_t)njobs, s);
  if (W <= 16 && t != nullptr)
    launch_tl<W, H, (W <= 16)>(src, ss, ref, rs, *t, jobs, njobs, step_param, cost, skip, method,
                               out, cost_lists, s, kind);
  else
    launch_tl<W, H, false>(src, ss, ref, rs, LavishRefTiles{}, jobs, njobs, step_param, cost,
                           skip, method, out, cost_lists, s, kind);
  hipLaunchKernelGGL((mesh_kernel<W, H>), dim3((njobs + kDkWaves - 1) / kDkWaves),
                     dim3(64 * kDkWaves), 0, s, src, ss, ref, rs, (const Job*)jobs, njobs, cost,
                     m, (const uint8_t*)kind, out, cost_lists);
  t_mesh.release(s);
}

template <int W, int H>
void launch(const uint8_t* src, int ss, const uint8_t* ref, int rs, const LavishRefTiles* t,
            const LavishDiamondJob* jobs, int njobs, int step_param,
            const LavishMvCostParams& cost, int skip, int method, LavishDiamondResult* out,
            int32_t* cost_lists, hipStream_t s) {
  if constexpr (W <= 16) {
    if (t != nullptr) {
      if constexpr (W == 16 && H == 16) {
        if (method == kDiamond) {  // eight jobs per wave
          const int waves = (njobs + kLjJobs - 1) / kLjJobs;
          constexpr int wpg = 4;
          const int nwg = (((waves + wpg - 1) / wpg) + 7) & ~7;
          const int cap = lj_grid_cap();
          const int grid = cap > 0 && cap < nwg ? cap : nwg;
          // a capped grid pulls its units from the queues (diamond_lj_dyn_kernel)
          const bool dyn = grid < nwg && g_lj_queue.load(std::memory_order_relaxed);
          constexpr size_t kDecBytes = 2 * kMvDecN * sizeof(int32_t);
          const size_t qbytes = dyn ? 8 * kLjQueueStride * sizeof(int) : 0;
          int32_t* dec = nullptr;
          int* queue = nullptr;
          char* scr = nullptr;
          if (cost.mv_cost_type == 0 || dyn) {
            scr = (char*)t_mvdec.acquire(kDecBytes + qbytes, s);
            if (dyn) queue = (int*)(scr + kDecBytes);
          }
          if (cost.mv_cost_type == 0) {
            dec = (int32_t*)scr;
            hipLaunchKernelGGL(mvcost_dec_kernel, dim3((2 * kMvDecN + 255) / 256), dim3(256), 0,
                               s, cost.mvcost[0], cost.mvcost[1], dec, queue);
          } else if (dyn) {
            hipLaunchKernelGGL(lj_queue_zero, dim3(1), dim3(8 * kLjQueueStride), 0, s, queue);
          }
          if (dyn)
            hipLaunchKernelGGL(diamond_lj_dyn_kernel<wpg>, dim3(grid), dim3(64 * wpg), 0, s, src,
                               ss, ref, rs, *t, (const Job*)jobs, njobs, step_param, cost,
                               (const int32_t*)dec, skip, out, cost_lists, queue);
          else
            hipLaunchKernelGGL(diamond_lj_kernel<wpg>, dim3(grid), dim3(64 * wpg), 0, s, src, ss,
                               ref, rs, *t, (const Job*)jobs, njobs, step_param, cost,
                               (const int32_t*)dec, skip, out, cost_lists, nwg);
          if (scr) t_mvdec.release(s);
          return;
        }
      }
      launch_tl<W, H, true>(src, ss, ref, rs, *t, jobs, njobs, step_param, cost, skip, method,
                            out, cost_lists, s);
      return;
    }
  }
  const LavishRefTiles none{};
  launch_tl<W, H, false>(src, ss, ref, rs, none, jobs, njobs, step_param, cost, skip, method,
                         out, cost_lists, s);
}

// LavishRefTiles copy through LDS, both sides coalesced: a workgroup takes
// field f, strips [k0, k0 + 8) and field rows [fy0, fy0 + 32): it reads the
// 32 source rows' 144-byte segments (the 8 strips + the 16 bytes the last
// strip row overlaps into) as 16-byte chunks, then writes the 8 strips' 1 KB
// runs (32 field rows x 32 bytes each).  Bytes past the row end or past the
// last row are zero.
constexpr int kTilesK = 8, kTilesF = 32, kTilesC = kTilesK + 1;  // chunks per row segment
__global__ __launch_bounds__(256) void ref_tiles_kernel(const uint8_t* __restrict__ ref,
                                                        int stride, int rows, int nstrips,
                                                        int fh, uint8_t* __restrict__ out,
                                                        int ktiles, int ftiles) {
  __shared__ u32x4 seg[kTilesF][kTilesC];
  const int t = threadIdx.x;
  int b = blockIdx.x;
  const int kt = b % ktiles;
  b /= ktiles;
  const int ft = b % ftiles;
  const int f = b / ftiles;
  const int k0 = kt * kTilesK, fy0 = ft * kTilesF;
  for (int idx = t; idx < kTilesF * kTilesC; idx += 256) {
    const int i = idx / kTilesC, m = idx - i * kTilesC;
    const int y = 2 * (fy0 + i) + f, x = 16 * (k0 + m);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (y < rows && x < stride) {
      const uint8_t* p = ref + (int64_t)y * stride + x;
      if (x + 16 <= stride) {
        const u32x4u w = *(const __attribute__((address_space(1))) u32x4u*)p;
        v = u32x4{w.x, w.y, w.z, w.w};
      } else {
        uint32_t q[4] = {0u, 0u, 0u, 0u};
        for (int j = 0; j < 16 && x + j < stride; ++j) q[j >> 2] |= (uint32_t)p[j] << (8 * (j & 3));
        v = u32x4{q[0], q[1], q[2], q[3]};
      }
    }
    seg[i][m] = v;
  }
  __syncthreads();
  for (int q = t; q < kTilesK * kTilesF * 2; q += 256) {
    const int kk = q >> 6, i = (q >> 1) & (kTilesF - 1), h = q & 1;
    const int k = k0 + kk, fy = fy0 + i;
    if (k < nstrips && fy < fh)
      *(u32x4*)(out + ((((int64_t)f * nstrips + k) * fh + fy) << 5) + 16 * h) = seg[i][kk + h];
  }
}

}  // namespace

int fullpel_batch(const uint8_t* src, int src_stride, const uint8_t* ref, int ref_stride, int w,
                  int h, const LavishDiamondJob* jobs, int njobs, int method, int step_param,
                  const LavishMvCostParams* cost, int use_downsampled_sad,
                  LavishDiamondResult* out, int32_t* cost_lists, hipStream_t s,
                  const LavishRefTiles* tiles = nullptr, const LavishMeshParams* mesh = nullptr) {
  if (njobs <= 0) return 0;
  // the mesh refinement: nothing to do unless it can run (run_mesh_search,
  // or the variance trigger after NSTEP / NSTEP_8PT) and the first pattern is
  // legal (full_pixel_exhaustive returns INT_MAX otherwise, changing nothing)
  MeshArgs ma{};
  bool with_mesh = false;
  if (mesh != nullptr) {
    const LavishMeshParams& mp = *mesh;
    const bool nstep = method == kNstep || method == kNstep8;
    const bool legal = mp.range[0] >= 7 && mp.range[0] <= 256 && mp.interval[0] >= 1 &&
                       mp.interval[0] <= mp.range[0];
    if ((mp.run_mesh_search || nstep) && legal) {
      // every later pass the walk can reach needs a positive interval (the
      // reference's would not end); passes follow while the interval is not 1
      for (int i = 1; i < 4; ++i) {
        if (mp.interval[i] < 1) return -6;
        if (mp.interval[i] == 1) break;
      }
      with_mesh = true;
      ma.run = mp.run_mesh_search != 0;
      ma.nstep = nstep;
      const int bw = 31 - __builtin_clz((unsigned)(w >> 2) | 1u);
      const int bh = 31 - __builtin_clz((unsigned)(h >> 2) | 1u);
      ma.thr = mp.force_mesh_thresh >> (10 - (bw + bh));  // mi_size_*_log2
      ma.prune = mp.prune_mesh_search != 0;
      ma.diff = mp.mesh_search_mv_diff_threshold;
      ma.intra = mp.is_intra_mode != 0;
      ma.fine = mp.fine_search_interval != 0;
      for (int i = 0; i < 4; ++i) {
        ma.range[i] = mp.range[i];
        ma.interval[i] = mp.interval[i];
      }
    }
  }
  if (tiles != nullptr && (tiles->data == nullptr || tiles->stride != ref_stride)) return -5;
  if (step_param < 0 || step_param >= method_steps(method)) return -1;
  if (cost == nullptr || cost->mv_cost_type < 0 || cost->mv_cost_type > 4) return -2;
  if (cost->mv_cost_type == 0 &&
      (cost->mvjcost == nullptr || cost->mvcost[0] == nullptr || cost->mvcost[1] == nullptr))
    return -2;
  // every method of av1_full_pixel_search but CLAMPED_DIAMOND (3)
  if (method < 0 || method > kVfastDiamond || method == 3) return -4;
#define LAVISH_DIA_CASE(W, H)                                                                 \
  if (w == W && h == H) {                                                                     \
    if (with_mesh)                                                                            \
      launch_mesh<W, H>(src, src_stride, ref, ref_stride, tiles, jobs, njobs, step_param,     \
                        *cost, use_downsampled_sad, method, out, cost_lists, ma, s);          \
    else                                                                                      \
      launch<W, H>(src, src_stride, ref, ref_stride, tiles, jobs, njobs, step_param, *cost,   \
                   use_downsampled_sad, method, out, cost_lists, s);                          \
    LAVISH_CHECK(hipGetLastError());                                                          \
    return 0;                                                                                 \
  }
  LAVISH_ENCODER_BLOCK_SIZES(LAVISH_DIA_CASE)
#undef LAVISH_DIA_CASE
  return -3;
}

}  // namespace lavish

using namespace lavish;

#if LAVISH_TPL_PROF
extern "C" int lavish_dbg_tpl_prof(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(lavish::g_tpl_prof), 16 * 8) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(lavish::g_tpl_prof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

extern "C" int lavish_set_search_schedule(int queued) {
  if (queued != 0 && queued != 1) return -1;
  lavish::g_lj_queue.store(queued, std::memory_order_relaxed);
  return 0;
}

extern "C" int lavish_set_search_workgroup_cap(int workgroups) {
  if (workgroups < 0) return -1;
  lavish::g_lj_cap.store((workgroups + 7) & ~7, std::memory_order_relaxed);
  return 0;
}

extern "C" int64_t lavish_tpl_motion_sync_ints(int nrefs, int rows) {
  if (nrefs <= 0 || rows <= 0) return -1;
  return 2;
}

extern "C" int lavish_tpl_motion_search(const uint8_t* src, int src_stride, const uint8_t* ref,
                                        int ref_stride, const LavishDiamondJob* jobs, int cols,
                                        int rows, int nrefs, const LavishTplMvParams* p,
                                        const LavishMvCostParams* cost,
                                        const int32_t* third_pass_mvs, int32_t* mvs,
                                        LavishDiamondResult* out, int32_t* cost_lists,
                                        int32_t* centers, int32_t* sync, void* stream) {
  if (cols <= 0 || rows <= 0 || nrefs <= 0) return cols == 0 || rows == 0 || nrefs == 0 ? 0 : -1;
  if (p == nullptr || jobs == nullptr || mvs == nullptr || out == nullptr || sync == nullptr)
    return -1;
  if ((int64_t)cols * rows * nrefs >= ((int64_t)1 << 31)) return -1;
  if (p->subpel_force_stop != 3) return -6;  // FULL_PEL only (speed >= 5)
  if (p->prune_starting_mv < 0 || p->prune_starting_mv > 3) return -1;
  if (p->skip_alike_starting_mv < 0 || p->skip_alike_starting_mv > 2) return -1;
  if (p->step_param < 0) return -1;
  if (cost == nullptr || cost->mv_cost_type < 0 || cost->mv_cost_type > 4) return -2;
  if (cost->mv_cost_type == 0 &&
      (cost->mvjcost == nullptr || cost->mvcost[0] == nullptr || cost->mvcost[1] == nullptr))
    return -2;
  const int m = p->search_method;
  if (m != kDiamond && m != kBigdia && m != kFastDiamond && m != kFastBigdia &&
      m != kVfastDiamond)
    return -4;
  hipStream_t s = (hipStream_t)stream;
  LAVISH_CHECK(hipMemsetAsync(sync, 0, sizeof(int32_t) * 2, s));
  LAVISH_CHECK(hipMemsetD32Async((hipDeviceptr_t)mvs, kInvalidMv, (size_t)cols * rows * nrefs, s));
  TplMvArgs a;
  a.src = src;
  a.ref = ref;
  a.ss = src_stride;
  a.rs = ref_stride;
  a.jobs = (const Job*)jobs;
  a.cols = cols;
  a.rows = rows;
  a.nrefs = nrefs;
  a.step_param = min(p->step_param, kMaxSteps - 2);  // motion_estimation (tpl_model.c:270-271)
  a.skip = p->use_downsampled_sad;
  a.method = m;
  a.prune = p->prune_starting_mv;
  a.alike_thr = p->skip_alike_starting_mv == 0 ? 1 : p->skip_alike_starting_mv == 1 ? 64 : 128;
  a.cost = *cost;
  a.third = third_pass_mvs;
  a.mvs = mvs;
  a.out = out;
  a.cost_lists = cost_lists;
  a.centers = centers;
  a.sync = sync;
  const dim3 grid((unsigned)(nrefs * rows));
  if (m == kDiamond)
    hipLaunchKernelGGL(tpl_mv_kernel<false>, grid, dim3(128), 0, s, a);
  else
    hipLaunchKernelGGL(tpl_mv_kernel<true>, grid, dim3(128), 0, s, a);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

static LavishMvCostParams l1_cost(int mv_cost_type) {
  LavishMvCostParams c = {};
  // the L1 entry points never took MV_COST_ENTROPY (it needs the tables)
  c.mv_cost_type = mv_cost_type == 0 ? -1 : mv_cost_type;
  return c;
}

extern "C" int lavish_full_pixel_search_batch(const uint8_t* src, int src_stride,
                                              const uint8_t* ref, int ref_stride, int w, int h,
                                              const LavishDiamondJob* jobs, int njobs,
                                              int search_method, int step_param,
                                              const LavishMvCostParams* cost,
                                              int use_downsampled_sad, LavishDiamondResult* out,
                                              int32_t* cost_lists, void* stream) {
  return fullpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, search_method,
                       step_param, cost, use_downsampled_sad, out, cost_lists,
                       (hipStream_t)stream);
}

extern "C" int lavish_full_pixel_search_batch_mesh(
    const uint8_t* src, int src_stride, const uint8_t* ref, int ref_stride,
    const LavishRefTiles* tiles, int w, int h, const LavishDiamondJob* jobs, int njobs,
    int search_method, int step_param, const LavishMvCostParams* cost, int use_downsampled_sad,
    const LavishMeshParams* mesh, LavishDiamondResult* out, int32_t* cost_lists, void* stream) {
  return fullpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, search_method,
                       step_param, cost, use_downsampled_sad, out, cost_lists,
                       (hipStream_t)stream, tiles, mesh);
}

static int64_t tiles_nstrips(int stride) { return (stride + 15) / 16; }

extern "C" int64_t lavish_ref_tiles_bytes(int stride, int rows) {
  if (stride <= 0 || rows <= 0) return -1;
  return 2 * tiles_nstrips(stride) * ((rows + 1) / 2) * 32;
}

extern "C" int lavish_ref_tiles_build(const uint8_t* ref, int stride, int rows, uint8_t* data,
                                      LavishRefTiles* tiles, void* stream) {
  const int64_t bytes = lavish_ref_tiles_bytes(stride, rows);
  if (ref == nullptr || data == nullptr || tiles == nullptr || bytes <= 0) return -1;
  if (bytes >= ((int64_t)1 << 31)) return -1;  // 32-bit offsets in the search kernels
  const int nstrips = (int)tiles_nstrips(stride), fh = (rows + 1) / 2;
  tiles->data = data;
  tiles->field_bytes = (int64_t)nstrips * fh * 32;
  tiles->field_rows = fh;
  tiles->stride = stride;
  const int ktiles = (nstrips + kTilesK - 1) / kTilesK, ftiles = (fh + kTilesF - 1) / kTilesF;
  hipLaunchKernelGGL(ref_tiles_kernel, dim3((unsigned)(2 * ktiles * ftiles)), dim3(256), 0,
                     (hipStream_t)stream, ref, stride, rows, nstrips, fh, data, ktiles, ftiles);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

extern "C" int lavish_full_pixel_search_batch_tiled(
    const uint8_t* src, int src_stride, const uint8_t* ref, int ref_stride,
    const LavishRefTiles* tiles, int w, int h, const LavishDiamondJob* jobs, int njobs,
    int search_method, int step_param, const LavishMvCostParams* cost, int use_downsampled_sad,
    LavishDiamondResult* out, int32_t* cost_lists, void* stream) {
  return fullpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, search_method,
                       step_param, cost, use_downsampled_sad, out, cost_lists,
                       (hipStream_t)stream, tiles);
}

extern "C" int lavish_txq_frame_search(
    const int16_t* residual, int stride, int width, int height, uint32_t size_mask,
    const uint32_t* type_masks, int bit_depth, int quant_kind, const LavishQuantParams* qp,
    int32_t* const* qcoeff, int32_t* const* dqcoeff, uint16_t* const* eob, const uint8_t* src,
    int src_stride, const uint8_t* ref, int ref_stride, const LavishRefTiles* tiles,
    const LavishDiamondJob* jobs, int njobs, int step_param, const LavishMvCostParams* cost,
    int use_downsampled_sad, LavishDiamondResult* out, int32_t* cost_lists, int every,
    void* stream) {
  const hipStream_t s = (hipStream_t)stream;
  if (every < 1) return -6;
  if (tiles == nullptr || tiles->data == nullptr || tiles->stride != ref_stride) return -5;
  if (step_param < 0 || step_param >= kMaxSteps) return -1;
  if (cost == nullptr || cost->mv_cost_type < 0 || cost->mv_cost_type > 4) return -2;
  if (cost->mv_cost_type == 0 &&
      (cost->mvjcost == nullptr || cost->mvcost[0] == nullptr || cost->mvcost[1] == nullptr))
    return -2;
  // C2: every requested size outside the <= 16-point class as lavish_txq_frame
  // runs it (the 64-point sizes, then the 32-point class's launch)
  uint32_t cls0 = 0;
  for (int t = 0; t < 19; ++t)
    if (((size_mask >> t) & 1) && tx_w(t) <= 32 && tx_h(t) <= 32 && !txq_class(t)) cls0 |= 1u << t;
  int rc = 0;
  if (size_mask & ~cls0) {
    rc = txq_frame(residual, stride, width, height, size_mask & ~cls0, type_masks, bit_depth,
                   quant_kind, qp, qcoeff, dqcoeff, eob, s);
    if (rc) return rc;
  }
  TxqMulti m;
  int g = 0;
  rc = txq_frame_plan(residual, stride, width, height, cls0, type_masks, bit_depth, quant_kind, qp,
                      qcoeff, dqcoeff, eob, 0, m, g);
  if (rc) return rc;
  LjLaunch c{};
  c.src = src;
  c.ss = src_stride;
  c.ref = ref;
  c.rs = ref_stride;
  c.tiles = *tiles;
  c.jobs = (const Job*)jobs;
  c.njobs = njobs > 0 ? njobs : 0;
  c.step_param = step_param;
  c.cost = *cost;
  c.skip = use_downsampled_sad;
  c.out = out;
  c.cost_lists = cost_lists;
  const int waves = (c.njobs + kLjJobs - 1) / kLjJobs;
  c.nvwg = (((waves + 3) / 4) + 7) & ~7;
  c.units = c.nvwg / 8;
  if (c.units > 0 && cost->mv_cost_type == 0) {
    c.dec = (const int32_t*)t_mvdec.acquire(2 * kMvDecN * sizeof(int32_t), s);
    hipLaunchKernelGGL(mvcost_dec_kernel, dim3((2 * kMvDecN + 255) / 256), dim3(256), 0, s,
                       cost->mvcost[0], cost->mvcost[1], (int32_t*)c.dec, (int*)nullptr);
  }
  // the search units must all lie inside the grid: units * every may not
  // pass the grid's units (clamp the spacing)
  const int u2 = g / 8, ut = u2 + c.units;
  c.every = c.units > 1 ? min(every, max(1, (ut - 1) / (c.units - 1))) : every;
  if (ut > 0)
    hipLaunchKernelGGL(txq_search_kernel, dim3(ut * 8), dim3(256), 0, s, m.d, m.a[0], m.a[1],
                       m.a[2], m.a[3], m.a[4], m.a[5], m.a[6], m.a[7], m.a[8], c);
  LAVISH_CHECK(hipGetLastError());
  if (c.dec) t_mvdec.release(s);
  return 0;
}

extern "C" int lavish_diamond_search_batch(const uint8_t* src, int src_stride, const uint8_t* ref,
                                           int ref_stride, int w, int h,
                                           const LavishDiamondJob* jobs, int njobs,
                                           int step_param, int mv_cost_type,
                                           int use_downsampled_sad, LavishDiamondResult* out,
                                           void* stream) {
  const LavishMvCostParams c = l1_cost(mv_cost_type);
  return fullpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, kDiamond, step_param,
                       &c, use_downsampled_sad, out, nullptr, (hipStream_t)stream);
}

extern "C" int lavish_fast_bigdia_search_batch(const uint8_t* src, int src_stride,
                                               const uint8_t* ref, int ref_stride, int w, int h,
                                               const LavishDiamondJob* jobs, int njobs,
                                               int step_param, int mv_cost_type,
                                               int use_downsampled_sad,
                                               LavishDiamondResult* out, void* stream) {
  const LavishMvCostParams c = l1_cost(mv_cost_type);
  return fullpel_batch(src, src_stride, ref, ref_stride, w, h, jobs, njobs, kFastBigdia,
                       step_param, &c, use_downsampled_sad, out, nullptr, (hipStream_t)stream);
}
