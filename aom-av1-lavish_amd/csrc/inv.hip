// inv.hip -- batched inverse 2-D transform + reconstruction add for gfx950
// (SURVEY.md section 8 row a17).
//
// Reference, per block: av1_inverse_transform_block (av1/common/idct.c:304-322)
// -> av1_inv_txfm_add_c (u8 through a u16 copy, :281-302) /
// av1_highbd_inv_txfm_add (:212-279) -> inv_txfm2d_add_facade ->
// inv_txfm2d_add_c (av1/common/av1_inv_txfm2d.c:234-316): rows (x NewInvSqrt2
// for 2:1 shapes, clamp to bd+8, row 1-D, round shift[0]), columns (lr flip,
// clamp to max(bd+6, 16), column 1-D, round shift[1], ud flip,
// highbd_clip_pixel_add).  64-point sizes read the packed 32x32 quadrant.
//
// Here one wave64 owns P = 64 / min(W,H) blocks ("tile") of one TX size:
//   dqcoeff (HBM, coalesced) -> LDS -> row transforms (one row per lane per
//   pass, registers) -> LDS (padded rows) -> column transforms -> add to the
//   destination pixels (each lane one column, rows coalesced across lanes).
// The 1-D transforms are the same straight-line code as the forward kernels
// (txfm_dev.h, inv_1d), with the reference's per-stage clamps at the bit
// depth's ranges (template BDI).
#include "lavish_internal.h"
#include "txfm_dev.h"

namespace lavish {
namespace {

struct InvJob {
  int64_t dst_off;
  int64_t coeff_off;
  int32_t tx_type;
  int32_t eob;
};
static_assert(sizeof(InvJob) == sizeof(LavishInvJob), "job layout");

constexpr uint8_t kVtx[16] = {0, 1, 0, 1, 2, 0, 2, 1, 2, 3, 0, 3, 1, 3, 2, 3};
constexpr uint8_t kHtx[16] = {0, 0, 1, 1, 0, 2, 2, 2, 1, 3, 3, 0, 3, 1, 3, 2};
constexpr uint32_t pack2(const uint8_t (&v)[16]) {
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r |= (uint32_t)v[i] << (2 * i);
  return r;
}
constexpr uint32_t kVtxP = pack2(kVtx), kHtxP = pack2(kHtx);

template <int W, int H>
struct InvTile {
  static constexpr int MN = W < H ? W : H;
  static constexpr int P = 64 / MN;            // blocks per wave
  static constexpr int CPT = W / MN;           // column transforms per lane
  static constexpr int KW = W > 32 ? 32 : W;   // stored coefficient columns
  static constexpr int KH = H > 32 ? 32 : H;   // stored coefficient rows
  // row transforms per lane: only the KH stored rows (rows >= 32 of a
  // 64-high block hold zero coefficients, so their row outputs are zero and
  // the column transforms take them as compile-time zeros)
  static constexpr int RPT = (P * KH + 63) / 64;
  static constexpr int NC = KW * KH;           // stored words per block
  static constexpr int T1S = W + 1;
};

// inv_1d with the consumer of the output inlined into each kind's branch:
// one output array per branch, so no pointer to a merged private array
// survives (a shared `out` written by three branches and read after them
// was left in scratch by the optimiser)
template <int N, int BIT, int RNG, typename F>
__device__ __forceinline__ void inv_1d_then(int kind, const int32_t* in, F&& use) {
  if (kind == 0) {
    int32_t o[N];
    idct<N, BIT, RNG>(in, o);
    use(o);
  } else if (kind == 1) {
    if constexpr (N <= 16) {
      int32_t o[N];
      iadst<N, BIT, RNG>(in, o);
      use(o);
    }
  } else {
    if constexpr (N <= 32) {
      int32_t o[N];
      iidentity<N>(in, o);
      use(o);
    }
  }
}

// LDS of one tile: the jobs, the staged coefficients and the row outputs
// (rows >= KH are zero, not stored); bytes
template <int W, int H>
constexpr int inv_lds_bytes() {
  using T = InvTile<W, H>;
  return (int)(T::P * sizeof(InvJob)) + 4 * T::P * T::NC + 4 * T::P * T::KH * T::T1S;
}

// one tile: the P jobs from j0; lds: inv_lds_bytes<W, H>() bytes, 8-aligned
template <int W, int H, int BDI, typename PIX>
__device__ __forceinline__ void inv_tile(const int32_t* __restrict__ dq,
                                         const InvJob* __restrict__ jobs, int njobs, int j0,
                                         PIX* __restrict__ dst, int stride, char* lds) {
  using T = InvTile<W, H>;
  using C = TxCfg<W, H>;
  using B = Bd<BDI>;
  constexpr int P = T::P, T1S = T::T1S;
  InvJob* const jb = (InvJob*)lds;
  int32_t* const cf = (int32_t*)(lds + P * sizeof(InvJob));
  int32_t* const t1 = cf + P * T::NC;

  const int lane = threadIdx.x;
  __syncthreads();  // the previous tile's readers of jb / cf / t1 are done
  if (lane < P) {
    // (two stores, not a select between the job and a local zero job: the
    // select made the local a scratch object read through a flat pointer)
    if (j0 + lane < njobs) {
      jb[lane] = jobs[j0 + lane];
    } else {
      InvJob z;
      z.dst_off = 0;
      z.coeff_off = 0;
      z.tx_type = 0;
      z.eob = 0;
      jb[lane] = z;
    }
  }
  __syncthreads();
  // eob 0 adds nothing (av1_inverse_transform_block returns, idct.c:308): a
  // tile without a coded block leaves before any load or transform
  if (!__builtin_amdgcn_ballot_w64(lane < P && jb[lane < P ? lane : 0].eob != 0)) return;
  // stage the tile's dequantized coefficients (coalesced within a block):
  // every load in flight before the first LDS store (a load-store loop
  // waited one memory latency per iteration).  An uncoded block reads
  // coefficient 0 of the list (a valid address) and stores zeros.
  {
    constexpr int NI = (P * T::NC + 63) / 64;
    int32_t v[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = min(64 * k + lane, P * T::NC - 1);
      const int b = i / T::NC, w = i - b * T::NC;
      const bool on = jb[b].eob != 0;
      v[k] = dq[on ? jb[b].coeff_off + w : 0];
      v[k] = on ? v[k] : 0;
    }
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = 64 * k + lane;
      if ((P * T::NC) % 64 == 0 || i < P * T::NC) cf[i] = v[k];
    }
  }
  __syncthreads();

  // ---- rows (inv_txfm2d_add_c "Rows") ----
  // Blocks of a tile may carry different TX types: a waterfall over the
  // distinct types keeps the transform-kind branches scalar (one pass when
  // the tile is uniform, the common case).
#pragma unroll
  for (int k = 0; k < T::RPT; ++k) {
    const int idx = k * 64 + lane;
    const int b = idx / T::KH, r = idx - b * T::KH;
    const bool live = (P * T::KH) % 64 == 0 || idx < P * T::KH;
    const int mine = live ? jb[b].tx_type : 0;
    bool pending = live;
    while (__ballot(pending)) {
      if (pending) {
        const int t = __builtin_amdgcn_readfirstlane(mine);
        if (mine == t) {
          pending = false;
          const int ht = (kHtxP >> (2 * t)) & 3;
          const int kr = ht == 3 ? 2 : (ht == 0 ? 0 : 1);
          int32_t in[W];
#pragma unroll
          for (int c = 0; c < W; ++c) {
            int32_t v = c < T::KW ? cf[b * T::NC + c * T::KH + r] : 0;
            if constexpr (C::rect2) v = rshift64((int64_t)v * 2896, 12);
            in[c] = clamp_bits<B::clamp_in_row>(v);
          }
          inv_1d_then<W, 12, B::rng_row>(kr, in, [&](const int32_t(&out)[W]) {
#pragma unroll
            for (int c = 0; c < W; ++c) t1[(b * T::KH + r) * T1S + c] = rshift_r(out[c], -C::is0);
          });
        }
      }
    }
  }
  __syncthreads();

  // ---- columns + reconstruction ("Columns", highbd_clip_pixel_add) ----
  constexpr int maxv = (1 << B::bd) - 1;
#pragma unroll
  for (int k = 0; k < T::CPT; ++k) {
    const int idx = k * 64 + lane;
    const int b = idx / W, c = idx - b * W;
    const int mine = jb[b].tx_type;
    bool pending = true;
    while (__ballot(pending)) {
      if (pending) {
        const int t = __builtin_amdgcn_readfirstlane(mine);
        if (mine == t) {
          pending = false;
          const int vt = (kVtxP >> (2 * t)) & 3, ht = (kHtxP >> (2 * t)) & 3;
          const int kc = vt == 3 ? 2 : (vt == 0 ? 0 : 1);
          const bool ud = vt == 2, lr = ht == 2;
          const int cc = lr ? W - 1 - c : c;
          int32_t in[H];
#pragma unroll
          for (int r = 0; r < H; ++r)
            in[r] = r < T::KH ? clamp_bits<B::clamp_in_col>(t1[(b * T::KH + r) * T1S + cc]) : 0;
          const bool coded = jb[b].eob != 0;
          PIX* d = dst + jb[b].dst_off + c;
          // the column's pixels read before the transform, so the H loads
          // are in flight together (interleaved with the stores they would
          // wait one latency per row: the rows may alias for all the
          // compiler knows)
          int px[H];
          if (coded) {
#pragma unroll
            for (int r = 0; r < H; ++r) px[r] = (int)d[(int64_t)r * stride];
          }
          inv_1d_then<H, 12, B::rng_col>(kc, in, [&](const int32_t(&out)[H]) {
            if (coded) {
#pragma unroll
              for (int r = 0; r < H; ++r) {
                const int32_t res = rshift_r(ud ? out[H - 1 - r] : out[r], -C::is1);
                const int v = px[r] + res;
                d[(int64_t)r * stride] = (PIX)(v < 0 ? 0 : (v > maxv ? maxv : v));
              }
            }
          });
        }
      }
    }
  }
}

// njobs jobs as one list, or -- when slot_cnt is given -- a job list built on
// the device in slots of slot_cap jobs (C4: one slot per SB, its chosen
// coded blocks first, slot_cnt[slot] of them): the grid strides over the
// tiles, a tile never straddles two slots, and tiles past a slot's count
// are skipped (one workgroup per slot serialised the tiles of SBs that
// chose small sizes: 21 -> 155 us for 60 SBs of 4x4, profiles/r04_v5_*)
template <int W, int H, int BDI, typename PIX>
__global__ __launch_bounds__(64) void inv_tile_kernel(const int32_t* __restrict__ dq,
                                                      const InvJob* __restrict__ jobs, int njobs,
                                                      const uint16_t* __restrict__ slot_cnt,
                                                      int slot_cap, PIX* __restrict__ dst,
                                                      int stride) {
  constexpr int P = InvTile<W, H>::P;
  __shared__ __attribute__((aligned(16))) char lds[inv_lds_bytes<W, H>()];
  const int tps = slot_cnt ? (slot_cap + P - 1) / P : 1;  // tiles per slot
  const int ntiles = slot_cnt ? (njobs / slot_cap) * tps : (njobs + P - 1) / P;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    if (slot_cnt) {
      const int sl = t / tps, k = t - sl * tps;
      const int c = slot_cnt[sl];
      if (k * P >= c) continue;
      inv_tile<W, H, BDI, PIX>(dq, jobs, sl * slot_cap + c, sl * slot_cap + k * P, dst, stride,
                               lds);
    } else {
      inv_tile<W, H, BDI, PIX>(dq, jobs, njobs, t * P, dst, stride, lds);
    }
  }
}

// slotted lists: at most this many workgroups, looping over the tiles.  A
// size no SB chose still costs ~6 us: 4 096 workgroups reading 8 counts
// each measured the same as 16 384 reading one (profiles/r04_v7_*)
constexpr int kInvMaxGrid = 16384;

template <int W, int H, int BDI, typename PIX>
void launch(const int32_t* dq, const LavishInvJob* jobs, int njobs, const uint16_t* slot_cnt,
            int slot_cap, PIX* dst, int stride, hipStream_t s) {
  constexpr int P = InvTile<W, H>::P;
  int grid = slot_cnt ? (njobs / slot_cap) * ((slot_cap + P - 1) / P) : (njobs + P - 1) / P;
  if (slot_cnt != nullptr && grid > kInvMaxGrid) grid = kInvMaxGrid;
  if (grid == 0) return;
  hipLaunchKernelGGL((inv_tile_kernel<W, H, BDI, PIX>), dim3(grid), dim3(64), 0, s, dq,
                     (const InvJob*)jobs, njobs, slot_cnt, slot_cap, dst, stride);
}

template <int W, int H>
int dispatch_bd(const int32_t* dq, const LavishInvJob* jobs, int njobs, const uint16_t* slot_cnt,
                int slot_cap, void* dst, int stride, int bd, int highbd, hipStream_t s) {
  if (!highbd) {
    if (bd != 8) return -4;
    launch<W, H, 0, uint8_t>(dq, jobs, njobs, slot_cnt, slot_cap, (uint8_t*)dst, stride, s);
  } else if (bd == 8) {
    launch<W, H, 0, uint16_t>(dq, jobs, njobs, slot_cnt, slot_cap, (uint16_t*)dst, stride, s);
  } else if (bd == 10) {
    launch<W, H, 1, uint16_t>(dq, jobs, njobs, slot_cnt, slot_cap, (uint16_t*)dst, stride, s);
  } else if (bd == 12) {
    launch<W, H, 2, uint16_t>(dq, jobs, njobs, slot_cnt, slot_cap, (uint16_t*)dst, stride, s);
  } else {
    return -4;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// The C4 reconstruction's inverse transforms in one launch (rdo.hip,
// sb_decide_kernel's per-SB job slots): wave (k, sb) -- k-major, so the
// first nsb waves take every SB's first tile -- runs tile k of the size SB
// sb chose, if the SB has that many coded blocks; every other wave leaves at
// once.  The sizes' tiles share one LDS buffer (the largest size's), so the
// one kernel holds no more LDS than the largest per-size kernel.  Replaces
// one launch per candidate size (and the fan-out / fan-in around them).
template <int W, int H>
constexpr int inv_tpsb() {  // tiles per SB of a size
  return ((64 / W) * (64 / H) + InvTile<W, H>::P - 1) / InvTile<W, H>::P;
}

#define LAVISH_INV_SIZES(X)                                                                      \
  X(0, 4, 4) X(1, 8, 8) X(2, 16, 16) X(3, 32, 32) X(4, 64, 64) X(5, 4, 8) X(6, 8, 4) X(7, 8, 16) \
  X(8, 16, 8) X(9, 16, 32) X(10, 32, 16) X(11, 32, 64) X(12, 64, 32) X(13, 4, 16) X(14, 16, 4)  \
  X(15, 8, 32) X(16, 32, 8) X(17, 16, 64) X(18, 64, 16)

constexpr int inv_max_lds() {
  int m = 0;
#define LAVISH_INV_LDS(S, W, H) m = m > inv_lds_bytes<W, H>() ? m : inv_lds_bytes<W, H>();
  LAVISH_INV_SIZES(LAVISH_INV_LDS)
#undef LAVISH_INV_LDS
  return m;
}

template <int BDI>
__global__ __launch_bounds__(64) void recon_sb_kernel(InvSbArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[inv_max_lds()];
  const int sb = blockIdx.x % a.nsb, k = blockIdx.x / a.nsb;
  const int s = a.sb_tx_size[sb];
  if (s >= 19) return;  // no candidate size tiles this SB: recon = pred
  const int c = a.cnt[s][sb];
  switch (s) {
#define LAVISH_INV_CASE(S, W, H)                                                               \
  case S: {                                                                                    \
    constexpr int P = InvTile<W, H>::P, CAP = (64 / W) * (64 / H);                            \
    if (k * P >= c) return;                                                                    \
    inv_tile<W, H, BDI, uint16_t>(a.dq[S], (const InvJob*)a.jobs[S], sb * CAP + c,              \
                                  sb * CAP + k * P, a.dst, a.stride, lds);                     \
    return;                                                                                    \
  }
    LAVISH_INV_SIZES(LAVISH_INV_CASE)
#undef LAVISH_INV_CASE
    default: return;
  }
}

}  // namespace

int recon_sb_launch(const InvSbArgs& a, int bd, hipStream_t s) {
  if (a.nsb <= 0) return 0;
  int tps = 1;  // tiles per SB of the candidate size with the most
  for (int t = 0; t < 19; ++t) {
    if (!a.jobs[t]) continue;
    int n = 0;
#define LAVISH_INV_TPS(S, W, H) \
    if (t == S) n = inv_tpsb<W, H>();
    LAVISH_INV_SIZES(LAVISH_INV_TPS)
#undef LAVISH_INV_TPS
    tps = n > tps ? n : tps;
  }
  const dim3 grid((unsigned)(a.nsb * tps));
  if (bd == 8) hipLaunchKernelGGL(recon_sb_kernel<0>, grid, dim3(64), 0, s, a);
  else if (bd == 10) hipLaunchKernelGGL(recon_sb_kernel<1>, grid, dim3(64), 0, s, a);
  else if (bd == 12) hipLaunchKernelGGL(recon_sb_kernel<2>, grid, dim3(64), 0, s, a);
  else return -4;
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

int inv_txfm_add_batch(const int32_t* dq, int tx_size, const LavishInvJob* jobs, int njobs,
                       void* dst, int stride, int bd, int highbd, hipStream_t s,
                       const uint16_t* slot_cnt, int slot_cap) {
  if (slot_cnt != nullptr && (slot_cap <= 0 || njobs % slot_cap)) return -3;
  if (njobs <= 0) return 0;
  int rc;
  switch (tx_size) {
    case 0: rc = dispatch_bd<4, 4>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 1: rc = dispatch_bd<8, 8>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 2: rc = dispatch_bd<16, 16>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 3: rc = dispatch_bd<32, 32>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 4: rc = dispatch_bd<64, 64>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 5: rc = dispatch_bd<4, 8>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 6: rc = dispatch_bd<8, 4>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 7: rc = dispatch_bd<8, 16>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 8: rc = dispatch_bd<16, 8>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 9: rc = dispatch_bd<16, 32>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 10: rc = dispatch_bd<32, 16>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 11: rc = dispatch_bd<32, 64>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 12: rc = dispatch_bd<64, 32>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 13: rc = dispatch_bd<4, 16>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 14: rc = dispatch_bd<16, 4>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 15: rc = dispatch_bd<8, 32>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 16: rc = dispatch_bd<32, 8>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 17: rc = dispatch_bd<16, 64>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    case 18: rc = dispatch_bd<64, 16>(dq, jobs, njobs, slot_cnt, slot_cap, dst, stride, bd, highbd, s); break;
    default: return -1;
  }
  if (rc == 0) LAVISH_CHECK(hipGetLastError());
  return rc;
}

}  // namespace lavish

extern "C" int lavish_inv_txfm_add_batch(const int32_t* dqcoeff, int tx_size,
                                         const LavishInvJob* jobs, int njobs, void* dst,
                                         int dst_stride, int bit_depth, int highbd,
                                         void* stream) {
  return lavish::inv_txfm_add_batch(dqcoeff, tx_size, jobs, njobs, dst, dst_stride, bit_depth,
                                    highbd, (hipStream_t)stream);
}
