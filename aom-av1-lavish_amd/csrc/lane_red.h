// lane_red.h -- reductions over aligned groups of N lanes of a wave64 (N a
// power of two <= 64) where every lane of a group ends with the group's
// result, as cross-lane moves inside the VALU: DPP quad_perm for the lane
// pairs at distance 1 and 2, row_half_mirror / row_mirror for the 8- and
// 16-lane halves, the gfx950 permlane16 / permlane32 swaps across rows.
// A ds_bpermute-based __shfl_xor step is an LDS round trip (~100+ cycles of
// latency per dependent step); these are a few cycles each.
//
// The 4- and 8-distance steps pair lane i with the mirror lane of its 8- /
// 16-lane half, not i ^ m; after the smaller steps have run every lane of an
// m-lane group holds the same value, so any pairing of the two halves gives
// the group result.  The op must be commutative and associative.  Every lane
// of the wave must be active (the callers reduce in uniform control flow).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lavish {

template <int M>
__device__ __forceinline__ uint32_t lane_partner(uint32_t v) {
  static_assert(M == 1 || M == 2 || M == 4 || M == 8, "DPP distances");
  constexpr int ctrl = M == 1 ? 0xB1 : M == 2 ? 0x4E : M == 4 ? 0x141 : 0x140;
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, 0xF, 0xF, false);
}

// v op partner(v) at distance M, 32-bit
template <int M, class F>
__device__ __forceinline__ uint32_t red_step32(uint32_t v, F op) {
  if constexpr (M <= 8) {
    return op(v, lane_partner<M>(v));
  } else if constexpr (M == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return op((uint32_t)p[0], (uint32_t)p[1]);
  } else {
    static_assert(M == 32, "distance");
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return op((uint32_t)p[0], (uint32_t)p[1]);
  }
}

// the same for a 64-bit value (both halves moved)
template <int M, class F>
__device__ __forceinline__ uint64_t red_step64(uint64_t v, F op) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  uint64_t a, b;
  if constexpr (M <= 8) {
    a = v;
    b = ((uint64_t)lane_partner<M>(hi) << 32) | lane_partner<M>(lo);
  } else if constexpr (M == 16) {
    const auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a = ((uint64_t)(uint32_t)ph[0] << 32) | (uint32_t)pl[0];
    b = ((uint64_t)(uint32_t)ph[1] << 32) | (uint32_t)pl[1];
  } else {
    static_assert(M == 32, "distance");
    const auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a = ((uint64_t)(uint32_t)ph[0] << 32) | (uint32_t)pl[0];
    b = ((uint64_t)(uint32_t)ph[1] << 32) | (uint32_t)pl[1];
  }
  return op(a, b);
}

template <int N, int M = 1, class F>
__device__ __forceinline__ uint32_t lane_reduce32(uint32_t v, F op) {
  if constexpr (M >= N) {
    return v;
  } else {
    return lane_reduce32<N, 2 * M>(red_step32<M>(v, op), op);
  }
}

template <int N, int M = 1, class F>
__device__ __forceinline__ uint64_t lane_reduce64(uint64_t v, F op) {
  if constexpr (M >= N) {
    return v;
  } else {
    return lane_reduce64<N, 2 * M>(red_step64<M>(v, op), op);
  }
}

// the common reductions
template <int N>
__device__ __forceinline__ int lane_sum(int v) {
  return (int)lane_reduce32<N>((uint32_t)v, [](uint32_t a, uint32_t b) { return a + b; });
}
template <int N>
__device__ __forceinline__ int lane_max(int v) {
  return (int)lane_reduce32<N>((uint32_t)v,
                               [](uint32_t a, uint32_t b) { return (uint32_t)max((int)a, (int)b); });
}
template <int N>
__device__ __forceinline__ int64_t lane_sum64(int64_t v) {
  return (int64_t)lane_reduce64<N>((uint64_t)v, [](uint64_t a, uint64_t b) { return a + b; });
}

}  // namespace lavish
