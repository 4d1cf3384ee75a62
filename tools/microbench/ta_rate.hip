// Vector-memory address-path rate on this box: cycles per wave load
// instruction (per CU) for the access shapes of the C3 search, with the data
// L2-resident (a 2 MB footprint read over and over).
//   same   : all 64 lanes one 16-byte address
//   coal   : lanes consecutive 16-byte words (1 KB per instruction)
//   rows   : each lane its own row (stride 2240 B, like a padded 1080p plane), 16 B aligned
//   rowsu  : same, byte-unaligned 16-byte loads
//   rows4  : same rows, one dword per lane
//   grp8   : 8 groups of 8 lanes, a group's lanes share one row (16 B each, same line)
//   grp8d  : 8 groups, a group's 8 lanes load the same dword (the mv-cost table reads)
//   one8d  : the same 8 dwords, loaded by one lane per group only
// Prints ns per instruction per CU (and cycles at the measured clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void ta(const uint8_t* __restrict__ buf, uint32_t* out, int iters) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
  uint32_t acc = 0;
  // each wave walks its own 2 KB-row neighbourhood inside the 2 MB buffer
  const uint32_t base = (uint32_t)(wave * 7919 * 64) & ((1u << 21) - 1 - (1u << 18));
  for (int it = 0; it < iters; ++it) {
    const uint32_t b = base + ((it * 4099u) & 0xFFFFu);
    uint32_t off;
    if (MODE == 0) off = b;
    else if (MODE == 1) off = b + lane * 16;
    else if (MODE == 2) off = b + lane * 2240;
    else if (MODE == 3) off = b + lane * 2240 + (lane & 15);
    else if (MODE == 4) off = b + lane * 2240;
    else if (MODE == 5) off = b + (lane >> 3) * 2240 + (lane & 7) * 2;
    else off = b + (lane >> 3) * 2240;  // 6, 7: a group's 8 lanes share one dword
    if (MODE == 7) {  // only one lane per group issues the load
      if ((lane & 7) == 0) acc += *(const __attribute__((address_space(1))) uint32_t*)(buf + off);
    } else if (MODE == 4 || MODE == 6) {
      acc += *(const __attribute__((address_space(1))) uint32_t*)(buf + off);
    } else {
      const u4 v = *(const __attribute__((address_space(1))) u4*)(buf + (MODE == 3 || MODE == 5 ? off : (off & ~15u)));
      acc += v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
  uint8_t* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, 1 << 22));
  CK(hipMemset(buf, 1, 1 << 22));
  CK(hipMalloc(&out, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[8] = {"same", "coal", "rows", "rowsu", "rows4", "grp8", "grp8d", "one8d"};
  const int grid = 256 * 8, iters = 2000;  // 8 workgroups (32 waves) per CU
  for (int m = 0; m < 8; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a));
      switch (m) {
        case 0: hipLaunchKernelGGL(ta<0>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        case 1: hipLaunchKernelGGL(ta<1>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        case 2: hipLaunchKernelGGL(ta<2>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        case 3: hipLaunchKernelGGL(ta<3>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        case 4: hipLaunchKernelGGL(ta<4>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        case 5: hipLaunchKernelGGL(ta<5>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        case 6: hipLaunchKernelGGL(ta<6>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        default: hipLaunchKernelGGL(ta<7>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
      }
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep == 1) {
        const double inst_per_cu = (double)grid * 4 * iters / 256.0;
        printf("%-6s %8.3f ms  %.3f ns/instr/CU  (%.1f cycles at 2.4 GHz)\n", names[m], ms,
               ms * 1e6 / inst_per_cu, ms * 1e6 / inst_per_cu * 2.4);
      }
    }
  }
  return 0;
}
