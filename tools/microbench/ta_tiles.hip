// Address-path rate of the candidate-row shapes a field-split strip layout
// of the reference gives the C3 search (cycles per wave load instruction per
// CU, L2-resident data; compare tools/microbench/ta_rate.hip "rows" /
// "rowsu" = today's linear layout: 64 lanes on 64 distinct rows):
//   rowsu  : linear layout, each lane its own row, byte-unaligned 16 B
//   t8u    : 8 groups far apart; a group's 8 lanes read 8 consecutive 32-byte
//            strip rows (256 contiguous bytes), 16 B at byte offset 0..15
//   t8a    : the same, 16-byte aligned
//   t8w    : 8 groups far apart, lanes read the two aligned halves a 16 B
//            unaligned segment spans (2 loads, v_alignbyte) -- not measured
//            separately: t8a x 2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u4 __attribute__((ext_vector_type(4), aligned(1)));

template <int MODE>
__global__ __launch_bounds__(256) void ta(const uint8_t* __restrict__ buf, uint32_t* out, int iters) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
  uint32_t acc = 0;
  const uint32_t base = (uint32_t)(wave * 7919 * 64) & ((1u << 21) - 1 - (1u << 18));
  for (int it = 0; it < iters; ++it) {
    const uint32_t b = base + ((it * 4099u) & 0xFFFFu);
    const int g = lane >> 3, l = lane & 7;
    uint32_t off;
    if (MODE == 0) off = b + lane * 2240 + (lane & 15);
    else if (MODE == 1) off = ((b + g * 9000) & ~31u) + l * 32 + ((g * 5 + it) & 15);
    else off = ((b + g * 9000) & ~31u) + l * 32;
    const u4 v = *(const __attribute__((address_space(1))) u4*)(buf + off);
    acc += v.x ^ v.y ^ v.z ^ v.w;
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
  const char* names[3] = {"rowsu", "t8u", "t8a"};
  const int grid = 256 * 8, iters = 2000;
  for (int m = 0; m < 3; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a));
      switch (m) {
        case 0: hipLaunchKernelGGL(ta<0>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        case 1: hipLaunchKernelGGL(ta<1>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
        default: hipLaunchKernelGGL(ta<2>, dim3(grid), dim3(256), 0, 0, buf, out, iters); break;
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
