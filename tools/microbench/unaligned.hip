// Probe: do 16-byte global and LDS loads at arbitrary byte addresses return
// the bytes at that address on this box (SH_MEM_CONFIG unaligned mode)?
// Prints the mismatch count per path; no timing.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void probe(const uint8_t* __restrict__ g, u4* __restrict__ out_g,
                                            u4* __restrict__ out_l) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2048];
  const int lane = threadIdx.x;
  for (int i = lane; i < 2048; i += 64) lds[i] = g[i];
  __syncthreads();
  const int off = lane * 17 + (lane & 3);  // every byte alignment
  out_g[lane] = *(const u4*)(g + off);
  out_l[lane] = *(const u4*)(lds + off);
}

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
  uint8_t h[2048];
  for (int i = 0; i < 2048; ++i) h[i] = (uint8_t)(i * 131 + 7);
  uint8_t* g;
  u4 *og, *ol;
  CK(hipMalloc(&g, 2048));
  CK(hipMalloc(&og, 64 * 16));
  CK(hipMalloc(&ol, 64 * 16));
  CK(hipMemcpy(g, h, 2048, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, g, og, ol);
  CK(hipDeviceSynchronize());
  uint8_t rg[64 * 16], rl[64 * 16];
  CK(hipMemcpy(rg, og, sizeof(rg), hipMemcpyDeviceToHost));
  CK(hipMemcpy(rl, ol, sizeof(rl), hipMemcpyDeviceToHost));
  int bad_g = 0, bad_l = 0;
  for (int lane = 0; lane < 64; ++lane) {
    const int off = lane * 17 + (lane & 3);
    for (int b = 0; b < 16; ++b) {
      bad_g += rg[lane * 16 + b] != h[off + b];
      bad_l += rl[lane * 16 + b] != h[off + b];
    }
  }
  printf("unaligned 16-byte loads: global mismatches %d, LDS mismatches %d (of 1024 bytes)\n", bad_g,
         bad_l);
  return 0;
}
