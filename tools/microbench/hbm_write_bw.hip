// HBM write-bandwidth ceiling on this box: grid-stride 16-byte stores
// (plain and nontemporal) over a 2.6 GB buffer -- the C2 output stream size.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void fill(v4i* p, size_t n, int val) {
  const size_t stride = (size_t)gridDim.x * 256;
  v4i v = {val, val + 1, val + 2, val + 3};
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    if (NT) __builtin_nontemporal_store(v, &p[i]);
    else p[i] = v;
  }
}
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
  const size_t bytes = 2616772080ull & ~(size_t)15;
  const size_t n = bytes / 16;
  v4i* p;
  CK(hipMalloc(&p, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int nt = 0; nt < 2; ++nt)
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
      for (int w = 0; w < 2; ++w) {
        if (nt) hipLaunchKernelGGL(fill<true>, dim3(grid), dim3(256), 0, 0, p, n, w);
        else hipLaunchKernelGGL(fill<false>, dim3(grid), dim3(256), 0, 0, p, n, w);
      }
      CK(hipEventRecord(a));
      for (int it = 0; it < 5; ++it) {
        if (nt) hipLaunchKernelGGL(fill<true>, dim3(grid), dim3(256), 0, 0, p, n, it);
        else hipLaunchKernelGGL(fill<false>, dim3(grid), dim3(256), 0, 0, p, n, it);
      }
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= 5;
      printf("%s grid=%5d ms=%.4f GB/s=%.0f\n", nt ? "nt   " : "plain", grid, ms, bytes / ms / 1e6);
    }
  CK(hipFree(p));
  return 0;
}
