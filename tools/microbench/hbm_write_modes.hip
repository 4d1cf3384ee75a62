// HBM write bandwidth by store pattern and cache policy, over a 2.6 GB
// buffer (the C2 output stream's size): is there headroom above the
// grid-stride ceiling of hbm_write_bw.hip (5.8 TB/s, profiles/r02_hbm_write_bw.txt)
// for C2's pattern -- each workgroup writing a few KB-sized contiguous runs?
//   chunk C:  workgroup b writes bytes [b C, (b + 1) C) (one-shot grid)
//   aux A:    buffer stores with cache-policy bits A (0..3), grid-stride
// hipcc -O3 --offload-arch=gfx950 tools/microbench/hbm_write_modes.hip -o hbm_write_modes
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));

// XCD: workgroup b (on XCD b % 8) writes chunk (b % 8) * (nwg / 8) + b / 8,
// so each XCD's workgroups write one contiguous eighth of the buffer
template <int CHUNK, bool XCD>
__global__ __launch_bounds__(256) void chunked(v4i* p, int val) {
  const size_t b = XCD ? (size_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3)
                       : (size_t)blockIdx.x;
  v4i* q = p + b * (CHUNK / 16);
  const v4i v = {val, val + 1, val + 2, val + 3};
#pragma unroll 4
  for (int i = threadIdx.x; i < CHUNK / 16; i += 256) __builtin_nontemporal_store(v, &q[i]);
}

template <int AUX>
__global__ __launch_bounds__(256) void buffered(v4i* p, size_t n, int val) {
  const v4i v = {val, val + 1, val + 2, val + 3};
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    // one descriptor per 1 GiB window (32-bit offsets)
    const size_t base = i & ~(((size_t)1 << 26) - 1);
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p + base), 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)((i - base) * 16), 0, AUX);
  }
}

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <class F>
static int timed(const char* name, F launch, size_t bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch(0);
  launch(1);
  CK(hipEventRecord(a));
  for (int it = 0; it < 5; ++it) launch(it);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 5;
  printf("%-24s ms=%.4f GB/s=%.0f\n", name, ms, bytes / ms / 1e6);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main() {
  const size_t bytes = (size_t)2616 << 20;  // multiple of every chunk below
  const size_t n = bytes / 16;
  v4i* p;
  CK(hipMalloc(&p, bytes));
#define CHUNK_RUN(C, X)                                                                      \
  timed("chunk " #C " xcd " #X, [&](int w) {                                                 \
    hipLaunchKernelGGL((chunked<C, X>), dim3((unsigned)(bytes / C)), dim3(256), 0, 0, p, w); \
  }, bytes);
  CHUNK_RUN(1024, false)
  CHUNK_RUN(2048, false)
  CHUNK_RUN(4096, false)
  CHUNK_RUN(4096, false)
  CHUNK_RUN(8192, false)
  CHUNK_RUN(16384, false)
  CHUNK_RUN(65536, false)
  CHUNK_RUN(4096, true)
  CHUNK_RUN(8192, true)
  CHUNK_RUN(16384, true)
  CHUNK_RUN(65536, true)
#define AUX_RUN(A, G)                                                                        \
  timed("aux " #A " grid " #G, [&](int w) {                                                  \
    hipLaunchKernelGGL(buffered<A>, dim3(G), dim3(256), 0, 0, p, n, w);                      \
  }, bytes);
  AUX_RUN(0, 16384)
  AUX_RUN(1, 16384)
  AUX_RUN(2, 16384)
  AUX_RUN(3, 16384)
  AUX_RUN(0, 32768)
  AUX_RUN(2, 32768)
  CK(hipFree(p));
  return 0;
}
