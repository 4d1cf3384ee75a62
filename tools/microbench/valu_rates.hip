// valu_rates.hip -- issue cost of the VALU instructions the C4 / C2 kernels
// lean on (gfx950), measured as the wall time of a launch whose waves run a
// long unrolled stream of ONE instruction on independent registers, 8
// waves per SIMD (so dependency latency is hidden and only the SIMD's issue
// rate shows).  Prints cycles per wave-instruction per SIMD, relative to
// v_add_u32 (the full-rate reference).
//
// hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates && ./valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

// Each kernel: 8 independent accumulator chains per lane, 64 x 8 x ITER
// instructions of one kind.
#define KERNEL(NAME, ASM)                                                        \
  __global__ __launch_bounds__(256) void NAME(int* out, int iters) {             \
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,      \
        a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                   \
    long b0 = a0, b1 = a1, b2 = a2, b3 = a3;                                     \
    int s = 3;                                                                   \
    for (int it = 0; it < iters; ++it) {                                         \
      REP8(ASM)                                                                  \
    }                                                                            \
    out[blockIdx.x * 256 + threadIdx.x] =                                        \
        a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (int)(b0 + b1 + b2 + b3);        \
  }

#define ADD32 asm volatile(                                                           \
    "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n"           \
    "v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n"           \
    "v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"                                  \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
    : "v"(s));
#define MULI24 asm volatile(                                                          \
    "v_mul_i32_i24 %0, %0, %8\n v_mul_i32_i24 %1, %1, %8\n v_mul_i32_i24 %2, %2, %8\n" \
    "v_mul_i32_i24 %3, %3, %8\n v_mul_i32_i24 %4, %4, %8\n v_mul_i32_i24 %5, %5, %8\n" \
    "v_mul_i32_i24 %6, %6, %8\n v_mul_i32_i24 %7, %7, %8\n"                            \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)   \
    : "v"(s));
#define MULHII24 asm volatile(                                                              \
    "v_mul_hi_i32_i24 %0, %0, %8\n v_mul_hi_i32_i24 %1, %1, %8\n v_mul_hi_i32_i24 %2, %2, %8\n" \
    "v_mul_hi_i32_i24 %3, %3, %8\n v_mul_hi_i32_i24 %4, %4, %8\n v_mul_hi_i32_i24 %5, %5, %8\n" \
    "v_mul_hi_i32_i24 %6, %6, %8\n v_mul_hi_i32_i24 %7, %7, %8\n"                                \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)             \
    : "v"(s));
#define MADI24 asm volatile(                                                                    \
    "v_mad_i32_i24 %0, %0, %8, %8\n v_mad_i32_i24 %1, %1, %8, %8\n v_mad_i32_i24 %2, %2, %8, %8\n" \
    "v_mad_i32_i24 %3, %3, %8, %8\n v_mad_i32_i24 %4, %4, %8, %8\n v_mad_i32_i24 %5, %5, %8, %8\n" \
    "v_mad_i32_i24 %6, %6, %8, %8\n v_mad_i32_i24 %7, %7, %8, %8\n"                                \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)               \
    : "v"(s));
#define MULLO asm volatile(                                                              \
    "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n"       \
    "v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n"       \
    "v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"                                  \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)       \
    : "v"(s));
#define ADD3 asm volatile(                                                                  \
    "v_add3_u32 %0, %0, %8, %8\n v_add3_u32 %1, %1, %8, %8\n v_add3_u32 %2, %2, %8, %8\n"    \
    "v_add3_u32 %3, %3, %8, %8\n v_add3_u32 %4, %4, %8, %8\n v_add3_u32 %5, %5, %8, %8\n"    \
    "v_add3_u32 %6, %6, %8, %8\n v_add3_u32 %7, %7, %8, %8\n"                                 \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)          \
    : "v"(s));
#define LSHLADD64 asm volatile(                                                                            \
    "v_lshl_add_u64 %0, %0, 0, %4\n v_lshl_add_u64 %1, %1, 0, %4\n v_lshl_add_u64 %2, %2, 0, %4\n"          \
    "v_lshl_add_u64 %3, %3, 0, %4\n v_lshl_add_u64 %0, %0, 0, %4\n v_lshl_add_u64 %1, %1, 0, %4\n"          \
    "v_lshl_add_u64 %2, %2, 0, %4\n v_lshl_add_u64 %3, %3, 0, %4\n"                                          \
    : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3)                                                                 \
    : "v"((long)s));
#define MADI64 asm volatile(                                                                                          \
    "v_mad_i64_i32 %0, vcc, %4, %4, %0\n v_mad_i64_i32 %1, vcc, %4, %4, %1\n v_mad_i64_i32 %2, vcc, %4, %4, %2\n"      \
    "v_mad_i64_i32 %3, vcc, %4, %4, %3\n v_mad_i64_i32 %0, vcc, %4, %4, %0\n v_mad_i64_i32 %1, vcc, %4, %4, %1\n"      \
    "v_mad_i64_i32 %2, vcc, %4, %4, %2\n v_mad_i64_i32 %3, vcc, %4, %4, %3\n"                                            \
    : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3)                                                                             \
    : "v"(s) : "vcc");
#define ASHR64 asm volatile(                                                                          \
    "v_ashrrev_i64 %0, 1, %0\n v_ashrrev_i64 %1, 1, %1\n v_ashrrev_i64 %2, 1, %2\n"                    \
    "v_ashrrev_i64 %3, 1, %3\n v_ashrrev_i64 %0, 1, %0\n v_ashrrev_i64 %1, 1, %1\n"                    \
    "v_ashrrev_i64 %2, 1, %2\n v_ashrrev_i64 %3, 1, %3\n"                                                \
    : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
#define CMP64 asm volatile(                                                                           \
    "v_cmp_lt_i64 vcc, %0, %1\n v_cmp_lt_i64 vcc, %1, %2\n v_cmp_lt_i64 vcc, %2, %3\n"                 \
    "v_cmp_lt_i64 vcc, %3, %0\n v_cmp_lt_i64 vcc, %0, %2\n v_cmp_lt_i64 vcc, %1, %3\n"                 \
    "v_cmp_lt_i64 vcc, %2, %0\n v_cmp_lt_i64 vcc, %3, %1\n"                                            \
    : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) :: "vcc");
#define DPPADD asm volatile(                                                                                    \
    "v_add_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                                  \
    "v_add_u32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                                  \
    "v_add_u32_dpp %2, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                                  \
    "v_add_u32_dpp %3, %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                                  \
    "v_add_u32_dpp %4, %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                                  \
    "v_add_u32_dpp %5, %5, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                                  \
    "v_add_u32_dpp %6, %6, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                                  \
    "v_add_u32_dpp %7, %7, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                                  \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
#define CND asm volatile(                                                                                  \
    "v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n"            \
    "v_cndmask_b32 %5, %5, %6, vcc\n v_cndmask_b32 %7, %7, %0, vcc\n v_cndmask_b32 %2, %2, %1, vcc\n"      \
    "v_cndmask_b32 %4, %4, %3, vcc\n v_cndmask_b32 %6, %6, %5, vcc\n"                                       \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                        \
    : "v"(s) : "vcc");

KERNEL(k_add32, ADD32)
KERNEL(k_muli24, MULI24)
KERNEL(k_mulhii24, MULHII24)
KERNEL(k_madi24, MADI24)
KERNEL(k_mullo, MULLO)
KERNEL(k_add3, ADD3)
KERNEL(k_lshladd64, LSHLADD64)
KERNEL(k_madi64, MADI64)
KERNEL(k_ashr64, ASHR64)
KERNEL(k_cmp64, CMP64)
KERNEL(k_dppadd, DPPADD)
KERNEL(k_cnd, CND)


#define OP2(NAME, OP) KERNEL(NAME, asm volatile(                                          \
    OP " %0, %0, %8\n" OP " %1, %1, %8\n" OP " %2, %2, %8\n" OP " %3, %3, %8\n"          \
    OP " %4, %4, %8\n" OP " %5, %5, %8\n" OP " %6, %6, %8\n" OP " %7, %7, %8\n"          \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)     \
    : "v"(s));)
OP2(k_sub32, "v_sub_u32")
OP2(k_xor32, "v_xor_b32")
OP2(k_max32, "v_max_i32")
OP2(k_ashr32, "v_ashrrev_i32")
OP2(k_and32, "v_and_b32")
OP2(k_addco, "v_add_co_u32")
// v_cndmask with an SGPR mask written once, before the loop (no hazard)
__global__ __launch_bounds__(256) void k_cndsgpr(int* out, int iters) {
  int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
      a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; ++it) {
    REP8(asm volatile(
        "v_cndmask_b32 %0, %0, %1, s[40:41]\n v_cndmask_b32 %1, %1, %2, s[40:41]\n"
        "v_cndmask_b32 %2, %2, %3, s[40:41]\n v_cndmask_b32 %3, %3, %4, s[40:41]\n"
        "v_cndmask_b32 %4, %4, %5, s[40:41]\n v_cndmask_b32 %5, %5, %6, s[40:41]\n"
        "v_cndmask_b32 %6, %6, %7, s[40:41]\n v_cndmask_b32 %7, %7, %0, s[40:41]\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        :: "s40", "s41");)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
// v_cmp writing an SGPR pair, the cndmask reading it 0 / 4 independent instructions later
__global__ __launch_bounds__(256) void k_cmpcnd0(int* out, int iters) {
  int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
      a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; ++it) {
    REP8(asm volatile(
        "v_cmp_gt_i32 s[40:41], %0, %1\n v_cndmask_b32 %2, %2, %3, s[40:41]\n"
        "v_cmp_gt_i32 s[42:43], %4, %5\n v_cndmask_b32 %6, %6, %7, s[42:43]\n"
        "v_cmp_gt_i32 s[44:45], %1, %2\n v_cndmask_b32 %3, %3, %4, s[44:45]\n"
        "v_cmp_gt_i32 s[46:47], %5, %6\n v_cndmask_b32 %7, %7, %0, s[46:47]\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        :: "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_cmpcnd4(int* out, int iters) {
  int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
      a6 = a0 + 6, a7 = a0 + 7;
  for (int it = 0; it < iters; ++it) {
    REP8(asm volatile(
        "v_cmp_gt_i32 s[40:41], %0, %1\n v_cmp_gt_i32 s[42:43], %4, %5\n"
        "v_cmp_gt_i32 s[44:45], %1, %2\n v_cmp_gt_i32 s[46:47], %5, %6\n"
        "v_cndmask_b32 %2, %2, %3, s[40:41]\n v_cndmask_b32 %6, %6, %7, s[42:43]\n"
        "v_cndmask_b32 %3, %3, %4, s[44:45]\n v_cndmask_b32 %7, %7, %0, s[46:47]\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        :: "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
// v_cmp alone (SGPR destinations, no reader)
__global__ __launch_bounds__(256) void k_cmponly(int* out, int iters) {
  int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  for (int it = 0; it < iters; ++it) {
    REP8(asm volatile(
        "v_cmp_gt_i32 s[40:41], %0, %1\n v_cmp_gt_i32 s[42:43], %2, %3\n"
        "v_cmp_gt_i32 s[44:45], %1, %2\n v_cmp_gt_i32 s[46:47], %3, %0\n"
        "v_cmp_gt_i32 s[40:41], %0, %2\n v_cmp_gt_i32 s[42:43], %1, %3\n"
        "v_cmp_gt_i32 s[44:45], %2, %0\n v_cmp_gt_i32 s[46:47], %3, %1\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
        :: "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}
// v_mov_b32
OP2(k_lshl32, "v_lshlrev_b32")

typedef void (*K)(int*, int);

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
  const int blocks = cus * 8;  // 8 x 256 threads per CU = 8 waves per SIMD
  int* out;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(int));
  const int iters = 4000;
  struct { const char* name; K k; } ks[] = {
      {"v_add_u32", k_add32},       {"v_mul_i32_i24", k_muli24}, {"v_mul_hi_i32_i24", k_mulhii24},
      {"v_mad_i32_i24", k_madi24},  {"v_mul_lo_u32", k_mullo},   {"v_add3_u32", k_add3},
      {"v_lshl_add_u64", k_lshladd64}, {"v_mad_i64_i32", k_madi64}, {"v_ashrrev_i64", k_ashr64},
      {"v_cmp_lt_i64", k_cmp64},    {"v_add_u32_dpp", k_dppadd}, {"v_cmp+v_cndmask (vcc)", k_cnd},
      {"v_sub_u32", k_sub32}, {"v_xor_b32", k_xor32}, {"v_max_i32", k_max32},
      {"v_ashrrev_i32", k_ashr32}, {"v_and_b32", k_and32}, {"v_lshlrev_b32", k_lshl32},
      {"v_add_co_u32", k_addco}, {"v_cndmask (sgpr mask, old)", k_cndsgpr},
      {"v_cmp->v_cndmask adjacent", k_cmpcnd0}, {"v_cmp x4 then v_cndmask x4", k_cmpcnd4},
      {"v_cmp (sgpr dst) only", k_cmponly}};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  double base = 0;
  printf("%d CUs, clock %d MHz (attribute), %d blocks x 256 threads, %d x 64 instr per thread\n",
         cus, clk / 1000, blocks, iters);
  for (auto& e : ks) {
    hipLaunchKernelGGL(e.k, dim3(blocks), dim3(256), 0, 0, out, 10);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(e.k, dim3(blocks), dim3(256), 0, 0, out, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    // wave-instructions per SIMD: waves per SIMD (8) x instructions per wave
    const double per_simd = 8.0 * iters * 64;
    const double cyc = best * 1e-3 * (clk * 1e3) / per_simd;
    if (base == 0) base = cyc;
    printf("%-26s %8.3f ms  %6.2f cycles/wave-instr/SIMD (x%.2f of v_add_u32)\n", e.name, best, cyc,
           cyc / base);
  }
  return 0;
}
