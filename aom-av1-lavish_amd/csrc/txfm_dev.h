// txfm_dev.h -- device-side AV1 1-D transforms for gfx950, fully unrolled.
//
// Every size, cos_bit and index is a template constant, so each transform
// becomes straight-line VALU code on registers (no LDS, no scratch).  The
// arithmetic is the reference's (av1/common/av1_txfm.h:75-102 half_btf /
// round_shift; av1/common/av1_inv_txfm1d.h:22 clamp_value), the data flow is
// the DCT/ADST recursion described in DESIGN.md section "Transforms":
//   forward DCT  (av1/encoder/av1_fwd_txfm1d.c:16-1640): X[2k] from the
//     half-size DCT of x[i]+x[N-1-i]; X[2k+1] = O[bitrev(k)], O = odd half
//     built from "rotate block middles" + "mirror butterfly" levels.
//   forward ADST (av1_fwd_txfm1d.c:676-1062): permuted/negated inputs, then
//     rotation/butterfly levels of growing span, then a last rotation level.
//   inverse DCT / ADST (av1/common/av1_inv_txfm1d.c): the transposed DCT
//     graph and the reversed ADST graph, every add/sub clamped.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "txfm_consts.h"

namespace lavish {

// ----------------------------------------------------------------------------
// compile-time helpers
// ----------------------------------------------------------------------------
// Iterative (never recursive) so that LLVM inlines and folds them after the
// surrounding loops are unrolled: every index below must become a constant.
__host__ __device__ __forceinline__ constexpr int ce_log2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}
__host__ __device__ __forceinline__ constexpr int ce_bitrev(int v, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
  return r;
}
__host__ __device__ __forceinline__ constexpr int ce_popcount(int v) {
  int c = 0;
  for (; v; v >>= 1) c += v & 1;
  return c;
}

template <int BIT>
__device__ __forceinline__ constexpr int32_t cospi(int j) {
  return kCospi[BIT - 10][j];
}

// (int64)(int32)(w0*in0) + (int64)(int32)(w1*in1), rounded shift by BIT.
// The 32-bit products wrap exactly like the reference's int multiply.
// The 64-bit sum is evaluated exactly with 32-bit VALU ops:
//   floor((p0 + p1 + h) / 2^B) = (p0 >> B) + (p1 >> B)
//                                + (((p0 & m) + (p1 & m) + h) >> B)
// (arithmetic shifts floor; the low-part sum is < 3 * 2^B).
//
// FAST = the caller has certified (tools/range_analysis.py) that every operand
// is below 2^23 in magnitude and every sum below 2^31: then the products are
// v_mul_i32_i24 (full rate) and the sum fits one 32-bit register, giving the
// same bits with 4 VALU ops instead of ~10.
__device__ __forceinline__ int32_t sext24(int32_t x) { return (x << 8) >> 8; }

// The low 32 bits of the product of the operands' sign-extended low 24 bits
// (v_mul_i32_i24, full rate).  Written as the instruction: where the
// optimizer can prove an operand already fits 24 bits it drops the sign
// extension of __mul24 / sext24 forms, and the selector then falls back to
// the quarter-rate v_mul_lo_u32 (seen in rdo_kernel's dequantisation).
__device__ __forceinline__ int32_t mul_i24(int32_t a, int32_t b) {
  int32_t r;
  asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int BIT, bool FAST = false>
__device__ __forceinline__ int32_t hbtf(int32_t w0, int32_t in0, int32_t w1,
                                        int32_t in1) {
  if constexpr (FAST) {
    return (w0 * sext24(in0) + w1 * sext24(in1) + (1 << (BIT - 1))) >> BIT;
  } else {
    const int32_t p0 = (int32_t)((uint32_t)w0 * (uint32_t)in0);
    const int32_t p1 = (int32_t)((uint32_t)w1 * (uint32_t)in1);
    constexpr int32_t m = (1 << BIT) - 1, h = 1 << (BIT - 1);
    return (p0 >> BIT) + (p1 >> BIT) + (((p0 & m) + (p1 & m) + h) >> BIT);
  }
}

__device__ __forceinline__ int32_t rshift64(int64_t v, int bit) {
  return (int32_t)((v + ((int64_t)1 << (bit - 1))) >> bit);
}

__device__ __forceinline__ int32_t add32(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a + (uint32_t)b);
}
__device__ __forceinline__ int32_t sub32(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a - (uint32_t)b);
}

// av1_round_shift_array_c (av1/common/av1_txfm.c:71-87) for one value
template <int BIT>
__device__ __forceinline__ int32_t round_shift_1(int32_t v) {
  if constexpr (BIT == 0) {
    return v;
  } else if constexpr (BIT > 0) {
    return rshift64(v, BIT);
  } else {
    int64_t t = (int64_t)v * ((int64_t)1 << (-BIT));
    t = t > INT32_MAX ? INT32_MAX : (t < INT32_MIN ? INT32_MIN : t);
    return (int32_t)t;
  }
}

template <int BITS>
__device__ __forceinline__ int32_t clamp_bits(int32_t v) {
  constexpr int32_t hi = (int32_t)(((int64_t)1 << (BITS - 1)) - 1);
  constexpr int32_t lo = (int32_t)(-((int64_t)1 << (BITS - 1)));
  return v < lo ? lo : (v > hi ? hi : v);
}

// ----------------------------------------------------------------------------
// forward DCT
// ----------------------------------------------------------------------------
template <int M, int BIT, bool FAST = false>
__device__ __forceinline__ void fdct_odd(const int32_t* v, int32_t* O) {
  int32_t a[M], t[M];
#pragma unroll
  for (int i = 0; i < M; ++i) a[i] = v[i];
#pragma unroll
  for (int S = M; S >= 4; S >>= 1) {
#pragma unroll
    for (int i = 0; i < M; ++i) t[i] = a[i];
    const int nb = (M / 2) / S > 0 ? (M / 2) / S : 1;
    const int nbits = ce_log2(nb);
    const int base = 32 * S / M;
#pragma unroll
    for (int j = 0; j < M / 2; ++j) {
      const int lj = j % S;
      const int al = base * (1 + 4 * ce_bitrev(j / S, nbits));
      const int p = M - 1 - j;
      if (lj >= S / 4 && lj < S / 2) {
        t[j] = hbtf<BIT, FAST>(-cospi<BIT>(al), a[j], cospi<BIT>(64 - al), a[p]);
        t[p] = hbtf<BIT, FAST>(cospi<BIT>(al), a[p], cospi<BIT>(64 - al), a[j]);
      } else if (lj >= S / 2 && lj < 3 * S / 4) {
        t[j] = hbtf<BIT, FAST>(-cospi<BIT>(64 - al), a[j], -cospi<BIT>(al), a[p]);
        t[p] = hbtf<BIT, FAST>(cospi<BIT>(64 - al), a[p], -cospi<BIT>(al), a[j]);
      }
    }
    const int B = S / 2;
#pragma unroll
    for (int g = 0; g < M; g += B) {
      const bool typeB = (g / B) & 1;
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const int32_t x = t[g + j], y = t[g + B - 1 - j];
        const bool first = j < B / 2;
        a[g + j] = (first != typeB) ? add32(x, y) : sub32(y, x);
      }
    }
  }
  const int base = 32 / M;
  const int nbits = ce_log2(M / 2);
#pragma unroll
  for (int j = 0; j < M / 2; ++j) {
    const int be = base * (1 + 4 * ce_bitrev(j, nbits));
    const int p = M - 1 - j;
    O[j] = hbtf<BIT, FAST>(cospi<BIT>(64 - be), a[j], cospi<BIT>(be), a[p]);
    O[p] = hbtf<BIT, FAST>(cospi<BIT>(64 - be), a[p], -cospi<BIT>(be), a[j]);
  }
}

template <int N, int BIT, bool FAST = false>
__device__ __forceinline__ void fdct(const int32_t* x, int32_t* X) {
  if constexpr (N == 2) {
    X[0] = hbtf<BIT, FAST>(cospi<BIT>(32), x[0], cospi<BIT>(32), x[1]);
    X[1] = hbtf<BIT, FAST>(-cospi<BIT>(32), x[1], cospi<BIT>(32), x[0]);
  } else {
    constexpr int M = N / 2;
    int32_t e[M], v[M], E[M], O[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      e[i] = add32(x[i], x[N - 1 - i]);
      v[i] = sub32(x[M - 1 - i], x[M + i]);
    }
    fdct<M, BIT, FAST>(e, E);
    fdct_odd<M, BIT, FAST>(v, O);
#pragma unroll
    for (int k = 0; k < M; ++k) {
      X[2 * k] = E[k];
      X[2 * k + 1] = O[ce_bitrev(k, ce_log2(M))];
    }
  }
}

// ----------------------------------------------------------------------------
// forward ADST
// ----------------------------------------------------------------------------
template <int BIT, bool FAST = false>
__device__ __forceinline__ void fadst4(const int32_t* in, int32_t* out) {
  constexpr const int32_t* s = kSinpi[BIT - 10];
  // 32-bit products as in the reference (av1_fwd_txfm1d.c:695-721); in the
  // FAST range they are exact 24-bit multiplies.
  auto mul = [](int32_t w, int32_t x) -> int32_t {
    if constexpr (FAST) return w * sext24(x);
    else return (int32_t)((uint32_t)w * (uint32_t)x);
  };
  const int32_t x0 = in[0], x1 = in[1], x2 = in[2], x3 = in[3];
  // the reference returns zeros early for an all-zero input; the arithmetic
  // below yields exactly 0 for it as well, so no branch is needed.
  const int32_t s0 = mul(s[1], x0);
  const int32_t s1 = mul(s[4], x0);
  const int32_t s2 = mul(s[2], x1);
  const int32_t s3 = mul(s[1], x1);
  const int32_t s4 = mul(s[3], x2);
  const int32_t s5 = mul(s[4], x3);
  const int32_t s6 = mul(s[2], x3);
  const int32_t s7 = sub32(add32(x0, x1), x3);
  const int32_t a0 = add32(add32(s0, s2), s5);
  const int32_t a1 = mul(s[3], s7);
  const int32_t a2 = add32(sub32(s1, s3), s6);
  const int32_t a3 = s4;
  if constexpr (FAST) {
    out[0] = (add32(a0, a3) + (1 << (BIT - 1))) >> BIT;
    out[1] = (a1 + (1 << (BIT - 1))) >> BIT;
    out[2] = (sub32(a2, a3) + (1 << (BIT - 1))) >> BIT;
    out[3] = (add32(sub32(a2, a0), a3) + (1 << (BIT - 1))) >> BIT;
  } else {
    out[0] = rshift64(add32(a0, a3), BIT);
    out[1] = rshift64(a1, BIT);
    out[2] = rshift64(sub32(a2, a3), BIT);
    out[3] = rshift64(add32(sub32(a2, a0), a3), BIT);
  }
}

// a-sequence of the fadst input permutation: a -> (e, M-1-e) expansion
// a_k of the expansion a -> (e, M-1-e), a^(4) = {0, 1}: walk the bits of k
// from the top (level N/2 ... 4 contributes its bit).
__host__ __device__ __forceinline__ constexpr int adst_a(int N, int k) {
  const int levels = ce_log2(N) - 2;  // N=4:0, 8:1, 16:2
  int a = k >> levels;                // index into a^(4)
  int m = 4;
  for (int l = levels - 1; l >= 0; --l) {
    a = ((k >> l) & 1) ? (m - 1 - a) : a;
    m <<= 1;
  }
  return a;
}

template <int N, int BIT, bool FAST = false>
__device__ __forceinline__ void fadst(const int32_t* in, int32_t* out) {
  if constexpr (N == 4) {
    fadst4<BIT, FAST>(in, out);
  } else {
    int32_t b[N], t[N];
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
      const bool neg = ce_popcount(k) & 1;
      const int32_t p = in[adst_a(N, k)], q = in[N - 1 - adst_a(N, k)];
      b[2 * k] = neg ? -p : p;
      b[2 * k + 1] = neg ? q : -q;
    }
#pragma unroll
    for (int G = 4; G <= N; G <<= 1) {
#pragma unroll
      for (int i = 0; i < N; ++i) t[i] = b[i];
#pragma unroll
      for (int g = 0; g < N; g += G) {
        const int npairs = G / 4;
#pragma unroll
        for (int q = 0; q < npairs; ++q) {
          const int p = g + G / 2 + 2 * q;
          const int half = npairs / 2;
          if (G == 4 || q < half) {
            const int ph = (1 + 4 * (G == 4 ? 0 : q)) * 128 / G;
            t[p] = hbtf<BIT, FAST>(cospi<BIT>(ph), b[p], cospi<BIT>(64 - ph), b[p + 1]);
            t[p + 1] = hbtf<BIT, FAST>(cospi<BIT>(64 - ph), b[p], -cospi<BIT>(ph), b[p + 1]);
          } else {
            const int ph = (1 + 4 * (q - half)) * 128 / G;
            t[p] = hbtf<BIT, FAST>(-cospi<BIT>(64 - ph), b[p], cospi<BIT>(ph), b[p + 1]);
            t[p + 1] = hbtf<BIT, FAST>(cospi<BIT>(ph), b[p], cospi<BIT>(64 - ph), b[p + 1]);
          }
        }
      }
      const int s = G / 2;
#pragma unroll
      for (int g = 0; g < N; g += G) {
#pragma unroll
        for (int i = 0; i < s; ++i) {
          b[g + i] = add32(t[g + i], t[g + s + i]);
          b[g + s + i] = sub32(t[g + i], t[g + s + i]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
      const int th = (1 + 4 * j) * 32 / N;
      t[2 * j] = hbtf<BIT, FAST>(cospi<BIT>(th), b[2 * j], cospi<BIT>(64 - th), b[2 * j + 1]);
      t[2 * j + 1] = hbtf<BIT, FAST>(cospi<BIT>(64 - th), b[2 * j], -cospi<BIT>(th), b[2 * j + 1]);
    }
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
      out[2 * k] = t[2 * k + 1];
      out[2 * k + 1] = t[N - 2 - 2 * k];
    }
  }
}

// FAST: the inputs are half_btf operands of the certified range (< 2^23,
// tools/range_analysis.py), so the x 5793 products are one 24-bit multiply
// pair (v_mul_i32_i24 + v_mul_hi_i32_i24) instead of a quarter-rate 64-bit
// multiply
template <int N, bool FAST = false>
__device__ __forceinline__ void fidentity(const int32_t* in, int32_t* out) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int64_t x = FAST ? (int64_t)sext24(in[i]) : (int64_t)in[i];
    if constexpr (N == 4) out[i] = rshift64(x * 5793, 12);
    else if constexpr (N == 8) out[i] = (int32_t)((uint32_t)in[i] * 2u);
    else if constexpr (N == 16) out[i] = rshift64(x * (2 * 5793), 12);
    else out[i] = (int32_t)((uint32_t)in[i] * 4u);
  }
}

// kind: 0 DCT, 1 ADST, 2 IDENTITY (uniform across the workgroup)
template <int N, int BIT, bool FAST = false>
__device__ __forceinline__ void fwd_1d(int kind, const int32_t* in, int32_t* out) {
  if (kind == 0) {
    fdct<N, BIT, FAST>(in, out);
  } else if (kind == 1) {
    if constexpr (N <= 16) fadst<N, BIT, FAST>(in, out);
  } else {
    if constexpr (N <= 32) fidentity<N, FAST>(in, out);
  }
}

// ----------------------------------------------------------------------------
// inverse DCT / ADST / identity (clamp range RNG, cos_bit 12)
// ----------------------------------------------------------------------------
template <int M, int BIT, int RNG>
__device__ __forceinline__ void idct_odd(const int32_t* O, int32_t* v) {
  int32_t a[M], t[M];
  {
    const int base = 32 / M;
    const int nb = ce_log2(M / 2);
#pragma unroll
    for (int j = 0; j < M / 2; ++j) {
      const int be = base * (1 + 4 * ce_bitrev(j, nb));
      const int p = M - 1 - j;
      a[j] = hbtf<BIT>(cospi<BIT>(64 - be), O[j], -cospi<BIT>(be), O[p]);
      a[p] = hbtf<BIT>(cospi<BIT>(be), O[j], cospi<BIT>(64 - be), O[p]);
    }
  }
#pragma unroll
  for (int S = 4; S <= M; S <<= 1) {
    const int B = S / 2;
#pragma unroll
    for (int g = 0; g < M; g += B) {
      const bool typeB = (g / B) & 1;
#pragma unroll
      for (int j = 0; j < B / 2; ++j) {
        const int q = B - 1 - j;
        const int32_t yj = a[g + j], yq = a[g + q];
        if (!typeB) {
          t[g + j] = clamp_bits<RNG>(add32(yj, yq));
          t[g + q] = clamp_bits<RNG>(sub32(yj, yq));
        } else {
          t[g + j] = clamp_bits<RNG>(sub32(yq, yj));
          t[g + q] = clamp_bits<RNG>(add32(yj, yq));
        }
      }
    }
    const int nbk = (M / 2) / S > 0 ? (M / 2) / S : 1;
    const int nbits = ce_log2(nbk);
    const int rb = 32 * S / M;
#pragma unroll
    for (int i = 0; i < M; ++i) a[i] = t[i];
#pragma unroll
    for (int j = 0; j < M / 2; ++j) {
      const int lj = j % S;
      const int al = rb * (1 + 4 * ce_bitrev(j / S, nbits));
      const int p = M - 1 - j;
      if (lj >= S / 4 && lj < S / 2) {
        a[j] = hbtf<BIT>(-cospi<BIT>(al), t[j], cospi<BIT>(64 - al), t[p]);
        a[p] = hbtf<BIT>(cospi<BIT>(64 - al), t[j], cospi<BIT>(al), t[p]);
      } else if (lj >= S / 2 && lj < 3 * S / 4) {
        a[j] = hbtf<BIT>(-cospi<BIT>(64 - al), t[j], -cospi<BIT>(al), t[p]);
        a[p] = hbtf<BIT>(-cospi<BIT>(al), t[j], cospi<BIT>(64 - al), t[p]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < M; ++i) v[i] = a[i];
}

template <int N, int BIT, int RNG>
__device__ __forceinline__ void idct(const int32_t* X, int32_t* x) {
  if constexpr (N == 2) {
    x[0] = hbtf<BIT>(cospi<BIT>(32), X[0], cospi<BIT>(32), X[1]);
    x[1] = hbtf<BIT>(cospi<BIT>(32), X[0], -cospi<BIT>(32), X[1]);
  } else {
    constexpr int M = N / 2;
    int32_t ev[M], od[M], E[M], v[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      ev[k] = X[2 * k];
      od[ce_bitrev(k, ce_log2(M))] = X[2 * k + 1];
    }
    idct<M, BIT, RNG>(ev, E);
    idct_odd<M, BIT, RNG>(od, v);
#pragma unroll
    for (int i = 0; i < M; ++i) {
      x[i] = clamp_bits<RNG>(add32(E[i], v[M - 1 - i]));
      x[N - 1 - i] = clamp_bits<RNG>(sub32(E[i], v[M - 1 - i]));
    }
  }
}

template <int BIT>
__device__ __forceinline__ void iadst4(const int32_t* in, int32_t* out) {
  constexpr const int32_t* s = kSinpi[BIT - 10];
  const int32_t x0 = in[0], x1 = in[1], x2 = in[2], x3 = in[3];
  int32_t s0 = (int32_t)((uint32_t)s[1] * (uint32_t)x0);
  int32_t s1 = (int32_t)((uint32_t)s[2] * (uint32_t)x0);
  const int32_t s2 = (int32_t)((uint32_t)s[3] * (uint32_t)x1);
  const int32_t s3 = (int32_t)((uint32_t)s[4] * (uint32_t)x2);
  const int32_t s4 = (int32_t)((uint32_t)s[1] * (uint32_t)x2);
  const int32_t s5 = (int32_t)((uint32_t)s[2] * (uint32_t)x3);
  const int32_t s6 = (int32_t)((uint32_t)s[4] * (uint32_t)x3);
  const int32_t s7 = add32(sub32(x0, x2), x3);
  s0 = add32(add32(s0, s3), s5);
  s1 = sub32(sub32(s1, s4), s6);
  const int32_t r3 = s2;
  const int32_t r2 = (int32_t)((uint32_t)s[3] * (uint32_t)s7);
  out[0] = rshift64(add32(s0, r3), BIT);
  out[1] = rshift64(add32(s1, r3), BIT);
  out[2] = rshift64(r2, BIT);
  out[3] = rshift64(sub32(add32(s0, s1), r3), BIT);
}

template <int N, int BIT, int RNG>
__device__ __forceinline__ void iadst(const int32_t* in, int32_t* out) {
  if constexpr (N == 4) {
    iadst4<BIT>(in, out);
  } else {
    int32_t b[N], t[N];
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
      b[2 * k] = in[N - 1 - 2 * k];
      b[2 * k + 1] = in[2 * k];
    }
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
      const int th = (1 + 4 * j) * 32 / N;
      t[2 * j] = hbtf<BIT>(cospi<BIT>(th), b[2 * j], cospi<BIT>(64 - th), b[2 * j + 1]);
      t[2 * j + 1] = hbtf<BIT>(cospi<BIT>(64 - th), b[2 * j], -cospi<BIT>(th), b[2 * j + 1]);
    }
#pragma unroll
    for (int G = N; G >= 4; G >>= 1) {
      const int s = G / 2;
#pragma unroll
      for (int g = 0; g < N; g += G) {
#pragma unroll
        for (int i = 0; i < s; ++i) {
          b[g + i] = clamp_bits<RNG>(add32(t[g + i], t[g + s + i]));
          b[g + s + i] = clamp_bits<RNG>(sub32(t[g + i], t[g + s + i]));
        }
      }
#pragma unroll
      for (int i = 0; i < N; ++i) t[i] = b[i];
#pragma unroll
      for (int g = 0; g < N; g += G) {
        const int npairs = G / 4;
#pragma unroll
        for (int q = 0; q < npairs; ++q) {
          const int p = g + G / 2 + 2 * q;
          const int half = npairs / 2;
          if (G == 4 || q < half) {
            const int ph = (1 + 4 * (G == 4 ? 0 : q)) * 128 / G;
            t[p] = hbtf<BIT>(cospi<BIT>(ph), b[p], cospi<BIT>(64 - ph), b[p + 1]);
            t[p + 1] = hbtf<BIT>(cospi<BIT>(64 - ph), b[p], -cospi<BIT>(ph), b[p + 1]);
          } else {
            const int ph = (1 + 4 * (q - half)) * 128 / G;
            t[p] = hbtf<BIT>(-cospi<BIT>(64 - ph), b[p], cospi<BIT>(ph), b[p + 1]);
            t[p + 1] = hbtf<BIT>(cospi<BIT>(ph), b[p], cospi<BIT>(64 - ph), b[p + 1]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
      const bool neg = ce_popcount(k) & 1;
      out[adst_a(N, k)] = neg ? -t[2 * k] : t[2 * k];
      out[N - 1 - adst_a(N, k)] = neg ? t[2 * k + 1] : -t[2 * k + 1];
    }
  }
}

template <int N>
__device__ __forceinline__ void iidentity(const int32_t* in, int32_t* out) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if constexpr (N == 4) out[i] = rshift64((int64_t)5793 * in[i], 12);
    else if constexpr (N == 8) out[i] = (int32_t)((int64_t)in[i] * 2);
    else if constexpr (N == 16) out[i] = rshift64((int64_t)5793 * 2 * in[i], 12);
    else out[i] = (int32_t)((int64_t)in[i] * 4);
  }
}

template <int N, int BIT, int RNG>
__device__ __forceinline__ void inv_1d(int kind, const int32_t* in, int32_t* out) {
  if (kind == 0) {
    idct<N, BIT, RNG>(in, out);
  } else if (kind == 1) {
    if constexpr (N <= 16) iadst<N, BIT, RNG>(in, out);
  } else {
    if constexpr (N <= 32) iidentity<N>(in, out);
  }
}

// ----------------------------------------------------------------------------
// per-size configuration (av1/encoder/av1_fwd_txfm2d.c:314-358,
// av1/common/av1_inv_txfm2d.c:132-150)
// ----------------------------------------------------------------------------
template <int W, int H>
struct TxCfg {
  static constexpr int wl = ce_log2(W) - 2, hl = ce_log2(H) - 2;
  static constexpr int8_t kColBit[5][5] = {{13, 13, 13, 0, 0},
                                           {13, 13, 13, 12, 0},
                                           {13, 13, 13, 12, 13},
                                           {0, 13, 13, 12, 13},
                                           {0, 0, 13, 12, 13}};
  static constexpr int8_t kRowBit[5][5] = {{13, 13, 12, 0, 0},
                                           {13, 13, 13, 12, 0},
                                           {13, 13, 12, 13, 12},
                                           {0, 12, 13, 12, 11},
                                           {0, 0, 12, 11, 10}};
  static constexpr int cos_bit_col = kColBit[wl][hl];
  static constexpr int cos_bit_row = kRowBit[wl][hl];
  // forward shifts {shift0, shift1, shift2}
  static constexpr int s0 = (W == 64 && H == 64) || (W == 32 && H == 64) || (W == 16 && H == 64) ? 0 : 2;
  static constexpr int s1 =
      (W * H <= 16) ? 0
      : (W == 64 && H == 64) || (W == 32 && H == 64) || (W == 16 && H == 64) ? -2
      : (W == 8 && H == 8) || (W == 4 && H == 8) || (W == 8 && H == 4) || (W == 4 && H == 16) || (W == 16 && H == 4) ? -1
      : (W == 16 && H == 16) || (W == 8 && H == 16) || (W == 16 && H == 8) || (W == 8 && H == 32) || (W == 32 && H == 8) ? -2
      : -4;
  static constexpr int s2 = (W == 64 && H == 64) || (W == 32 && H == 64) || (W == 64 && H == 32) ? -2 : 0;
  static constexpr bool rect2 = (W == 2 * H) || (H == 2 * W);
  static constexpr int n_coef = (W == 64 || H == 64) ? ((W == 16 || H == 16) ? 512 : 1024) : W * H;
  static constexpr int log_scale = (W * H > 256) + (W * H > 1024);
  // inverse shifts
  static constexpr int is0 =
      (W == 4 && H == 4) || (W == 4 && H == 8) || (W == 8 && H == 4) ? 0
      : (W == 8 && H == 8) || (W == 8 && H == 16) || (W == 16 && H == 8) || (W == 16 && H == 32) ||
              (W == 32 && H == 16) || (W == 32 && H == 64) || (W == 64 && H == 32) || (W == 4 && H == 16) ||
              (W == 16 && H == 4)
          ? -1
          : -2;
  static constexpr int is1 = -4;
};

// Inverse-transform ranges per bit depth (index 0 -> 8, 1 -> 10, 2 -> 12):
// row / column stage ranges of av1_gen_inv_stage_range with opt_range_row /
// opt_range_col, and the input clamps of inv_txfm2d_add_c.
template <int BDI>
struct Bd {
  static constexpr int bd = 8 + 2 * BDI;
  static constexpr int rng_row = BDI == 0 ? 16 : (BDI == 1 ? 18 : 20);
  static constexpr int rng_col = BDI == 2 ? 18 : 16;
  static constexpr int clamp_in_row = bd + 8;
  static constexpr int clamp_in_col = bd + 6 > 16 ? bd + 6 : 16;
};

__device__ __forceinline__ int32_t rshift_r(int32_t v, int bit) {
  return bit == 0 ? v : (int32_t)(((int64_t)v + ((int64_t)1 << (bit - 1))) >> bit);
}

}  // namespace lavish
