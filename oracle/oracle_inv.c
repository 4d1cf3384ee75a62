/*
 * oracle_inv.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Inverse transforms of the reference, restated:
 *   av1_idct4..64, av1_iadst4/8/16, av1_iidentity*_c
 *                                  av1/common/av1_inv_txfm1d.c:16-1841
 *   clamp_value                    av1/common/av1_inv_txfm1d.h:22-27
 *   av1_get_inv_txfm_cfg / av1_gen_inv_stage_range / inv_txfm2d_add_c /
 *   64-point input re-expansion    av1/common/av1_inv_txfm2d.c:132-484
 *
 * The inverse DCT is the transpose of the forward flow graph of
 * oracle_txfm.c: bit-reversed odd inputs, transposed final rotations, then
 * per level the transposed mirror-butterflies (every add/sub clamped to the
 * stage range) and transposed middle rotations, and a last clamped
 * butterfly joining the even (recursive) and odd halves.  The inverse ADST
 * runs the forward ADST levels in reverse order with clamped butterflies and
 * undoes the forward input permutation at the end.  Checked bit-exact against
 * the golden vectors from the reference statement lists.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static inline int32_t hbtf(int32_t w0, int32_t in0, int32_t w1, int32_t in1,
                           int bit) {
  const int64_t r = (int64_t)(int32_t)((uint32_t)w0 * (uint32_t)in0) +
                    (int64_t)(int32_t)((uint32_t)w1 * (uint32_t)in1);
  return (int32_t)((r + ((int64_t)1 << (bit - 1))) >> bit);
}

static inline int32_t rshift(int64_t v, int bit) {
  return (int32_t)((v + ((int64_t)1 << (bit - 1))) >> bit);
}

static inline int32_t clampv(int64_t v32, int bit) {
  const int32_t v = (int32_t)v32;
  if (bit <= 0) return v;
  const int64_t hi = ((int64_t)1 << (bit - 1)) - 1, lo = -((int64_t)1 << (bit - 1));
  return (int32_t)(v < lo ? lo : (v > hi ? hi : v));
}

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

static int bitrev(int v, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
  return r;
}

/* transposed odd half: O[] (internal order) -> v[] with
 * v[j] pairing x[M-1-j] (plus) and x[M+j] (minus) in the last butterfly */
static void idct_odd(const int32_t *O, int32_t *v, int M, const int32_t *c,
                     int bit, int rng) {
  int32_t a[32], t[32];
  const int base = 32 / M;
  const int nb = ilog2(M / 2);
  for (int j = 0; j < M / 2; ++j) {
    const int be = base * (1 + 4 * bitrev(j, nb));
    const int p = M - 1 - j;
    a[j] = hbtf(c[64 - be], O[j], -c[be], O[p], bit);
    a[p] = hbtf(c[be], O[j], c[64 - be], O[p], bit);
  }
  for (int S = 4; S <= M; S <<= 1) {
    /* transposed mirror butterflies, block B = S/2 */
    const int B = S / 2;
    for (int g = 0; g < M; g += B) {
      const int typeB = (g / B) & 1;
      for (int j = 0; j < B / 2; ++j) {
        const int q = B - 1 - j;
        const int32_t yj = a[g + j], yq = a[g + q];
        if (!typeB) {
          t[g + j] = clampv((int64_t)yj + yq, rng);
          t[g + q] = clampv((int64_t)yj - yq, rng);
        } else {
          t[g + j] = clampv((int64_t)yq - yj, rng);
          t[g + q] = clampv((int64_t)yj + yq, rng);
        }
      }
    }
    /* transposed rotations of level S */
    const int nbk = (M / 2) / S > 0 ? (M / 2) / S : 1;
    const int nbits = ilog2(nbk);
    const int rb = 32 * S / M;
    memcpy(a, t, sizeof(int32_t) * M);
    for (int j = 0; j < M / 2; ++j) {
      const int lj = j % S;
      const int al = rb * (1 + 4 * bitrev(j / S, nbits));
      const int p = M - 1 - j;
      if (lj >= S / 4 && lj < S / 2) {
        a[j] = hbtf(-c[al], t[j], c[64 - al], t[p], bit);
        a[p] = hbtf(c[64 - al], t[j], c[al], t[p], bit);
      } else if (lj >= S / 2 && lj < 3 * S / 4) {
        a[j] = hbtf(-c[64 - al], t[j], -c[al], t[p], bit);
        a[p] = hbtf(-c[al], t[j], c[64 - al], t[p], bit);
      }
    }
  }
  memcpy(v, a, sizeof(int32_t) * M);
}

static void idct(const int32_t *X, int32_t *x, int N, const int32_t *c, int bit,
                 int rng) {
  if (N == 2) {
    x[0] = hbtf(c[32], X[0], c[32], X[1], bit);
    x[1] = hbtf(c[32], X[0], -c[32], X[1], bit);
    return;
  }
  const int M = N / 2;
  int32_t ev[32], od[32], E[32], v[32];
  const int mb = ilog2(M);
  for (int k = 0; k < M; ++k) {
    ev[k] = X[2 * k];
    od[bitrev(k, mb)] = X[2 * k + 1];
  }
  idct(ev, E, M, c, bit, rng);
  idct_odd(od, v, M, c, bit, rng);
  for (int i = 0; i < M; ++i) {
    x[i] = clampv((int64_t)E[i] + v[M - 1 - i], rng);
    x[N - 1 - i] = clampv((int64_t)E[i] - v[M - 1 - i], rng);
  }
}

static void iadst4(const int32_t *in, int32_t *out, int bit) {
  /* av1/common/av1_inv_txfm1d.c:656-711 */
  static const int32_t kS[7][5] = {
    { 0, 330, 621, 836, 951 },       { 0, 660, 1241, 1672, 1901 },
    { 0, 1321, 2482, 3344, 3803 },   { 0, 2642, 4964, 6689, 7606 },
    { 0, 5283, 9929, 13377, 15212 }, { 0, 10566, 19858, 26755, 30424 },
    { 0, 21133, 39716, 53510, 60849 }
  };
  const int32_t *s = kS[bit - 10];
  int32_t x0 = in[0], x1 = in[1], x2 = in[2], x3 = in[3];
  if (!(x0 | x1 | x2 | x3)) {
    out[0] = out[1] = out[2] = out[3] = 0;
    return;
  }
#define M32(a, b) ((int32_t)((uint32_t)(a) * (uint32_t)(b)))
#define A32(a, b) ((int32_t)((uint32_t)(a) + (uint32_t)(b)))
#define S32(a, b) ((int32_t)((uint32_t)(a) - (uint32_t)(b)))
  int32_t s0 = M32(s[1], x0), s1 = M32(s[2], x0), s2 = M32(s[3], x1);
  int32_t s3 = M32(s[4], x2), s4 = M32(s[1], x2), s5 = M32(s[2], x3);
  int32_t s6 = M32(s[4], x3);
  const int32_t s7 = A32(S32(x0, x2), x3);
  s0 = A32(s0, s3);
  s1 = S32(s1, s4);
  s3 = s2;
  s2 = M32(s[3], s7);
  s0 = A32(s0, s5);
  s1 = S32(s1, s6);
  x0 = A32(s0, s3);
  x1 = A32(s1, s3);
  x2 = s2;
  x3 = A32(s0, s1);
  x3 = S32(x3, s3);
  out[0] = rshift(x0, bit);
  out[1] = rshift(x1, bit);
  out[2] = rshift(x2, bit);
  out[3] = rshift(x3, bit);
#undef M32
#undef A32
#undef S32
}

static void iadst_n(const int32_t *in, int32_t *out, int N, const int32_t *c,
                    int bit, int rng) {
  int a_seq[8] = { 0, 1 };
  int len = 2;
  for (int m = 4; m <= N / 2; m <<= 1) {
    int nxt[8];
    for (int i = 0; i < len; ++i) {
      nxt[2 * i] = a_seq[i];
      nxt[2 * i + 1] = m - 1 - a_seq[i];
    }
    len *= 2;
    memcpy(a_seq, nxt, sizeof(int) * len);
  }
  int32_t b[16], t[16];
  for (int k = 0; k < N / 2; ++k) {
    b[2 * k] = in[N - 1 - 2 * k];
    b[2 * k + 1] = in[2 * k];
  }
  for (int j = 0; j < N / 2; ++j) {
    const int th = (1 + 4 * j) * 32 / N;
    t[2 * j] = hbtf(c[th], b[2 * j], c[64 - th], b[2 * j + 1], bit);
    t[2 * j + 1] = hbtf(c[64 - th], b[2 * j], -c[th], b[2 * j + 1], bit);
  }
  for (int G = N; G >= 4; G >>= 1) {
    const int s = G / 2;
    for (int g = 0; g < N; g += G)
      for (int i = 0; i < s; ++i) {
        b[g + i] = clampv((int64_t)t[g + i] + t[g + s + i], rng);
        b[g + s + i] = clampv((int64_t)t[g + i] - t[g + s + i], rng);
      }
    memcpy(t, b, sizeof(int32_t) * N);
    for (int g = 0; g < N; g += G) {
      const int npairs = G / 4;
      for (int q = 0; q < npairs; ++q) {
        const int p = g + G / 2 + 2 * q;
        const int half = npairs / 2;
        if (G == 4 || q < half) {
          const int ph = (1 + 4 * (G == 4 ? 0 : q)) * 128 / G;
          t[p] = hbtf(c[ph], b[p], c[64 - ph], b[p + 1], bit);
          t[p + 1] = hbtf(c[64 - ph], b[p], -c[ph], b[p + 1], bit);
        } else {
          const int ph = (1 + 4 * (q - half)) * 128 / G;
          t[p] = hbtf(-c[64 - ph], b[p], c[ph], b[p + 1], bit);
          t[p + 1] = hbtf(c[ph], b[p], c[64 - ph], b[p + 1], bit);
        }
      }
    }
  }
  for (int k = 0; k < N / 2; ++k) {
    const int neg = __builtin_popcount(k) & 1;
    out[a_seq[k]] = neg ? -t[2 * k] : t[2 * k];
    out[N - 1 - a_seq[k]] = neg ? t[2 * k + 1] : -t[2 * k + 1];
  }
}

static void iidentity(const int32_t *in, int32_t *out, int n) {
  for (int i = 0; i < n; ++i) {
    switch (n) {
      case 4: out[i] = rshift((int64_t)5793 * in[i], 12); break;
      case 8: out[i] = (int32_t)((int64_t)in[i] * 2); break;
      case 16: out[i] = rshift((int64_t)5793 * 2 * in[i], 12); break;
      default: out[i] = (int32_t)((int64_t)in[i] * 4); break;
    }
  }
}

void orc_inv_txfm1d(int kind, int n, const int32_t *in, int32_t *out,
                    int cos_bit, const int8_t *stage_range) {
  const int rng = stage_range ? stage_range[1] : 0;
  if (kind == 0) {
    idct(in, out, n, &orc_cospi_table(cos_bit)[0], cos_bit, rng);
  } else if (kind == 1) {
    if (n == 4)
      iadst4(in, out, cos_bit);
    else
      iadst_n(in, out, n, &orc_cospi_table(cos_bit)[0], cos_bit, rng);
  } else {
    iidentity(in, out, n);
  }
}

static const int kTxW[ORC_TX_SIZES_ALL] = { 4,  8,  16, 32, 64, 4, 8,
                                            8,  16, 16, 32, 32, 64, 4,
                                            16, 8,  32, 16, 64 };
static const int kTxH[ORC_TX_SIZES_ALL] = { 4,  8,  16, 32, 64, 8, 4,
                                            16, 8,  32, 16, 64, 32, 16,
                                            4,  32, 8,  64, 16 };
/* inv_shift_* (av1/common/av1_inv_txfm2d.c:132-150) */
static const int8_t kInvShift[ORC_TX_SIZES_ALL][2] = {
  { 0, -4 },  { -1, -4 }, { -2, -4 }, { -2, -4 }, { -2, -4 },
  { 0, -4 },  { 0, -4 },  { -1, -4 }, { -1, -4 }, { -1, -4 },
  { -1, -4 }, { -1, -4 }, { -1, -4 }, { -1, -4 }, { -1, -4 },
  { -2, -4 }, { -2, -4 }, { -2, -4 }, { -2, -4 }
};
static const int8_t kVtx[16] = { 0, 1, 0, 1, 2, 0, 2, 1, 2, 3, 0, 3, 1, 3, 2, 3 };
static const int8_t kHtx[16] = { 0, 0, 1, 1, 0, 2, 2, 2, 1, 3, 3, 0, 3, 1, 3, 2 };

static void round_shift_array(int32_t *a, int n, int bit) {
  if (bit == 0) return;
  if (bit > 0) {
    for (int i = 0; i < n; ++i) a[i] = rshift(a[i], bit);
  } else {
    for (int i = 0; i < n; ++i) {
      int64_t v = ((int64_t)1 << (-bit)) * a[i];
      if (v > INT32_MAX) v = INT32_MAX;
      if (v < INT32_MIN) v = INT32_MIN;
      a[i] = (int32_t)v;
    }
  }
}

void orc_inv_txfm2d_add(const int32_t *input, uint16_t *output, int stride,
                        int tx_type, int tx_size, int bd) {
  const int W = kTxW[tx_size], H = kTxH[tx_size];
  /* 64-point sizes receive the packed low-frequency quadrant */
  int32_t *in = (int32_t *)calloc((size_t)W * H, sizeof(int32_t));
  if (W == 64 || H == 64) {
    const int kw = W > 32 ? 32 : W, kh = H > 32 ? 32 : H;
    for (int c = 0; c < kw; ++c)
      for (int r = 0; r < kh; ++r) in[c * H + r] = input[c * kh + r];
  } else {
    memcpy(in, input, sizeof(int32_t) * W * H);
  }
  const int vt = kVtx[tx_type], ht = kHtx[tx_type];
  const int ud = vt == 2, lr = ht == 2;
  const int kc = vt == 3 ? 2 : (vt == 0 ? 0 : 1);
  const int kr = ht == 3 ? 2 : (ht == 0 ? 0 : 1);
  const int8_t *shift = kInvShift[tx_size];
  const int rect = (W == 2 * H || H == 2 * W);
  const int opt_row = bd == 8 ? 16 : (bd == 10 ? 18 : 20);
  const int opt_col = bd == 12 ? 18 : 16;
  int8_t sr_row[12], sr_col[12];
  memset(sr_row, opt_row, sizeof(sr_row));
  memset(sr_col, opt_col, sizeof(sr_col));
  const int cb = 12; /* INV_COS_BIT, av1/common/av1_inv_txfm1d_cfg.h:43 */
  int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * W * H);
  int32_t tin[64], tout[64];
  const int hi8 = bd + 8, hi6 = bd + 6 > 16 ? bd + 6 : 16;
  for (int r = 0; r < H; ++r) {
    for (int c = 0; c < W; ++c) {
      int32_t v = in[c * H + r];
      if (rect) v = rshift((int64_t)v * 2896, 12);
      tin[c] = clampv(v, hi8);
    }
    orc_inv_txfm1d(kr, W, tin, buf + r * W, cb, sr_row);
    round_shift_array(buf + r * W, W, -shift[0]);
  }
  const int maxv = (1 << bd) - 1;
  for (int c = 0; c < W; ++c) {
    for (int r = 0; r < H; ++r)
      tin[r] = clampv(buf[r * W + (lr ? W - 1 - c : c)], hi6);
    orc_inv_txfm1d(kc, H, tin, tout, cb, sr_col);
    round_shift_array(tout, H, -shift[1]);
    for (int r = 0; r < H; ++r) {
      const int v = output[r * stride + c] + tout[ud ? H - 1 - r : r];
      output[r * stride + c] = (uint16_t)(v < 0 ? 0 : (v > maxv ? maxv : v));
    }
  }
  free(buf);
  free(in);
}
