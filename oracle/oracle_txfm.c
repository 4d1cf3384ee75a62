/*
 * oracle_txfm.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Forward transforms of the reference, restated.
 *   half_btf / round_shift           av1/common/av1_txfm.h:75-102
 *   av1_round_shift_array_c          av1/common/av1_txfm.c:71-87
 *   av1_fdct4..64                    av1/encoder/av1_fwd_txfm1d.c:16,59,144,315,1096
 *   av1_fadst4/8/16                  av1/encoder/av1_fwd_txfm1d.c:676,735,849
 *   av1_fidentity4..32_c             av1/encoder/av1_fwd_txfm1d.c:1064-1094
 *   fwd_txfm2d_c + 64-pt repack      av1/encoder/av1_fwd_txfm2d.c:56-312
 *   cfg tables                       av1/encoder/av1_fwd_txfm2d.c:314-423
 *
 * The DCT is written as the recursion its statement lists implement:
 * X[2k] = DCT_{N/2}(x[i] + x[N-1-i])[k] and X[2k+1] = O[bitrev(k)], where
 * the odd half O alternates "rotate the middle of each block" and
 * "mirror-butterfly" levels and ends with one rotation per output pair.  The
 * ADST is a fixed input permutation followed by alternating rotation /
 * butterfly levels.  Both are checked bit-exact against the golden vectors
 * produced from the reference statement lists (tests/test_oracle_golden.py).
 */
#include <assert.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static const int kTxW[ORC_TX_SIZES_ALL] = { 4,  8,  16, 32, 64, 4, 8,
                                            8,  16, 16, 32, 32, 64, 4,
                                            16, 8,  32, 16, 64 };
static const int kTxH[ORC_TX_SIZES_ALL] = { 4,  8,  16, 32, 64, 8, 4,
                                            16, 8,  32, 16, 64, 32, 16,
                                            4,  32, 8,  64, 16 };

int orc_tx_w(int s) { return kTxW[s]; }
int orc_tx_h(int s) { return kTxH[s]; }

int orc_max_eob(int s) {
  if (s == ORC_TX_16X64 || s == ORC_TX_64X16) return 512;
  if (kTxW[s] == 64 || kTxH[s] == 64) return 1024;
  return kTxW[s] * kTxH[s];
}

int orc_tx_scale(int s) {
  const int pels = kTxW[s] * kTxH[s];
  return (pels > 256) + (pels > 1024);
}

int orc_tx_type_valid(int s, int t) {
  const int m = kTxW[s] > kTxH[s] ? kTxW[s] : kTxH[s];
  if (m == 64) return t == 0;              /* EXT_TX_SET_DCTONLY */
  if (m == 32) return t == 0 || t == 9;    /* EXT_TX_SET_DCT_IDTX */
  return t >= 0 && t < 16;                 /* EXT_TX_SET_ALL16 */
}

/* ---- tables ---- */
static int32_t g_cospi[7][64];
static int g_tables_ready = 0;
/* sinpi: round(sqrt(2) sin(j pi/9) 2/3 2^bit) with the reference's
 * sinpi[1]+sinpi[2]==sinpi[4] adjustment (av1/common/av1_txfm.c:58-69). */
static const int32_t kSinpi[7][5] = {
  { 0, 330, 621, 836, 951 },       { 0, 660, 1241, 1672, 1901 },
  { 0, 1321, 2482, 3344, 3803 },   { 0, 2642, 4964, 6689, 7606 },
  { 0, 5283, 9929, 13377, 15212 }, { 0, 10566, 19858, 26755, 30424 },
  { 0, 21133, 39716, 53510, 60849 }
};

static void init_tables(void) {
  if (g_tables_ready) return;
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 64; ++j)
      g_cospi[i][j] = (int32_t)lround(cos(M_PI * j / 128.0) * (1 << (10 + i)));
  g_tables_ready = 1;
}

int32_t orc_cospi(int cos_bit, int idx) {
  init_tables();
  return g_cospi[cos_bit - 10][idx];
}
const int32_t *orc_cospi_table(int cos_bit) {
  init_tables();
  return g_cospi[cos_bit - 10];
}
int32_t orc_sinpi(int cos_bit, int idx) { return kSinpi[cos_bit - 10][idx]; }

/* fwd shifts per TX_SIZE (av1/encoder/av1_fwd_txfm2d.c:314-332) */
static const int8_t kFwdShift[ORC_TX_SIZES_ALL][3] = {
  { 2, 0, 0 },  { 2, -1, 0 }, { 2, -2, 0 }, { 2, -4, 0 },  { 0, -2, -2 },
  { 2, -1, 0 }, { 2, -1, 0 }, { 2, -2, 0 }, { 2, -2, 0 },  { 2, -4, 0 },
  { 2, -4, 0 }, { 0, -2, -2 }, { 2, -4, -2 }, { 2, -1, 0 }, { 2, -1, 0 },
  { 2, -2, 0 }, { 2, -2, 0 }, { 0, -2, 0 },  { 2, -4, 0 }
};
/* [log2(w)-2][log2(h)-2] (av1/encoder/av1_fwd_txfm2d.c:343-358) */
static const int8_t kCosBitCol[5][5] = { { 13, 13, 13, 0, 0 },
                                         { 13, 13, 13, 12, 0 },
                                         { 13, 13, 13, 12, 13 },
                                         { 0, 13, 13, 12, 13 },
                                         { 0, 0, 13, 12, 13 } };
static const int8_t kCosBitRow[5][5] = { { 13, 13, 12, 0, 0 },
                                         { 13, 13, 13, 12, 0 },
                                         { 13, 13, 12, 13, 12 },
                                         { 0, 12, 13, 12, 11 },
                                         { 0, 0, 12, 11, 10 } };

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

void orc_fwd_shift(int s, int8_t out[3]) { memcpy(out, kFwdShift[s], 3); }
int orc_fwd_cos_bit_col(int s) {
  return kCosBitCol[ilog2(kTxW[s]) - 2][ilog2(kTxH[s]) - 2];
}
int orc_fwd_cos_bit_row(int s) {
  return kCosBitRow[ilog2(kTxW[s]) - 2][ilog2(kTxH[s]) - 2];
}

/* ---- arithmetic primitives ---- */
static inline int32_t hbtf(int32_t w0, int32_t in0, int32_t w1, int32_t in1,
                           int bit) {
  /* the products are 32-bit (they wrap exactly like the C int multiply in the
   * reference), the sum is 64-bit */
  const int64_t r = (int64_t)(int32_t)((uint32_t)w0 * (uint32_t)in0) +
                    (int64_t)(int32_t)((uint32_t)w1 * (uint32_t)in1);
  return (int32_t)((r + ((int64_t)1 << (bit - 1))) >> bit);
}

static inline int32_t rshift(int64_t v, int bit) {
  return (int32_t)((v + ((int64_t)1 << (bit - 1))) >> bit);
}

static inline int32_t add32(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a + (uint32_t)b);
}
static inline int32_t sub32(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a - (uint32_t)b);
}

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

static int bitrev(int v, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
  return r;
}

/* ---- DCT ---- */
/* Odd half of the N-point DCT (M = N/2 inputs v[j] = x[M-1-j] - x[M+j]).
 * Output O[] in the reference's internal order (X[2k+1] = O[bitrev(k)]). */
static void fdct_odd(const int32_t *vin, int32_t *O, int M, const int32_t *c,
                     int bit) {
  int32_t a[32], t[32];
  memcpy(a, vin, sizeof(int32_t) * M);
  for (int S = M; S >= 4; S >>= 1) {
    /* rotation level, block size S; pairs (j, M-1-j), j in the first half */
    const int nb = (M / 2) / S > 0 ? (M / 2) / S : 1;
    const int nbits = ilog2(nb);
    const int base = 32 * S / M;
    memcpy(t, a, sizeof(int32_t) * M);
    for (int j = 0; j < M / 2; ++j) {
      const int lj = j % S;
      const int b = j / S;
      const int al = base * (1 + 4 * bitrev(b, nbits));
      const int p = M - 1 - j;
      if (lj >= S / 4 && lj < S / 2) {
        t[j] = hbtf(-c[al], a[j], c[64 - al], a[p], bit);
        t[p] = hbtf(c[al], a[p], c[64 - al], a[j], bit);
      } else if (lj >= S / 2 && lj < 3 * S / 4) {
        t[j] = hbtf(-c[64 - al], a[j], -c[al], a[p], bit);
        t[p] = hbtf(c[64 - al], a[p], -c[al], a[j], bit);
      }
    }
    /* mirror butterflies, block size B = S/2, blocks alternate A,B,A,B */
    const int B = S / 2;
    for (int g = 0; g < M; g += B) {
      const int typeB = (g / B) & 1;
      for (int j = 0; j < B; ++j) {
        const int32_t x = t[g + j], y = t[g + B - 1 - j];
        const int first = j < B / 2;
        if (first ^ typeB)
          a[g + j] = add32(x, y);
        else
          a[g + j] = sub32(y, x);
      }
    }
  }
  /* final rotations: O[j], O[M-1-j] with beta_j = (64/N)(1 + 4 bitrev(j)) */
  const int base = 32 / M;
  const int nbits = ilog2(M / 2);
  for (int j = 0; j < M / 2; ++j) {
    const int be = base * (1 + 4 * bitrev(j, nbits));
    const int p = M - 1 - j;
    O[j] = hbtf(c[64 - be], a[j], c[be], a[p], bit);
    O[p] = hbtf(c[64 - be], a[p], -c[be], a[j], bit);
  }
}

static void fdct(const int32_t *x, int32_t *X, int N, const int32_t *c,
                 int bit) {
  if (N == 2) {
    X[0] = hbtf(c[32], x[0], c[32], x[1], bit);
    X[1] = hbtf(-c[32], x[1], c[32], x[0], bit);
    return;
  }
  const int M = N / 2;
  int32_t e[32], v[32], E[32], O[32];
  for (int i = 0; i < M; ++i) {
    e[i] = add32(x[i], x[N - 1 - i]);
    v[i] = sub32(x[M - 1 - i], x[M + i]);
  }
  fdct(e, E, M, c, bit);
  fdct_odd(v, O, M, c, bit);
  const int mb = ilog2(M);
  for (int k = 0; k < M; ++k) {
    X[2 * k] = E[k];
    X[2 * k + 1] = O[bitrev(k, mb)];
  }
}

/* ---- ADST ---- */
static void fadst4(const int32_t *in, int32_t *out, int bit) {
  const int32_t *s = kSinpi[bit - 10];
  int32_t x0 = in[0], x1 = in[1], x2 = in[2], x3 = in[3];
  if (!(x0 | x1 | x2 | x3)) {
    out[0] = out[1] = out[2] = out[3] = 0;
    return;
  }
  /* av1/encoder/av1_fwd_txfm1d.c:695-727 (32-bit products) */
  const int32_t s0 = (int32_t)((uint32_t)s[1] * (uint32_t)x0);
  const int32_t s1 = (int32_t)((uint32_t)s[4] * (uint32_t)x0);
  const int32_t s2 = (int32_t)((uint32_t)s[2] * (uint32_t)x1);
  const int32_t s3 = (int32_t)((uint32_t)s[1] * (uint32_t)x1);
  const int32_t s4 = (int32_t)((uint32_t)s[3] * (uint32_t)x2);
  const int32_t s5 = (int32_t)((uint32_t)s[4] * (uint32_t)x3);
  const int32_t s6 = (int32_t)((uint32_t)s[2] * (uint32_t)x3);
  const int32_t s7 = sub32(add32(x0, x1), x3);
  int32_t a0 = add32(s0, s2);
  const int32_t a1 = (int32_t)((uint32_t)s[3] * (uint32_t)s7);
  int32_t a2 = sub32(s1, s3);
  const int32_t a3 = s4;
  a0 = add32(a0, s5);
  a2 = add32(a2, s6);
  const int32_t o0 = add32(a0, a3);
  const int32_t o2 = sub32(a2, a3);
  const int32_t o3 = add32(sub32(a2, a0), a3);
  out[0] = rshift(o0, bit);
  out[1] = rshift(a1, bit);
  out[2] = rshift(o2, bit);
  out[3] = rshift(o3, bit);
}

/* input permutation/sign of fadst8/16 (av1/encoder/av1_fwd_txfm1d.c:748,863):
 * slot 2k gets sign(k) x[a_k], slot 2k+1 gets -sign(k) x[N-1-a_k], where a
 * is built by a -> (e, M-1-e) expansion and sign(k) is the Thue-Morse bit. */
static void fadst_n(const int32_t *in, int32_t *out, int N, int bit) {
  const int32_t *c = g_cospi[bit - 10];
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
    const int neg = __builtin_popcount(k) & 1;
    const int32_t p = in[a_seq[k]], q = in[N - 1 - a_seq[k]];
    b[2 * k] = neg ? -p : p;
    b[2 * k + 1] = neg ? q : -q;
  }
  for (int G = 4; G <= N; G <<= 1) {
    /* rotation level on the second half of every G-group */
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
    /* butterflies of span G/2 inside every G-group */
    const int s = G / 2;
    for (int g = 0; g < N; g += G)
      for (int i = 0; i < s; ++i) {
        b[g + i] = add32(t[g + i], t[g + s + i]);
        b[g + s + i] = sub32(t[g + i], t[g + s + i]);
      }
  }
  /* last rotation level over all pairs, theta_j = (1 + 4j) 32 / N */
  for (int j = 0; j < N / 2; ++j) {
    const int th = (1 + 4 * j) * 32 / N;
    t[2 * j] = hbtf(c[th], b[2 * j], c[64 - th], b[2 * j + 1], bit);
    t[2 * j + 1] = hbtf(c[64 - th], b[2 * j], -c[th], b[2 * j + 1], bit);
  }
  for (int k = 0; k < N / 2; ++k) {
    out[2 * k] = t[2 * k + 1];
    out[2 * k + 1] = t[N - 2 - 2 * k];
  }
}

static void fidentity(const int32_t *in, int32_t *out, int n) {
  for (int i = 0; i < n; ++i) {
    switch (n) {
      case 4: out[i] = rshift((int64_t)in[i] * 5793, 12); break;
      case 8: out[i] = (int32_t)((uint32_t)in[i] * 2u); break;
      case 16: out[i] = rshift((int64_t)in[i] * 2 * 5793, 12); break;
      default: out[i] = (int32_t)((uint32_t)in[i] * 4u); break;
    }
  }
}

void orc_fwd_txfm1d(int kind, int n, const int32_t *in, int32_t *out,
                    int cos_bit) {
  init_tables();
  if (kind == 0) {
    fdct(in, out, n, g_cospi[cos_bit - 10], cos_bit);
  } else if (kind == 1) {
    if (n == 4)
      fadst4(in, out, cos_bit);
    else
      fadst_n(in, out, n, cos_bit);
  } else {
    fidentity(in, out, n);
  }
}

/* vtx_tab / htx_tab (av1/common/common_data.h:149-159): 0 DCT 1 ADST
 * 2 FLIPADST 3 IDTX */
static const int8_t kVtx[16] = { 0, 1, 0, 1, 2, 0, 2, 1, 2, 3, 0, 3, 1, 3, 2, 3 };
static const int8_t kHtx[16] = { 0, 0, 1, 1, 0, 2, 2, 2, 1, 3, 3, 0, 3, 1, 3, 2 };

void orc_fwd_txfm2d(const int16_t *input, int32_t *output, int stride,
                    int tx_type, int tx_size, int bd) {
  (void)bd; /* only feeds the (disabled) range checks, av1_fwd_txfm2d.c:41 */
  init_tables();
  const int W = kTxW[tx_size], H = kTxH[tx_size];
  const int8_t *shift = kFwdShift[tx_size];
  const int vt = kVtx[tx_type], ht = kHtx[tx_type];
  const int ud = vt == 2, lr = ht == 2;
  const int kc = vt == 3 ? 2 : (vt == 0 ? 0 : 1);
  const int kr = ht == 3 ? 2 : (ht == 0 ? 0 : 1);
  const int cbc = orc_fwd_cos_bit_col(tx_size);
  const int cbr = orc_fwd_cos_bit_row(tx_size);
  int rect = 0;
  if (W == 2 * H || H == 2 * W) rect = 1;
  int32_t buf[64 * 64];
  int32_t full[64 * 64];
  int32_t tin[64], tout[64];
  for (int c = 0; c < W; ++c) {
    for (int r = 0; r < H; ++r)
      tin[r] = input[(ud ? H - 1 - r : r) * stride + c];
    round_shift_array(tin, H, -shift[0]);
    orc_fwd_txfm1d(kc, H, tin, tout, cbc);
    round_shift_array(tout, H, -shift[1]);
    for (int r = 0; r < H; ++r) buf[r * W + (lr ? W - 1 - c : c)] = tout[r];
  }
  for (int r = 0; r < H; ++r) {
    orc_fwd_txfm1d(kr, W, buf + r * W, tout, cbr);
    round_shift_array(tout, W, -shift[2]);
    for (int c = 0; c < W; ++c) {
      int32_t v = tout[c];
      if (rect) v = rshift((int64_t)v * 5793, 12);
      full[c * H + r] = v;
    }
  }
  /* 64-point sizes: the reference zeroes the high-frequency half/quadrant and
   * re-packs the kept 32-row columns densely, in place
   * (av1_fwd_txfm2d.c:248-311); the same in-place steps are replayed here so
   * that every word of the output buffer matches, not only the first n. */
  memcpy(output, full, sizeof(int32_t) * W * H);
  if (H == 64) {
    for (int c = 0; c < (W < 32 ? W : 32); ++c)
      memset(output + c * 64 + 32, 0, 32 * sizeof(int32_t));
    if (W == 64) memset(output + 32 * 64, 0, 32 * 64 * sizeof(int32_t));
    for (int c = 1; c < (W < 32 ? W : 32); ++c)
      memmove(output + c * 32, output + c * 64, 32 * sizeof(int32_t));
  } else if (W == 64) {
    memset(output + H * 32, 0, (size_t)H * 32 * sizeof(int32_t));
  }
}

void orc_fwht4x4(const int16_t *input, int32_t *output, int stride) {
  /* av1/encoder/hybrid_fwd_txfm.c:24-76 */
  int64_t a, b, c, d, e;
  for (int i = 0; i < 4; ++i) {
    a = input[0 * stride + i];
    b = input[1 * stride + i];
    c = input[2 * stride + i];
    d = input[3 * stride + i];
    a += b;
    d = d - c;
    e = (a - d) >> 1;
    b = e - b;
    c = e - c;
    a -= c;
    d += b;
    output[4 * i + 0] = (int32_t)a;
    output[4 * i + 1] = (int32_t)c;
    output[4 * i + 2] = (int32_t)d;
    output[4 * i + 3] = (int32_t)b;
  }
  for (int i = 0; i < 4; ++i) {
    a = output[0 + i];
    b = output[4 + i];
    c = output[8 + i];
    d = output[12 + i];
    a += b;
    d -= c;
    e = (a - d) >> 1;
    b = e - b;
    c = e - c;
    a -= c;
    d += b;
    output[0 + i] = (int32_t)(a * 4);
    output[4 + i] = (int32_t)(c * 4);
    output[8 + i] = (int32_t)(d * 4);
    output[12 + i] = (int32_t)(b * 4);
  }
}
