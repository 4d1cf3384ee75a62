#!/usr/bin/env python3
"""Worst-case magnitude analysis of the forward 2-D transforms (symmetric
interval propagation through the same DCT/ADST/identity graphs the kernels
run).  For an input bound |residual| <= T it reports, per TX size:
  * max |operand| fed to a half_btf multiply (must be < 2^23 for v_mul_i24)
  * max |w0*x0 + w1*x1 + round| (must be < 2^31 for a 32-bit mad chain)
The FAST kernel path is taken only when the whole workgroup's residual obeys
the threshold this script certifies (DESIGN.md "Exact fast path")."""
import math, sys

def cospi(bit):
    return [int(round(math.cos(math.pi * j / 128) * (1 << bit))) for j in range(64)]

SINPI = {b: v for b, v in zip(range(10, 17), [[0, 330, 621, 836, 951], [0, 660, 1241, 1672, 1901],
         [0, 1321, 2482, 3344, 3803], [0, 2642, 4964, 6689, 7606], [0, 5283, 9929, 13377, 15212],
         [0, 10566, 19858, 26755, 30424], [0, 21133, 39716, 53510, 60849]])}

class St:
    def __init__(s): s.op = 0; s.sum = 0

def hb(st, w0, a, w1, b, bit):
    st.op = max(st.op, a, b)
    S = abs(w0) * a + abs(w1) * b + (1 << (bit - 1))
    st.sum = max(st.sum, S)
    return (S + (1 << bit) - 1) >> bit

def ilog2(v):
    l = 0
    while (1 << l) < v: l += 1
    return l

def bitrev(v, bits):
    r = 0
    for i in range(bits): r |= ((v >> i) & 1) << (bits - 1 - i)
    return r

def fdct_odd(st, v, M, c, bit):
    a = list(v)
    S = M
    while S >= 4:
        t = list(a)
        nb = max((M // 2) // S, 1); nbits = ilog2(nb); base = 32 * S // M
        for j in range(M // 2):
            lj = j % S; al = base * (1 + 4 * bitrev(j // S, nbits)); p = M - 1 - j
            if S // 4 <= lj < S // 2 or S // 2 <= lj < 3 * S // 4:
                t[j] = hb(st, c[al], a[j], c[64 - al], a[p], bit)
                t[p] = hb(st, c[al], a[p], c[64 - al], a[j], bit)
        B = S // 2
        for g in range(0, M, B):
            for j in range(B):
                a[g + j] = t[g + j] + t[g + B - 1 - j]
        S //= 2
    base = 32 // M; nbits = ilog2(M // 2); O = [0] * M
    for j in range(M // 2):
        be = base * (1 + 4 * bitrev(j, nbits)); p = M - 1 - j
        O[j] = hb(st, c[64 - be], a[j], c[be], a[p], bit)
        O[p] = hb(st, c[64 - be], a[p], c[be], a[j], bit)
    return O

def fdct(st, x, N, c, bit):
    if N == 2:
        v = hb(st, c[32], x[0], c[32], x[1], bit)
        return [v, v]
    M = N // 2
    e = [x[i] + x[N - 1 - i] for i in range(M)]
    v = [x[M - 1 - i] + x[M + i] for i in range(M)]
    E = fdct(st, e, M, c, bit); O = fdct_odd(st, v, M, c, bit)
    X = [0] * N
    for k in range(M):
        X[2 * k] = E[k]; X[2 * k + 1] = O[bitrev(k, ilog2(M))]
    return X

def fadst(st, x, N, c, bit):
    if N == 4:
        s = SINPI[bit]; m = max(x)
        # all products and sums in 32 bits (no 64-bit sum in fadst4)
        st.op = max(st.op, 3 * m)
        tot = (s[1] + s[2] + s[4] + s[3] + s[1]) * m + s[3] * 3 * m
        st.sum = max(st.sum, tot)
        return [(tot + (1 << bit) - 1) >> bit] * 4
    b = list(x)
    G = 4
    while G <= N:
        t = list(b)
        for g in range(0, N, G):
            for q in range(G // 4):
                p = g + G // 2 + 2 * q
                t[p] = hb(st, c[32], b[p], c[32], b[p + 1], bit) if G == 4 else hb(st, c[16], b[p], c[48], b[p + 1], bit) * 0 + max(hb(st, c[k], b[p], c[64 - k], b[p + 1], bit) for k in range(1, 64))
                t[p + 1] = t[p]
        s = G // 2
        for g in range(0, N, G):
            for i in range(s):
                b[g + i] = t[g + i] + t[g + s + i]; b[g + s + i] = b[g + i]
        G *= 2
    out = [max(hb(st, c[k], b[2 * j], c[64 - k], b[2 * j + 1], bit) for k in range(1, 64)) for j in range(N // 2)]
    return [max(out)] * N

def fidt(x, N):
    return [int(math.ceil(v * {4: 5793 / 4096, 8: 2, 16: 2 * 5793 / 4096, 32: 4}[N])) + 1 for v in x]

def one_d(st, kind, x, N, bit):
    c = cospi(bit)
    if kind == 0: return fdct(st, x, N, c, bit)
    if kind == 1: return fadst(st, x, N, c, bit)
    return fidt(x, N)

SHIFT = {(4, 4): (2, 0, 0), (8, 8): (2, -1, 0), (16, 16): (2, -2, 0), (32, 32): (2, -4, 0),
         (4, 8): (2, -1, 0), (8, 4): (2, -1, 0), (8, 16): (2, -2, 0), (16, 8): (2, -2, 0),
         (16, 32): (2, -4, 0), (32, 16): (2, -4, 0), (4, 16): (2, -1, 0), (16, 4): (2, -1, 0),
         (8, 32): (2, -2, 0), (32, 8): (2, -2, 0),
         # 64-point sizes (DCT_DCT only; fwd_shift_* of av1_fwd_txfm2d.c)
         (64, 64): (0, -2, -2), (32, 64): (0, -2, -2), (64, 32): (2, -4, -2),
         (16, 64): (0, -2, 0), (64, 16): (2, -4, 0)}
CBC = [[13, 13, 13, 0, 0], [13, 13, 13, 12, 0], [13, 13, 13, 12, 13], [0, 13, 13, 12, 13], [0, 0, 13, 12, 13]]
CBR = [[13, 13, 12, 0, 0], [13, 13, 13, 12, 0], [13, 13, 12, 13, 12], [0, 12, 13, 12, 11], [0, 0, 12, 11, 10]]

_last_out = [0]


def analyse(W, H, T):
    st = St()
    s0, s1, s2 = SHIFT[(W, H)]
    wl, hl = ilog2(W) - 2, ilog2(H) - 2
    worst_row_in = 0
    for kc in (0, 1, 2):
        if kc == 1 and H > 16: continue
        if kc != 0 and (W == 64 or H == 64): continue
        col = one_d(st, kc, [T << s0] * H, H, CBC[wl][hl])
        m = max(col)
        m = (m + (1 << -s1) - 1) >> -s1 if s1 < 0 else m
        worst_row_in = max(worst_row_in, m)
    out = 0
    for kr in (0, 1, 2):
        if kr == 1 and W > 16: continue
        if kr != 0 and (W == 64 or H == 64): continue
        row = one_d(st, kr, [worst_row_in] * W, W, CBR[wl][hl])
        m = max(row)
        m = (m + (1 << -s2) - 1) >> -s2 if s2 < 0 else m << s2
        if 2 * W == H or 2 * H == W:   # the 2:1 sizes' NewSqrt2 scaling (x 5793 >> 12)
            m = (m * 5793 + 4095) >> 12
        out = max(out, m)
    _last_out[0] = out
    return st.op, st.sum


def coeff_bound(W, H, T):
    """max |coefficient| out of the forward 2-D transform of a residual
    bounded by T (what the quantizer and the block error see)."""
    analyse(W, H, T)
    return _last_out[0]

if __name__ == "__main__":
    for T in (255, 1023, 4095):
        print("T =", T)
        for (W, H) in SHIFT:
            op, sm = analyse(W, H, T)
            print("  %2dx%-2d  max|operand| 2^%.2f  max|sum| 2^%.2f  max|coeff| 2^%.2f  %s" % (
                W, H, math.log2(op), math.log2(sm), math.log2(_last_out[0]),
                "OK" if op < 2 ** 23 and sm < 2 ** 31 else "--"))
