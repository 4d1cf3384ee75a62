"""Pins the oracle's pixel kernels (oracle/oracle_dsp.c) to the reference's own
tests: the checkers those tests hold (restated here in numpy, each citing its
file:line), driven by the same input patterns (ACMRandom with the gtest seed,
extremes, strides) and the tests' closed-form known answers.

The reference's C sources cannot be compiled here without its generated
config headers ("Oracle"), so this is how parity is pinned for
rows a10-a16 of SURVEY.md section 8."""
import numpy as np
import pytest

import _oracle as O

SIZES = [(128, 128), (128, 64), (64, 128), (64, 64), (64, 32), (32, 64), (32, 32), (32, 16),
         (16, 32), (16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4), (4, 16), (16, 4),
         (8, 32), (32, 8), (16, 64), (64, 16)]


# --------------------------------------------- checkers of the ref tests --
def ref_sad(src, ref, w, h, skip=False):
    """test/sad_test.cc:182-226 ReferenceSAD / ReferenceSADSkip."""
    rows = slice(0, h, 2) if skip else slice(0, h)
    s = int(np.abs(src[rows, :w].astype(np.int64) - ref[rows, :w].astype(np.int64)).sum())
    return (2 * s) & 0xFFFFFFFF if skip else s & 0xFFFFFFFF


def ref_sad_avg(src, ref, second, w, h):
    """test/sad_test.cc:231-256 ReferenceSADavg."""
    comp = (second[:h, :w].astype(np.int64) + ref[:h, :w] + 1) >> 1
    return int(np.abs(src[:h, :w].astype(np.int64) - comp).sum()) & 0xFFFFFFFF


def _round_hbd(bd, se, sse):
    """test/variance_test.cc:74-88 RoundHighBitDepth."""
    if bd == 12:
        return (se + 8) >> 4, (sse + 128) >> 8
    if bd == 10:
        return (se + 2) >> 2, (sse + 8) >> 4
    return se, sse


def ref_variance(src, ref, w, h, bd=8):
    """test/variance_test.cc:103-131 variance_ref (diff = src - ref)."""
    d = src[:h, :w].astype(np.int64) - ref[:h, :w].astype(np.int64)
    se, sse = _round_hbd(bd, int(d.sum()), int((d * d).sum()))
    sse32 = sse & 0xFFFFFFFF
    return (sse - ((se * se) >> (int(np.log2(w)) + int(np.log2(h))))) & 0xFFFFFFFF, sse32


def ref_subpel_variance(ref, src, w, h, xoff, yoff, bd=8, second=None):
    """test/variance_test.cc:138-180 subpel_variance_ref and :182-230
    subpel_avg_variance_ref: 16th-pel bilinear written as a1 + ((a2-a1)*x+8)>>4
    over a (h+1) x (w+1) ref block of stride w+1."""
    r = ref.astype(np.int64)
    x, y = xoff << 1, yoff << 1
    a = r[:h, :w] + (((r[:h, 1:w + 1] - r[:h, :w]) * x + 8) >> 4)
    b = r[1:h + 1, :w] + (((r[1:h + 1, 1:w + 1] - r[1:h + 1, :w]) * x + 8) >> 4)
    p = a + (((b - a) * y + 8) >> 4)
    if second is not None:
        p = (p + second[:h, :w].astype(np.int64) + 1) >> 1
    d = p - src[:h, :w].astype(np.int64)
    se, sse = _round_hbd(bd, int(d.sum()), int((d * d).sum()))
    return (sse - ((se * se) >> (int(np.log2(w)) + int(np.log2(h))))) & 0xFFFFFFFF, \
        sse & 0xFFFFFFFF


def _had4_pass(a):
    """test/hadamard_test.cc:35-47 Hadamard4x4 over columns of a 4x4 array."""
    b0 = (a[0] + a[1]) >> 1
    b1 = (a[0] - a[1]) >> 1
    b2 = (a[2] + a[3]) >> 1
    b3 = (a[2] - a[3]) >> 1
    return np.stack([b0 + b2, b1 + b3, b0 - b2, b1 - b3])


def _had8_pass(a):
    """test/hadamard_test.cc:69-93 HadamardLoop over columns of an 8xk array."""
    b = [a[2 * i] + a[2 * i + 1] if k == 0 else a[2 * i] - a[2 * i + 1]
         for i in range(4) for k in range(2)]
    c = []
    for i in (0, 4):
        c += [b[i] + b[i + 2], b[i + 1] + b[i + 3], b[i] - b[i + 2], b[i + 1] - b[i + 3]]
    out = [None] * 8
    out[0] = c[0] + c[4]
    out[7] = c[1] + c[5]
    out[3] = c[2] + c[6]
    out[4] = c[3] + c[7]
    out[2] = c[0] - c[4]
    out[6] = c[1] - c[5]
    out[1] = c[2] - c[6]
    out[5] = c[3] - c[7]
    return np.stack(out)


def _ref_had_small(blk, n):
    """ReferenceHadamard4x4 / 8x8 (hadamard_test.cc:49-117): input[i*n+j] =
    a[i][j]; pass 1 over the columns, pass 2 over the rows of that, then the
    extra transpose."""
    inp = blk.astype(np.int64)
    p = _had4_pass if n == 4 else _had8_pass
    buf = p(inp)                    # buf[k][i]: output k of column i -> stored buf[i*n+k]
    buf_mem = buf.T                 # memory layout buf[i][k]
    out = p(buf_mem)                # second: column i of buf_mem -> b[i*n+k] = out[k][i]
    b = out.T                       # b[i][k]
    return b.T.reshape(-1)          # extra transpose


def ref_hadamard(blk, n, shift=True):
    """test/hadamard_test.cc:127-215 ReferenceHadamard (lowbd, do_shift=true)."""
    if n in (4, 8):
        return _ref_had_small(blk, n)
    if n == 16:
        b = np.concatenate([_ref_had_small(blk[0:8, 0:8], 8), _ref_had_small(blk[0:8, 8:16], 8),
                            _ref_had_small(blk[8:16, 0:8], 8),
                            _ref_had_small(blk[8:16, 8:16], 8)])
        a0, a1, a2, a3 = b[0:64], b[64:128], b[128:192], b[192:256]
        b0, b1, b2, b3 = (a0 + a1) >> 1, (a0 - a1) >> 1, (a2 + a3) >> 1, (a2 - a3) >> 1
        b = np.concatenate([b0 + b2, b1 + b3, b0 - b2, b1 - b3])
        if shift:
            m = b.reshape(16, 16).copy()
            m[:, 4:8], m[:, 8:12] = b.reshape(16, 16)[:, 8:12], b.reshape(16, 16)[:, 4:8]
            b = m.reshape(-1)
        return b
    b = np.concatenate([ref_hadamard(blk[0:16, 0:16], 16, shift),
                        ref_hadamard(blk[0:16, 16:32], 16, shift),
                        ref_hadamard(blk[16:32, 0:16], 16, shift),
                        ref_hadamard(blk[16:32, 16:32], 16, shift)])
    a0, a1, a2, a3 = b[0:256], b[256:512], b[512:768], b[768:1024]
    b0, b1, b2, b3 = (a0 + a1) >> 2, (a0 - a1) >> 2, (a2 + a3) >> 2, (a2 - a3) >> 2
    return np.concatenate([b0 + b2, b1 + b3, b0 - b2, b1 - b3])


def _fill(rnd, n, fn):
    return np.array([fn() for _ in range(n)])


# ---------------------------------------------------------------- tests --
@pytest.mark.parametrize("w,h", SIZES)
def test_sad_vs_reference_checker(w, h):
    rnd = O.ACMRandom()
    stride = w + 8
    for trial in range(3):
        if trial == 0:  # MaxRef (sad_test.cc): src 0, ref 255
            src = np.zeros((h, stride), np.uint8)
            ref = np.full((h, stride), 255, np.uint8)
        else:
            src = _fill(rnd, h * stride, rnd.rand8).astype(np.uint8).reshape(h, stride)
            ref = _fill(rnd, h * stride, rnd.rand8).astype(np.uint8).reshape(h, stride)
        second = _fill(rnd, w * h, rnd.rand8).astype(np.uint8).reshape(h, w)
        assert O.sad(src, stride, ref, stride, w, h) == ref_sad(src, ref, w, h)
        assert O.sad(src, stride, ref, stride, w, h, skip=True) == ref_sad(src, ref, w, h, True)
        assert O.sad(src, stride, ref, stride, w, h, second_pred=second) == \
            ref_sad_avg(src, ref, second, w, h)
        if trial == 0:
            assert O.sad(src, stride, ref, stride, w, h) == 255 * w * h
        for bd in (10, 12):
            mask = (1 << bd) - 1
            s16 = (_fill(rnd, h * stride, rnd.rand16) & mask).astype(np.uint16).reshape(h, stride)
            r16 = (_fill(rnd, h * stride, rnd.rand16) & mask).astype(np.uint16).reshape(h, stride)
            p16 = (_fill(rnd, w * h, rnd.rand16) & mask).astype(np.uint16).reshape(h, w)
            assert O.sad(s16, stride, r16, stride, w, h, highbd=True) == ref_sad(s16, r16, w, h)
            assert O.sad(s16, stride, r16, stride, w, h, highbd=True, skip=True) == \
                ref_sad(s16, r16, w, h, True)
            assert O.sad(s16, stride, r16, stride, w, h, highbd=True, second_pred=p16) == \
                ref_sad_avg(s16, r16, p16, w, h)


@pytest.mark.parametrize("w,h", SIZES)
def test_variance_vs_reference_checker(w, h):
    rnd = O.ACMRandom()
    for bd in (8, 10, 12):
        hb = bd > 8
        for _ in range(2):
            if hb:
                mask = (1 << bd) - 1
                src = (_fill(rnd, w * h, rnd.rand16) & mask).astype(np.uint16).reshape(h, w)
                ref = (_fill(rnd, w * h, rnd.rand16) & mask).astype(np.uint16).reshape(h, w)
            else:
                src = _fill(rnd, w * h, rnd.rand8).astype(np.uint8).reshape(h, w)
                ref = _fill(rnd, w * h, rnd.rand8).astype(np.uint8).reshape(h, w)
            v, s = O.variance(src, w, ref, w, w, h, bd, hb)
            rv, rs = ref_variance(src, ref, w, h, bd)
            assert (v, s) == (rv, rs)
        # OneQuarterTest (variance_test.cc:820-837)
        dt = np.uint16 if hb else np.uint8
        src = np.full((h, w), 255 << (bd - 8), dt)
        ref = np.zeros((h, w), dt)
        ref.reshape(-1)[:w * h // 2] = 255 << (bd - 8)
        v, _ = O.variance(src, w, ref, w, w, h, bd, hb)
        assert v == w * h * 255 * 255 // 4
        # ZeroTest (variance_test.cc:744-765): constant planes i, j << (bd-8)
        for i, j in ((0, 255), (7, 200), (255, 0), (128, 128)):
            src = np.full((h, w), i << (bd - 8), dt)
            ref = np.full((h, w), j << (bd - 8), dt)
            assert O.variance(src, w, ref, w, w, h, bd, hb)[0] == 0


@pytest.mark.parametrize("w,h", SIZES)
def test_subpel_variance_vs_reference_checker(w, h):
    rnd = O.ACMRandom()
    offs = [(x, y) for x in range(8) for y in range(8)]
    if w * h >= 64 * 64:
        offs = offs[::7]
    for bd in (8, 10, 12):
        hb = bd > 8
        mask = (1 << bd) - 1
        dt = np.uint16 if hb else np.uint8
        gen = (lambda: rnd.rand16() & mask) if hb else rnd.rand8
        for x, y in offs:
            ref = _fill(rnd, (h + 1) * (w + 1), gen).astype(dt).reshape(h + 1, w + 1)
            src = _fill(rnd, w * h, gen).astype(dt).reshape(h, w)
            sec = _fill(rnd, w * h, gen).astype(dt).reshape(h, w)
            got = O.sub_pixel_variance(ref, w + 1, x, y, src, w, w, h, bd, hb)
            assert got == ref_subpel_variance(ref, src, w, h, x, y, bd), (bd, x, y)
            got = O.sub_pixel_variance(ref, w + 1, x, y, src, w, w, h, bd, hb, second_pred=sec)
            assert got == ref_subpel_variance(ref, src, w, h, x, y, bd, sec), (bd, x, y)
        # ExtremeRefTest (variance_test.cc:1353-1384): half 0 / half max
        half = (h + 1) * (w + 1) // 2
        ref = np.zeros((h + 1) * (w + 1), dt)
        ref[half:] = mask
        ref = ref.reshape(h + 1, w + 1)
        src = np.zeros(w * h, dt)
        src[: w * h // 2] = mask
        src = src.reshape(h, w)
        for x, y in offs[::5]:
            got = O.sub_pixel_variance(ref, w + 1, x, y, src, w, w, h, bd, hb)
            assert got == ref_subpel_variance(ref, src, w, h, x, y, bd)


def test_mse_known_answers():
    """AvxMseTest MaxMse (variance_test.cc:1235-1243) and SumOfSquares
    ConstTest (:361-371)."""
    for w, h in ((16, 16), (16, 8), (8, 16), (8, 8)):
        src = np.full((h, w), 255, np.uint8)
        ref = np.zeros((h, w), np.uint8)
        assert O.mse(src, w, ref, w, w, h)[1] == w * h * 255 * 255
    for v in range(0, 256, 17):
        blk = np.full((16, 16), v, np.int16)
        assert O.sum_squares_2d_i16(blk, 16, 16, 16) == 256 * v * v


@pytest.mark.parametrize("n", [4, 8, 16, 32])
def test_hadamard_vs_reference_checker(n):
    """HadamardLowbdTest CompareReferenceRandom + VaryStride
    (hadamard_test.cc:246-282), Rand9Signed inputs."""
    rnd = O.ACMRandom()
    a = _fill(rnd, n * n, rnd.rand9signed).astype(np.int16).reshape(n, n)
    np.testing.assert_array_equal(O.hadamard(n, a, n), ref_hadamard(a, n))
    big = _fill(rnd, n * n * 8, rnd.rand9signed).astype(np.int16)
    for stride in range(8, 64, 8):
        if stride < n:
            continue
        blk = np.lib.stride_tricks.as_strided(big, (n, n), (stride * 2, 2))
        np.testing.assert_array_equal(O.hadamard(n, big, stride), ref_hadamard(blk, n))


@pytest.mark.parametrize("n", [8, 16, 32])
def test_highbd_hadamard_relations(n):
    """aom_highbd_hadamard_* (avg.c:350-507) equals the lowbd transform without
    the output transpose / AVX2 group swap when no int16 intermediate
    overflows (9-bit inputs); 13-bit inputs exercise the int32 second pass."""
    rnd = O.ACMRandom()
    a = _fill(rnd, n * n, rnd.rand9signed).astype(np.int16).reshape(n, n)
    hb = O.hadamard(n, a, n, highbd=True)
    if n == 8:
        np.testing.assert_array_equal(hb, ref_hadamard(a, 8).reshape(8, 8).T.reshape(-1))
    elif n == 16:
        sub = np.concatenate([ref_hadamard(a[r:r + 8, c:c + 8], 8).reshape(8, 8).T.reshape(-1)
                              for r in (0, 8) for c in (0, 8)])
        a0, a1, a2, a3 = sub[0:64], sub[64:128], sub[128:192], sub[192:256]
        b0, b1, b2, b3 = (a0 + a1) >> 1, (a0 - a1) >> 1, (a2 + a3) >> 1, (a2 - a3) >> 1
        np.testing.assert_array_equal(hb, np.concatenate([b0 + b2, b1 + b3, b0 - b2, b1 - b3]))
    a13 = (_fill(rnd, n * n, rnd.rand16) % 8191 - 4095).astype(np.int16).reshape(n, n)
    out = O.hadamard(n, a13, n, highbd=True)
    assert np.abs(out).max() > 32767 or n > 8  # int32 range is genuinely used


def test_block_error_known_answers():
    """av1_block_error semantics (rdopt.c:635-682): error = sum (c - dq)^2,
    ssz = sum c^2; highbd rounds by 2*(bd-8)."""
    rnd = O.ACMRandom()
    for n in (16, 64, 256, 1024):
        c = np.array([rnd.rand15signed() for _ in range(n)], np.int32)
        d = np.array([rnd.rand15signed() for _ in range(n)], np.int32)
        e, s = O.block_error(c, d, n)
        assert e == int(((c.astype(np.int64) - d) ** 2).sum())
        assert s == int((c.astype(np.int64) ** 2).sum())
        for bd in (8, 10, 12):
            e2, s2 = O.block_error(c, d, n, bd)
            sh = 2 * (bd - 8)
            r = (1 << (sh - 1)) if sh else 0
            assert e2 == (e + r) >> sh and s2 == (s + r) >> sh
