"""GPU parity of the pixel-domain kernels
against the oracle, bit-exact, through the C ABI:

* per-call RTCD shims (`aom_sad16x16_hip` ...), every @encoder_block_sizes
  entry, lowbd and highbd (tagged pointers), strided planes, extremes;
* the batch API (`lavish_sad_batch` ...) over many jobs at random positions
  of a synthetic 1080p-like plane."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

SIZES = [(128, 128), (128, 64), (64, 128), (64, 64), (64, 32), (32, 64), (32, 32), (32, 16),
         (16, 32), (16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4), (4, 16), (16, 4),
         (8, 32), (32, 8), (16, 64), (64, 16)]


@pytest.fixture(scope="module")
def P():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp.pixel as P
    return P


def _plane(rng, h, w, bd, fill=None):
    dt = np.uint16 if bd > 8 else np.uint8
    if fill == "max":
        return np.full((h, w), (1 << bd) - 1, dt)
    if fill == "zero":
        return np.zeros((h, w), dt)
    return rng.integers(0, 1 << bd, size=(h, w)).astype(dt)


@pytest.mark.parametrize("w,h", SIZES)
def test_sad_shims(P, w, h):
    rng = np.random.default_rng(w * 1000 + h)
    stride = w + 40
    for bd in (8, 10, 12):
        hb = bd > 8
        for fill in (None, "max"):
            src = _plane(rng, h + 8, stride, bd, "zero" if fill else None)
            refp = _plane(rng, h + 8, stride, bd, fill)
            second = _plane(rng, h, w, bd)
            refs = [refp[k:k + h, 3 * k:3 * k + w] for k in range(4)]
            s = src[:h, :w]
            for k in range(4):
                r = refs[k]
                assert P.sad(w, h, s, stride, r, stride, hb) == O.sad(s, stride, r, stride, w, h,
                                                                        hb)
                assert P.sad(w, h, s, stride, r, stride, hb, skip=True) == \
                    O.sad(s, stride, r, stride, w, h, hb, skip=True)
                assert P.sad(w, h, s, stride, r, stride, hb, second_pred=second) == \
                    O.sad(s, stride, r, stride, w, h, hb, second_pred=second)
            exp = [O.sad(s, stride, r, stride, w, h, hb) for r in refs]
            exp_skip = [O.sad(s, stride, r, stride, w, h, hb, skip=True) for r in refs]
            np.testing.assert_array_equal(P.sad_x4d(w, h, s, stride, refs, stride, hb), exp)
            np.testing.assert_array_equal(P.sad_x4d(w, h, s, stride, refs, stride, hb, "x3d"),
                                          exp)
            np.testing.assert_array_equal(
                P.sad_x4d(w, h, s, stride, refs, stride, hb, "skip_x4d"), exp_skip)
            if not hb:
                exp_avg = [O.sad(s, stride, r, stride, w, h, second_pred=second) for r in refs]
                np.testing.assert_array_equal(
                    P.sad_x4d(w, h, s, stride, refs, stride, False, "x4d_avg", second), exp_avg)


@pytest.mark.parametrize("w,h", SIZES)
def test_variance_shims(P, w, h):
    rng = np.random.default_rng(7 * w + h)
    stride = w + 24
    for bd in (8, 10, 12):
        hb = bd > 8
        for fill in (None, "max"):
            a = _plane(rng, h + 2, stride, bd, "zero" if fill else None)
            b = _plane(rng, h + 2, stride, bd, fill)
            sec = _plane(rng, h, w, bd)
            va = a[:h, :w]
            vb = b[1:h + 1, 2:w + 2]
            assert P.variance(w, h, va, stride, vb, stride, bd, hb) == \
                O.variance(va, stride, vb, stride, w, h, bd, hb)
            offs = [(0, 0), (4, 0), (0, 4), (7, 7), (3, 5)] if fill is None else [(2, 6)]
            for xo, yo in offs:
                assert P.sub_pixel_variance(w, h, va, stride, xo, yo, vb, stride, bd, hb) == \
                    O.sub_pixel_variance(va, stride, xo, yo, vb, stride, w, h, bd, hb), (bd, xo, yo)
                assert P.sub_pixel_variance(w, h, va, stride, xo, yo, vb, stride, bd, hb, sec) == \
                    O.sub_pixel_variance(va, stride, xo, yo, vb, stride, w, h, bd, hb, sec)


def test_mse_getvar_shims(P):
    rng = np.random.default_rng(3)
    for bd in (8, 10, 12):
        hb = bd > 8
        for fill in (None, "max"):
            a = _plane(rng, 40, 48, bd, "zero" if fill else None)
            b = _plane(rng, 40, 48, bd, fill)
            for w, h in ((16, 16), (16, 8), (8, 16), (8, 8)):
                assert P.mse(w, h, a, 48, b, 48, bd, hb) == O.mse(a, 48, b, 48, w, h, bd, hb)
            for n in (8, 16):
                assert P.get_var(n, a, 48, b, 48, bd, hb) == \
                    O.get_var(a, 48, b, 48, n, n, bd, hb)


def test_sse_subtract_sumsq_shims(P):
    rng = np.random.default_rng(11)
    for w, h in ((4, 4), (8, 8), (16, 16), (64, 64), (128, 128), (36, 20), (1920, 8)):
        stride = w + 16
        for bd in (8, 10, 12):
            hb = bd > 8
            a = _plane(rng, h, stride, bd)
            b = _plane(rng, h, stride, bd)
            assert P.sse(a, stride, b, stride, w, h, hb) == O.sse(a, stride, b, stride, w, h, hb)
            d1 = np.full((h, stride), 77, np.int16)
            d2 = d1.copy()
            P.subtract_block(h, w, d1, stride, a, stride, b, stride, hb)
            O.subtract_block(h, w, d2, stride, a, stride, b, stride, hb)
            np.testing.assert_array_equal(d1, d2)
        res = rng.integers(-4095, 4096, size=(h, stride)).astype(np.int16)
        assert P.sum_squares_2d_i16(res, stride, w, h) == O.sum_squares_2d_i16(res, stride, w, h)


@pytest.mark.parametrize("n", [4, 8, 16, 32])
def test_hadamard_satd_shims(P, n):
    rng = np.random.default_rng(n)
    for stride in (n, n + 8, 64):
        for lim in (255, 256):
            a = rng.integers(-lim, lim + 1, size=(n, stride)).astype(np.int16)
            got = P.hadamard(n, a, stride)
            np.testing.assert_array_equal(got, O.hadamard(n, a, stride))
            assert P.satd(got, n * n) == O.satd(got, n * n)
        if n >= 8:
            a = rng.integers(-4095, 4096, size=(n, stride)).astype(np.int16)
            np.testing.assert_array_equal(P.hadamard(n, a, stride, highbd=True),
                                          O.hadamard(n, a, stride, highbd=True))


def test_block_error_shims(P):
    rng = np.random.default_rng(5)
    for n in (16, 64, 256, 1024):
        for lim in (1 << 15, 1 << 19):
            c = rng.integers(-lim, lim, size=n).astype(np.int32)
            d = (c + rng.integers(-300, 300, size=n)).astype(np.int32)
            if lim == 1 << 15:
                assert P.block_error(c, d, n) == O.block_error(c, d, n)
            for bd in (8, 10, 12):
                assert P.block_error(c, d, n, bd) == O.block_error(c, d, n, bd)


# ---------------------------------------------------------------- batch --
def _jobs(P, rng, njobs, W, H, w, h, nrefs=1, sub=False, aux_stride=0):
    j = np.zeros(njobs, P.JOB_DTYPE)
    mx, my = W - w - (1 if sub else 0), H - h - (1 if sub else 0)
    j["src_off"] = rng.integers(0, my, njobs) * W + rng.integers(0, mx, njobs)
    for k in range(nrefs):
        j["ref_off"][:, k] = rng.integers(0, my, njobs) * W + rng.integers(0, mx, njobs)
    j["aux_off"] = np.arange(njobs) * aux_stride
    j["xoff"] = rng.integers(0, 8, njobs)
    j["yoff"] = rng.integers(0, 8, njobs)
    return j


@pytest.mark.parametrize("bd", [8, 10])
def test_sad_variance_batch(P, bd):
    import torch
    rng = np.random.default_rng(bd)
    W, H = 640, 360
    hb = bd > 8
    src = _plane(rng, H, W, bd)
    ref = _plane(rng, H, W, bd)
    tdt = torch.int16 if hb else torch.uint8
    view = (lambda a: a.view(np.int16)) if hb else (lambda a: a)
    ts = torch.from_numpy(view(src)).cuda()
    tr = torch.from_numpy(view(ref)).cuda()
    assert ts.dtype == tdt
    for w, h in ((16, 16), (8, 8), (32, 32), (64, 64), (4, 16), (128, 128)):
        nj = 300
        jobs = _jobs(P, rng, nj, W, H, w, h, nrefs=4, sub=True, aux_stride=w * h)
        tj = P.jobs_tensor(jobs, "cuda")
        second = _plane(rng, nj * h, w, bd)
        tsec = torch.from_numpy(view(second)).cuda()
        got = P.sad_batch(ts, tr, w, h, tj, nrefs=4).cpu().numpy()
        got_skip = P.sad_batch(ts, tr, w, h, tj, nrefs=4, mode=1).cpu().numpy()
        got_avg = P.sad_batch(ts, tr, w, h, tj, nrefs=1, mode=2, second_pred=tsec).cpu().numpy()
        vb = P.variance_batch(ts, tr, w, h, tj, kind=0, bit_depth=bd)
        sb = P.variance_batch(ts, tr, w, h, tj, kind=3, bit_depth=bd)
        ab = P.variance_batch(ts, tr, w, h, tj, kind=5, bit_depth=bd, second_pred=tsec)
        e64 = P.variance_batch(ts, tr, w, h, tj, kind=4, bit_depth=bd)["sse64"].cpu().numpy()
        vb = {k: v.cpu().numpy() for k, v in vb.items()}
        sb = {k: v.cpu().numpy() for k, v in sb.items()}
        ab = {k: v.cpu().numpy() for k, v in ab.items()}
        fs, fr = src.reshape(-1), ref.reshape(-1)
        for i in range(0, nj, 7):
            so = int(jobs["src_off"][i])
            sv = fs[so:].reshape(-1)
            s2 = np.lib.stride_tricks.as_strided(sv, (h + 1, w + 1), (W * sv.itemsize,
                                                                      sv.itemsize))
            sec_i = second[i * h:(i + 1) * h]
            for k in range(4):
                ro = int(jobs["ref_off"][i, k])
                rv = fr[ro:]
                r2 = np.lib.stride_tricks.as_strided(rv, (h + 1, w + 1), (W * rv.itemsize,
                                                                          rv.itemsize))
                assert got[i, k] == O.sad(s2, W, r2, W, w, h, hb)
                assert got_skip[i, k] == O.sad(s2, W, r2, W, w, h, hb, skip=True)
                if k == 0:
                    assert got_avg[i, 0] == O.sad(s2, W, r2, W, w, h, hb, second_pred=sec_i)
                    v, s = O.variance(s2, W, r2, W, w, h, bd, hb)
                    assert (vb["var"][i], vb["sse"][i]) == (v, s)
                    xo, yo = int(jobs["xoff"][i]), int(jobs["yoff"][i])
                    v, s = O.sub_pixel_variance(s2, W, xo, yo, r2, W, w, h, bd, hb)
                    assert (sb["var"][i], sb["sse"][i]) == (v, s)
                    v, s = O.sub_pixel_variance(s2, W, xo, yo, r2, W, w, h, bd, hb, sec_i)
                    assert (ab["var"][i], ab["sse"][i]) == (v, s)
                    assert e64[i] == O.sse(s2, W, r2, W, w, h, hb)


def test_residual_batches(P):
    """subtract -> hadamard -> satd, sum_squares and block_error batches."""
    import torch
    rng = np.random.default_rng(99)
    W, H = 256, 128
    src = _plane(rng, H, W, 8)
    pred = _plane(rng, H, W, 8)
    ts, tp = torch.from_numpy(src).cuda(), torch.from_numpy(pred).cuda()
    n = 16
    bw, bh = W // n, H // n
    jobs = np.zeros(bw * bh, P.JOB_DTYPE)
    for by in range(bh):
        for bx in range(bw):
            j = by * bw + bx
            jobs["src_off"][j] = by * n * W + bx * n
            jobs["ref_off"][j, 0] = by * n * W + bx * n
            jobs["aux_off"][j] = by * n * W + bx * n
    tj = P.jobs_tensor(jobs, "cuda")
    diff = torch.zeros((H, W), dtype=torch.int16, device="cuda")
    P.subtract_batch(n, n, diff, ts, tp, tj)
    d_ref = np.zeros((H, W), np.int16)
    O.subtract_block(H, W, d_ref, W, src, W, pred, W)
    np.testing.assert_array_equal(diff.cpu().numpy(), d_ref)

    hj = jobs.copy()
    hj["src_off"] = jobs["aux_off"]
    hj["aux_off"] = np.arange(len(jobs)) * n * n
    thj = P.jobs_tensor(hj, "cuda")
    for nn in (4, 8, 16):
        coeff = P.hadamard_batch(nn, diff, thj, len(jobs) * n * n)
        c = coeff.cpu().numpy().reshape(len(jobs), n * n)
        for j in range(0, len(jobs), 5):
            so = int(hj["src_off"][j])
            blk = d_ref.reshape(-1)[so:]
            np.testing.assert_array_equal(c[j, :nn * nn], O.hadamard(nn, blk, W))
        sat = P.satd_batch(coeff.view(len(jobs), n * n)[:, :nn * nn].contiguous()).cpu().numpy()
        for j in range(len(jobs)):
            assert sat[j] == O.satd(np.ascontiguousarray(c[j, :nn * nn]), nn * nn)
    ss = P.sum_squares_batch(diff, n, n, thj).cpu().numpy()
    for j in range(len(jobs)):
        so = int(hj["src_off"][j])
        assert ss[j] == O.sum_squares_2d_i16(d_ref.reshape(-1)[so:], W, n, n)

    cf = rng.integers(-(1 << 15), 1 << 15, size=(64, 256)).astype(np.int32)
    dq = (cf + rng.integers(-64, 64, size=cf.shape)).astype(np.int32)
    for bd in (0, 8, 10, 12):
        e, z = P.block_error_batch(torch.from_numpy(cf).cuda(), torch.from_numpy(dq).cuda(), bd)
        e, z = e.cpu().numpy(), z.cpu().numpy()
        for j in range(64):
            assert (e[j], z[j]) == O.block_error(cf[j], dq[j], 256, None if bd == 0 else bd)
