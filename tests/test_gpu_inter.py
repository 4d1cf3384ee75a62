"""GPU parity of single-reference inter prediction (lavish_build_inter_pred_batch,
av1_enc_build_one_inter_predictor) and the per-call convolve shims
(av1_convolve_{x,y,2d}_sr_hip, highbd forms, aom_convolve_copy_hip) against the
oracle's restatement (oracle/oracle_convolve.c): every output pixel
bit-exact, for every block size, filter pair, phase, bit depth and
subsampling, with mvs that reach the border clamp."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


def _bordered(W, H, ss, dt, bd, seed):
    # the reference's frame buffers: AOM_BORDER_IN_PIXELS >> ss on each side,
    # per direction -- the border clamp keeps every read inside it
    # (12-tap kernels at the clamp extremes read one row / column beyond it,
    # as the C does: two spare rows / columns each side)
    rng = np.random.default_rng(seed)
    bx, by = (288 >> ss[0]) + 2, (288 >> ss[1]) + 2
    stride = W + 2 * bx + 24
    plane = rng.integers(0, 1 << bd, size=(H + 2 * by, stride)).astype(dt)
    return plane, by * stride + bx


def _jobs(W, H, bw, bh, seed, filters=None, far=0.05):
    import lavish_dsp.inter as I
    rng = np.random.default_rng(seed)
    n = (W // bw) * (H // bh)
    mvs = rng.integers(-300, 300, size=(n, 2))
    big = rng.random(n) < far
    mvs[big] = rng.integers(-16000, 16000, size=(int(big.sum()), 2))
    if filters is None:
        filters = rng.integers(0, 5, size=(n, 2))
    return I.plane_jobs(W, H, bw, bh, mvs, filters)


def _run(W, H, bw, bh, bd=8, hbd=False, ss=(0, 0), seed=0, filters=None, mvs=None):
    import torch
    import lavish_dsp.inter as I
    import lavish_dsp.motion as M
    dt = np.uint16 if hbd else np.uint8
    plane, org = _bordered(W, H, ss, dt, bd, seed)
    jobs = _jobs(W, H, bw, bh, seed + 1, filters)
    tref = torch.from_numpy(plane.view(np.int16) if hbd else plane).cuda()
    dmvs = None
    if mvs is not None:
        dmvs = M.to_device(mvs)
    got = I.build_inter_pred_batch(tref, org, W, H, bw, bh, M.to_device(jobs), bit_depth=bd,
                                   ss=ss, mvs=dmvs)
    torch.cuda.synchronize()
    got = got.cpu().numpy().view(np.uint16) if hbd else got.cpu().numpy()
    exp = O.build_inter_pred(plane, org, W, H, ss[0], ss[1], bw, bh, jobs, (H, W), bd=bd,
                             mvs=mvs)
    np.testing.assert_array_equal(got, exp)
    return jobs


SIZES = [(4, 4), (8, 8), (16, 16), (32, 32), (64, 64), (128, 128), (4, 8), (8, 4), (16, 8),
         (8, 32), (64, 16), (4, 16), (16, 4), (32, 8), (2, 2), (2, 4), (4, 2), (2, 8)]


@pytest.mark.parametrize("bw,bh", SIZES)
def test_inter_pred_sizes_lowbd(bw, bh):
    _run(128, 128, bw, bh, seed=bw * 131 + bh)


@pytest.mark.parametrize("bd", [8, 10, 12])
@pytest.mark.parametrize("bw,bh", [(4, 4), (16, 16), (8, 32), (64, 64), (2, 4)])
def test_inter_pred_highbd(bd, bw, bh):
    _run(128, 64, bw, bh, bd=bd, hbd=True, seed=bd * 7 + bw)


@pytest.mark.parametrize("ss", [(1, 1), (1, 0), (0, 1)])
@pytest.mark.parametrize("hbd", [False, True])
def test_inter_pred_subsampled(ss, hbd):
    _run(96, 64, 8, 8, bd=10 if hbd else 8, hbd=hbd, ss=ss, seed=5)
    _run(96, 64, 2, 4, bd=10 if hbd else 8, hbd=hbd, ss=ss, seed=6)


@pytest.mark.parametrize("fx", range(5))
@pytest.mark.parametrize("fy", range(5))
def test_inter_pred_filter_pairs(fx, fy):
    _run(64, 64, 16, 16, seed=fx * 5 + fy, filters=(fx, fy))


def test_inter_pred_ragged_plane():
    # width / height not multiples of the block: only full blocks are jobs
    _run(100, 70, 16, 16, seed=9)


def test_inter_pred_after_subpel():
    import lavish_dsp.motion as M
    rng = np.random.default_rng(12)
    n = (64 // 16) * (64 // 16)
    mvs = np.zeros(n, M.SUBPEL_RESULT_DTYPE)
    mvs["best_row"] = rng.integers(-200, 200, n)
    mvs["best_col"] = rng.integers(-200, 200, n)
    _run(64, 64, 16, 16, seed=12, mvs=mvs)


def test_inter_pred_rejects():
    import torch
    import lavish_dsp.inter as I
    import lavish_dsp.motion as M
    plane = torch.zeros((64, 64), dtype=torch.uint8, device="cuda")
    jobs = M.to_device(I.plane_jobs(16, 16, 8, 8, (0, 0)))
    for kw in (dict(w=3, h=8), dict(w=8, h=256), dict(w=8, h=8, bit_depth=10),
               dict(w=8, h=8, ss=(2, 0))):
        w, h = kw.pop("w"), kw.pop("h")
        with pytest.raises(ValueError):
            I.build_inter_pred_batch(plane, 0, 16, 16, w, h, jobs, **kw)
    # an empty job list is a no-op
    out = torch.full((16, 16), 7, dtype=torch.uint8, device="cuda")
    I.build_inter_pred_batch(plane, 0, 16, 16, 8, 8, jobs[:0], dst=out)
    assert (out == 7).all()


# ---------------------------------------------------------------- RTCD shims --
def _shim_case(kind, dt, bd, w, h, f, seed, r0=None, r1=None):
    import lavish_dsp.inter as I
    rng = np.random.default_rng(seed)
    S = 160
    plane = rng.integers(0, 1 << bd, size=(S, S)).astype(dt)
    off = 12 * S + 12
    sx, sy = int(rng.integers(0, 16)), int(rng.integers(0, 16))
    taps = 12 if f == 4 else 8
    tabx = np.stack([O.interp_kernel(f, w, p) for p in range(16)])
    taby = np.stack([O.interp_kernel(f, h, p) for p in range(16)])
    fpx, fpy = I.filter_params(tabx, taps, f), I.filter_params(taby, taps, f)
    dr0, dr1 = O.conv_rounds(bd)
    r0 = dr0 if r0 is None else r0
    r1 = dr1 if r1 is None else r1
    path = {"copy": 0, "x": 1, "y": 2, "2d": 3}[kind]
    dst = np.zeros((h, w + 5), dt)
    I.convolve(kind, plane, off, S, dst, 0, w + 5, w, h, fpx, fpy, sx, sy, r0, r1, bd)
    exp = O.convolve_block(plane, off, S, w, h, path, tabx[sx], taby[sy], r0, r1, bd)
    np.testing.assert_array_equal(dst[:, :w], exp)
    assert (dst[:, w:] == 0).all()


@pytest.mark.parametrize("kind", ["2d", "x", "y", "copy"])
@pytest.mark.parametrize("bd,dt", [(8, np.uint8), (10, np.uint16), (12, np.uint16)])
@pytest.mark.parametrize("w,h", [(4, 4), (16, 8), (2, 2), (128, 128)])
def test_convolve_shims(kind, bd, dt, w, h):
    for f in range(5):
        _shim_case(kind, dt, bd, w, h, f, seed=f + w + h + bd)


def test_convolve_shim_compound_rounding():
    # the 2-D function with the compound round_1 (COMPOUND_ROUND1_BITS = 7)
    _shim_case("2d", np.uint8, 8, 16, 16, 0, seed=3, r0=3, r1=7)
