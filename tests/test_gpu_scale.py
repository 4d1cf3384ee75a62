"""GPU parity of the scaled convolution:
  - lavish_convolve_2d_scale_batch and the av1_convolve_2d_scale_hip /
    av1_highbd_convolve_2d_scale_hip shims against av1_convolve_2d_scale_c /
    av1_highbd_convolve_2d_scale_c executed from the reference
    (tests/golden/fix_scale.npz: steps 512 .. 2048, every start phase form,
    the five filters incl. 12-tap, bd 8 both forms / 10 / 12, single
    prediction, compound first pass, plain and distance-weighted average),
    no oracle in the loop;
  - the batch API against the oracle restatement (orc_convolve_2d_scale) on
    large random batches: every block size 2x2 .. 128x128 class, steps drawn
    over [1, 2048] and the limits, the four conv-param forms;
  - the out-of-range steps: a block is left untouched."""
import ctypes
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIELDS = ("subpel_x_qn", "x_step_qn", "subpel_y_qn", "y_step_qn")


@pytest.fixture(scope="module")
def S():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp.scale as S
    return S


def _fp(table):
    from lavish_dsp.compound import filter_params
    return filter_params(table)


def _row(F, k):
    J = {n: i for i, n in enumerate(F["row_fields"])}
    r = F["rows"][k]
    g = lambda n: int(r[J[n]])
    m = g("mode")
    cp = dict(do_average=int(m > 1), round_0=g("round_0"), round_1=g("round_1"),
              is_compound=int(m > 0), use_dist_wtd_comp_avg=int(m == 3),
              fwd_offset=g("fwd_offset"), bck_offset=g("bck_offset"))
    return g, cp


def _cparams(cp, conv=None, stride=0):
    from lavish_dsp.inter import ConvolveParams
    d = conv.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)) if conv is not None else None
    return ConvolveParams(cp["do_average"], d, stride, cp["round_0"], cp["round_1"], 0,
                          cp["is_compound"], cp["use_dist_wtd_comp_avg"], cp["fwd_offset"],
                          cp["bck_offset"])


def test_scale_batch_vs_reference(S):
    import torch
    F = dict(np.load(os.path.join(GOLD, "fix_scale.npz")))
    SW, DS, CS, org = (int(v) for v in F["geom"])
    for k in range(len(F["rows"])):
        g, cp = _row(F, k)
        hb, bd, w, h = g("highbd"), g("bd"), g("w"), g("h")
        pdt = np.uint16 if hb else np.uint8
        v = (lambda a: a.view(np.int16)) if hb else (lambda a: a)
        src = torch.from_numpy(v(np.ascontiguousarray(F["src"][g("src_index")].astype(pdt)))).cuda()
        dst = torch.from_numpy(v(F["dst_in"][k].astype(pdt).copy())).cuda()
        conv = torch.from_numpy(F["conv_in"][k].view(np.int16).copy()).cuda()
        fpx, _ = _fp(O.interp_table(g("filter_x"), w))
        fpy, _ = _fp(O.interp_table(g("filter_y"), h))
        assert fpx.taps == g("taps_x") and fpy.taps == g("taps_y")
        job = np.zeros(1, S.JOB_DTYPE)
        job["src_off"] = org
        for f in FIELDS:
            job[f] = g(f)
        S.convolve_2d_scale_batch(src, SW, dst, DS, conv, CS, w, h,
                                  torch.from_numpy(job.view(np.uint8)).cuda(), 1, fpx, fpy,
                                  _cparams(cp), bd)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(conv.cpu().numpy().view(np.uint16), F["conv"][k],
                                      err_msg="row %d conv" % k)
        np.testing.assert_array_equal(dst.cpu().numpy().view(pdt).astype(np.uint16), F["dst"][k],
                                      err_msg="row %d dst" % k)


def test_scale_shims_vs_reference(S):
    F = dict(np.load(os.path.join(GOLD, "fix_scale.npz")))
    SW, DS, CS, org = (int(v) for v in F["geom"])
    for k in range(0, len(F["rows"]), 3):
        g, cp = _row(F, k)
        hb, bd, w, h = g("highbd"), g("bd"), g("w"), g("h")
        pdt = np.uint16 if hb else np.uint8
        src = np.ascontiguousarray(F["src"][g("src_index")].astype(pdt))
        dst = F["dst_in"][k].astype(pdt).copy()
        conv = F["conv_in"][k].copy()
        fpx, _ = _fp(O.interp_table(g("filter_x"), w))
        fpy, _ = _fp(O.interp_table(g("filter_y"), h))
        c = _cparams(cp, conv, CS)
        addr = ctypes.c_void_p(src.ctypes.data + org * src.itemsize)
        S.convolve_2d_scale_shim(addr, SW, dst, DS, w, h, fpx, fpy, *(g(f) for f in FIELDS), c,
                                 bd)
        np.testing.assert_array_equal(conv, F["conv"][k], err_msg="row %d conv" % k)
        np.testing.assert_array_equal(dst.astype(np.uint16), F["dst"][k], err_msg="row %d" % k)


def _random_batch(S, rng, w, h, nj, W, H, steps=None):
    jobs = np.zeros(nj, S.JOB_DTYPE)
    if steps is None:
        steps = np.where(rng.integers(0, 4, (nj, 2)) == 0,
                         rng.choice([1, 64, 1024, 2048], (nj, 2)),
                         rng.integers(1, 2049, (nj, 2)))
    jobs["x_step_qn"], jobs["y_step_qn"] = steps[:, 0], steps[:, 1]
    jobs["subpel_x_qn"] = rng.integers(0, 1024, nj)
    jobs["subpel_y_qn"] = rng.integers(0, 1024, nj)
    ex = ((w - 1) * 2048 + 1023 >> 10) + 12
    ey = ((h - 1) * 2048 + 1023 >> 10) + 12
    ys = rng.integers(6, H - ey, nj)
    xs = rng.integers(6, W - ex, nj)
    jobs["src_off"] = ys * W + xs
    jobs["dst_off"] = np.arange(nj) * w * h
    jobs["conv_off"] = np.arange(nj) * w * h
    return jobs


@pytest.mark.parametrize("bd,hb", [(8, 0), (8, 1), (10, 1), (12, 1)])
@pytest.mark.parametrize("w,h", [(2, 2), (4, 4), (8, 8), (16, 8), (32, 32), (64, 128),
                                 (128, 128)])
def test_scale_batch_vs_oracle(S, bd, hb, w, h):
    import torch
    rng = np.random.default_rng(bd * 1000 + hb * 500 + w * 10 + h)
    pdt = np.uint16 if hb else np.uint8
    W, H = 2 * w + 48, 2 * h + 48
    src = rng.integers(0, 1 << bd, (H, W)).astype(pdt)
    nj = 64 if w * h <= 1024 else 8
    jobs = _random_batch(S, rng, w, h, nj, W, H)
    fxi, fyi = int(rng.integers(0, 5)), int(rng.integers(0, 5))
    fx, fy = O.interp_table(fxi, w), O.interp_table(fyi, h)
    fpx, _ = _fp(fx)
    fpy, _ = _fp(fy)
    intbuf = bd + 7 - 3 + 2
    r0 = 3 + max(intbuf - 16, 0)
    conv0 = rng.integers(0, 1 << (bd + 4), (nj * h, w)).astype(np.uint16)
    dst0 = rng.integers(0, 1 << bd, (nj * h, w)).astype(pdt)
    t = lambda a: torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a.copy()).cuda()
    tjobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
    for mode in range(4):
        comp = int(mode > 0)
        cp = dict(do_average=int(mode > 1), round_0=r0,
                  round_1=7 if comp else 2 * 7 - r0, is_compound=comp,
                  use_dist_wtd_comp_avg=int(mode == 3), fwd_offset=9 if mode == 3 else 0,
                  bck_offset=7 if mode == 3 else 0)
        tsrc, tdst, tconv = t(src), t(dst0.copy()), t(conv0.copy())
        S.convolve_2d_scale_batch(tsrc, W, tdst, w, tconv, w, w, h, tjobs, nj, fpx, fpy,
                                  _cparams(cp), bd)
        torch.cuda.synchronize()
        gd = tdst.cpu().numpy().view(pdt)
        gc = tconv.cpu().numpy().view(np.uint16)
        ed, ec = dst0.copy(), conv0.copy()
        for i in range(nj):
            O.convolve_2d_scale(src, W, ed[i * h:(i + 1) * h], w, w, h, fx, fy,
                                *(int(jobs[f][i]) for f in FIELDS), cp,
                                ec[i * h:(i + 1) * h], w, bd, hb,
                                src_off=int(jobs["src_off"][i]))
        np.testing.assert_array_equal(gc, ec, err_msg="mode %d conv" % mode)
        np.testing.assert_array_equal(gd, ed, err_msg="mode %d dst" % mode)


def test_scale_out_of_range_steps_untouched(S):
    """Steps outside [1, 2048] or phases outside [0, 1023]: the block's
    outputs are left as they were; the in-range blocks of the same batch are
    computed."""
    import torch
    rng = np.random.default_rng(77)
    w = h = 16
    W, H = 2 * w + 48, 2 * h + 48
    src = rng.integers(0, 256, (H, W)).astype(np.uint8)
    jobs = _random_batch(S, rng, w, h, 6, W, H, steps=np.full((6, 2), 1024))
    jobs["x_step_qn"][1] = 2049
    jobs["y_step_qn"][2] = 0
    jobs["subpel_x_qn"][3] = 1024
    jobs["subpel_y_qn"][4] = -1
    fx = O.interp_table(0, w)
    fpx, _ = _fp(fx)
    cp = dict(do_average=0, round_0=3, round_1=11, is_compound=0, use_dist_wtd_comp_avg=0,
              fwd_offset=0, bck_offset=0)
    dst = torch.full((6 * h, w), 0x5a, dtype=torch.uint8, device="cuda")
    S.convolve_2d_scale_batch(torch.from_numpy(src).cuda(), W, dst, w, None, 0, w, h,
                              torch.from_numpy(jobs.view(np.uint8)).cuda(), 6, fpx, fpx,
                              _cparams(cp), 8)
    torch.cuda.synchronize()
    got = dst.cpu().numpy()
    for i in (1, 2, 3, 4):
        assert (got[i * h:(i + 1) * h] == 0x5a).all(), i
    for i in (0, 5):
        e = np.zeros((h, w), np.uint8)
        O.convolve_2d_scale(src, W, e, w, w, h, fx, fx, *(int(jobs[f][i]) for f in FIELDS), cp,
                            np.zeros((h, w), np.uint16), w, 8, 0, src_off=int(jobs["src_off"][i]))
        np.testing.assert_array_equal(got[i * h:(i + 1) * h], e, err_msg=str(i))


def test_scale_rejects(S):
    import torch
    src = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    jobs = torch.zeros(S.JOB_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    fx = O.interp_table(0, 8)
    fpx, _ = _fp(fx)
    cp = _cparams(dict(do_average=0, round_0=3, round_1=11, is_compound=0,
                       use_dist_wtd_comp_avg=0, fwd_offset=0, bck_offset=0))
    for w, h in ((3, 8), (256, 8), (8, 0), (8, 129)):
        with pytest.raises(ValueError):
            S.convolve_2d_scale_batch(src, 64, src, 8, None, 0, w, h, jobs, 1, fpx, fpx, cp, 8)
    with pytest.raises(ValueError):  # lowbd at bd 10
        S.convolve_2d_scale_batch(src, 64, src, 8, None, 0, 8, 8, jobs, 1, fpx, fpx, cp, 10)


def _bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_scale_bench_workload_vs_oracle(S):
    """bench.py --workload scale's call (every 16x16 block x 7 references at
    1.5x resolution, EIGHTTAP_REGULAR, single prediction, 8-bit) on a
    1920x256 strip of the same construction, against the oracle's batch
    restatement (orc_convolve_2d_scale_batch, pinned by fix_scale)."""
    import torch
    from lavish_dsp.compound import filter_params
    b = _bench()
    W, H, R = 1920, 256, 7
    refs, st, jobs = b.scale_setup(W, H, R, 99)
    tab = b.compound_tables()
    fp, keep = filter_params(tab)
    pred = torch.full((R * W * H,), 7, dtype=torch.uint8, device="cuda")
    S.convolve_2d_scale_batch(torch.from_numpy(refs.reshape(-1)).cuda(), st, pred, W, None, 0,
                              16, 16, torch.from_numpy(jobs.view(np.uint8)).cuda(), len(jobs),
                              fp, fp, _cparams(b.SCALE_CP), 8)
    torch.cuda.synchronize()
    exp = np.full(R * W * H, 7, np.uint8)
    O.convolve_2d_scale_batch(refs.reshape(-1), st, exp, W, None, 0, 16, 16, jobs, tab, tab,
                              b.SCALE_CP, threads=8)
    np.testing.assert_array_equal(pred.cpu().numpy(), exp)
    assert (exp != 7).mean() > 0.9
