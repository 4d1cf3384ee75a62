"""GPU parity of the compound (CONV_BUF) convolutions:
  - lavish_dist_wtd_convolve_batch and the eight av1_*dist_wtd_convolve*_hip
    shims against av1_dist_wtd_convolve_{2d_copy,x,y,2d}_c and the highbd
    forms executed from the reference (tests/golden/fix_compound.npz), no
    oracle in the loop;
  - the batch API against the oracle restatement on large batches (every
    path, first pass / average / dist-wtd, bd 8/10/12, several block sizes)."""
import ctypes
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def Cm():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp.compound as Cm
    return Cm


def _table(interp_filter, size):
    return np.stack([O.interp_kernel(interp_filter, size, p) for p in range(16)])


def _row(F, r, J):
    g = lambda n: int(r[J[n]])
    cp = dict(round_0=g("round_0"), round_1=g("round_1"), do_average=int(g("mode") > 0),
              dist_wtd=int(g("mode") == 2), fwd=g("fwd_offset"), bck=g("bck_offset"))
    return g, cp


def _conv_params(Cm, cp, conv=None, stride=0):
    from lavish_dsp.inter import ConvolveParams
    d = conv.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)) if conv is not None else None
    return ConvolveParams(cp["do_average"], d, stride, cp["round_0"], cp["round_1"], 0, 1,
                          cp["dist_wtd"], cp["fwd"], cp["bck"])


def test_compound_batch_vs_reference(Cm):
    import torch
    F = dict(np.load(os.path.join(GOLD, "fix_compound.npz")))
    J = {n: i for i, n in enumerate(F["row_fields"])}
    SS, DS, CS, org = (int(v) for v in F["geom"])
    for k, r in enumerate(F["rows"]):
        g, cp = _row(F, r, J)
        bd, w, h = g("bd"), g("w"), g("h")
        hb = bd > 8
        pdt = np.uint16 if hb else np.uint8
        v = (lambda a: a.view(np.int16)) if hb else (lambda a: a)
        src = torch.from_numpy(v(np.ascontiguousarray(F["src"][g("src_index")].astype(pdt)))).cuda()
        dst = torch.from_numpy(v(F["dst_in"][k].astype(pdt).copy())).cuda()
        conv = torch.from_numpy(F["conv_in"][k].view(np.int16).copy()).cuda()
        fpx, tx = Cm.filter_params(_table(g("filter_x"), w))
        fpy, ty = Cm.filter_params(_table(g("filter_y"), h))
        job = np.zeros(1, Cm.JOB_DTYPE)
        job["src_off"] = org * SS + org
        job["subpel_x_qn"], job["subpel_y_qn"] = g("subpel_x"), g("subpel_y")
        Cm.dist_wtd_convolve_batch(src, SS, dst, DS, conv, CS, w, h,
                                   torch.from_numpy(job.view(np.uint8)).cuda(), 1, fpx, fpy,
                                   _conv_params(Cm, cp), bd)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(conv.cpu().numpy().view(np.uint16), F["conv"][k],
                                      err_msg="row %d conv" % k)
        np.testing.assert_array_equal(dst.cpu().numpy().view(pdt).astype(np.uint16), F["dst"][k],
                                      err_msg="row %d dst" % k)


def test_compound_shims_vs_reference(Cm):
    F = dict(np.load(os.path.join(GOLD, "fix_compound.npz")))
    J = {n: i for i, n in enumerate(F["row_fields"])}
    SS, DS, CS, org = (int(v) for v in F["geom"])
    for k, r in enumerate(F["rows"]):
        if k % 2:
            continue
        g, cp = _row(F, r, J)
        bd, w, h = g("bd"), g("w"), g("h")
        pdt = np.uint16 if bd > 8 else np.uint8
        src = np.ascontiguousarray(F["src"][g("src_index")].astype(pdt))
        dst = F["dst_in"][k].astype(pdt).copy()
        conv = F["conv_in"][k].copy()
        fpx, tx = Cm.filter_params(_table(g("filter_x"), w))
        fpy, ty = Cm.filter_params(_table(g("filter_y"), h))
        c = _conv_params(Cm, cp, conv, CS)
        addr = ctypes.c_void_p(src.ctypes.data + (org * SS + org) * src.itemsize)
        Cm.dist_wtd_convolve_shim(g("path"), addr, SS, dst, DS, w, h, fpx, fpy, g("subpel_x"),
                                  g("subpel_y"), c, bd)
        np.testing.assert_array_equal(conv, F["conv"][k], err_msg="row %d conv" % k)
        np.testing.assert_array_equal(dst.astype(np.uint16), F["dst"][k], err_msg="row %d" % k)


@pytest.mark.parametrize("bd", [8, 10, 12])
@pytest.mark.parametrize("w,h", [(4, 4), (8, 8), (16, 16), (32, 8), (64, 64), (128, 128)])
def test_compound_batch_vs_oracle(Cm, bd, w, h):
    import torch
    rng = np.random.default_rng(bd * 1000 + w * 10 + h)
    hb = bd > 8
    pdt = np.uint16 if hb else np.uint8
    W, H = 400, 300
    src = rng.integers(0, 1 << bd, (H, W)).astype(pdt)
    nj = 96 if w * h <= 1024 else 12
    jobs = np.zeros(nj, Cm.JOB_DTYPE)
    ys = rng.integers(8, H - h - 8, nj)
    xs = rng.integers(8, W - w - 8, nj)
    jobs["src_off"] = ys * W + xs
    jobs["dst_off"] = np.arange(nj) * w * h
    jobs["conv_off"] = np.arange(nj) * w * h
    jobs["subpel_x_qn"] = rng.integers(0, 16, nj) * (rng.integers(0, 4, nj) > 0)
    jobs["subpel_y_qn"] = rng.integers(0, 16, nj) * (rng.integers(0, 4, nj) > 0)
    fxi, fyi = int(rng.integers(0, 4)), int(rng.integers(0, 4))
    fpx, tx = Cm.filter_params(_table(fxi, w))
    fpy, ty = Cm.filter_params(_table(fyi, h))
    r0 = 3 + max(bd + 7 - 3 + 2 - 16, 0)
    conv0 = rng.integers(0, 1 << (bd + 4), (nj * h, w)).astype(np.uint16)
    dst0 = rng.integers(0, 1 << bd, (nj * h, w)).astype(pdt)
    for mode in range(3):
        cp = dict(round_0=r0, round_1=7, do_average=int(mode > 0), dist_wtd=int(mode == 2),
                  fwd=12 if mode == 2 else 0, bck=4 if mode == 2 else 0)
        t = lambda a: torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a.copy()).cuda()
        tsrc, tdst, tconv = t(src), t(dst0.copy()), t(conv0.copy())
        Cm.dist_wtd_convolve_batch(tsrc, W, tdst, w, tconv, w, w, h,
                                   torch.from_numpy(jobs.view(np.uint8)).cuda(), nj, fpx, fpy,
                                   _conv_params(Cm, cp), bd)
        torch.cuda.synchronize()
        gd = tdst.cpu().numpy().view(pdt)
        gc = tconv.cpu().numpy().view(np.uint16)
        ed, ec = dst0.copy(), conv0.copy()
        ocp = dict(do_average=cp["do_average"], round_0=r0, round_1=7, is_compound=1,
                   use_dist_wtd_comp_avg=cp["dist_wtd"], fwd_offset=cp["fwd"],
                   bck_offset=cp["bck"])
        for i in range(nj):
            sx, sy = int(jobs["subpel_x_qn"][i]), int(jobs["subpel_y_qn"][i])
            path = (sx != 0) + 2 * (sy != 0)
            O.dist_wtd_convolve(path, src, W, ed[i * h:(i + 1) * h], w, w, h, tx[sx], ty[sy],
                                ocp, ec[i * h:(i + 1) * h], w, bd, int(hb),
                                src_off=int(jobs["src_off"][i]))
        np.testing.assert_array_equal(gc, ec, err_msg="mode %d conv" % mode)
        np.testing.assert_array_equal(gd, ed, err_msg="mode %d dst" % mode)
