"""GPU parity of the affine warp predictor:
  - lavish_warp_affine_batch and the av1_warp_affine_hip /
    av1_highbd_warp_affine_hip shims against av1_warp_affine_c /
    av1_highbd_warp_affine_c executed from the reference
    (tests/golden/fix_warp.npz): prediction and compound buffer of every row,
    no oracle in the loop;
  - the batch API against the oracle restatement on large batches (many
    blocks, stacked references, cropped shapes, every conv form, bd 8/10/12,
    subsampling)."""
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def Wp():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp.warp as Wp
    return Wp


def _case(F, r, J):
    g = lambda k: int(r[J[k]])
    W, H, RS, PS, DS = (int(v) for v in F["geom"])
    bd = g("bd")
    mode = g("mode")
    cp = dict(round_0=g("round_0"), round_1=g("round_1"), is_compound=int(mode > 0),
              do_average=int(mode >= 2), dist_wtd=int(mode == 3), fwd_offset=g("fwd_offset"),
              bck_offset=g("bck_offset"))
    return g, W, H, RS, PS, DS, bd, cp


def test_warp_batch_vs_reference(Wp):
    import torch
    F = dict(np.load(os.path.join(GOLD, "fix_warp.npz")))
    J = {n: i for i, n in enumerate(F["row_fields"])}
    for k, r in enumerate(F["rows"]):
        g, W, H, RS, PS, DS, bd, cp = _case(F, r, J)
        hb = bd > 8
        pdt = np.uint16 if hb else np.uint8
        ref = torch.from_numpy(F["refs"][g("ref_index")].astype(pdt).view(np.int16) if hb else
                               F["refs"][g("ref_index")].astype(pdt)).cuda()
        pin = F["pred_in"][k].astype(pdt)
        pred = torch.from_numpy(pin.view(np.int16) if hb else pin.copy()).cuda()
        dst = torch.from_numpy(F["dst_in"][k].view(np.int16).copy()).cuda()
        job = np.zeros(1, Wp.JOB_DTYPE)
        job["mat"] = [g("m%d" % i) for i in range(6)]
        for f in ("alpha", "beta", "gamma", "delta", "p_col", "p_row", "p_width", "p_height"):
            job[f] = g(f)
        tj = torch.from_numpy(job.view(np.uint8)).cuda()
        Wp.warp_affine_batch(ref, W, H, RS, pred, PS, tj, 1, Wp.conv_params(**cp), bd,
                             conv_dst=dst, dst_stride=DS, subsampling_x=g("ss_x"),
                             subsampling_y=g("ss_y"))
        torch.cuda.synchronize()
        got = pred.cpu().numpy().view(pdt).astype(np.uint16)
        np.testing.assert_array_equal(got, F["pred"][k], err_msg="row %d" % k)
        np.testing.assert_array_equal(dst.cpu().numpy().view(np.uint16), F["dst"][k],
                                      err_msg="row %d dst" % k)


def test_warp_shims_vs_reference(Wp):
    F = dict(np.load(os.path.join(GOLD, "fix_warp.npz")))
    J = {n: i for i, n in enumerate(F["row_fields"])}
    for k, r in enumerate(F["rows"]):
        if k % 3:
            continue
        g, W, H, RS, PS, DS, bd, cp = _case(F, r, J)
        pdt = np.uint16 if bd > 8 else np.uint8
        ref = np.ascontiguousarray(F["refs"][g("ref_index")].astype(pdt))
        pred = F["pred_in"][k].astype(pdt).copy()
        dst = F["dst_in"][k].copy()
        c = Wp.conv_params(dst=dst, dst_stride=DS, **cp)
        Wp.warp_affine_shim([g("m%d" % i) for i in range(6)], ref, W, H, RS, pred, g("p_col"),
                            g("p_row"), g("p_width"), g("p_height"), PS, g("ss_x"), g("ss_y"), c,
                            tuple(g(f) for f in ("alpha", "beta", "gamma", "delta")), bd)
        np.testing.assert_array_equal(pred.astype(np.uint16), F["pred"][k], err_msg="row %d" % k)
        np.testing.assert_array_equal(dst, F["dst"][k], err_msg="row %d dst" % k)


def _models(rng, n):
    """n random valid affine models (the reference test's parameter ranges)
    with their av1_get_shear_params values."""
    out = []
    while len(out) < n:
        m = [int(rng.integers(-(1 << 20), 1 << 20)), int(rng.integers(-(1 << 20), 1 << 20)),
             (1 << 16) + int(rng.integers(-4000, 4001)), int(rng.integers(-4000, 4001)), 0, 0]
        if rng.integers(0, 3) == 0:  # ROTZOOM
            m[4], m[5] = -m[3], m[2]
        else:
            m[4], m[5] = int(rng.integers(-4000, 4001)), (1 << 16) + int(rng.integers(-4000, 4001))
        ok, prm = O.get_shear_params(m)
        if ok:
            out.append((m, prm))
    return out


@pytest.mark.parametrize("bd", [8, 10, 12])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_warp_batch_vs_oracle(Wp, bd, mode):
    import torch
    rng = np.random.default_rng(7 * bd + mode)
    hb = bd > 8
    pdt = np.uint16 if hb else np.uint8
    W, H, NR = 320, 192, 3
    RS = W + 13
    refs = rng.integers(0, 1 << bd, (NR * H, RS)).astype(pdt)
    ss = (mode + bd) % 2
    shapes = [(8, 8), (16, 16), (4, 4), (16, 8), (32, 32), (8, 32), (12, 20)]
    nj = 300
    models = _models(rng, nj)
    PS, DS = 32, 32
    jobs = np.zeros(nj, Wp.JOB_DTYPE)
    pred_in = rng.integers(0, 1 << bd, (nj * 32, PS)).astype(pdt)
    dst_in = rng.integers(0, 1 << (bd + 4), (nj * 32, DS)).astype(np.uint16)
    for i, (m, prm) in enumerate(models):
        w, h = shapes[i % len(shapes)]
        jobs[i]["mat"] = m
        jobs[i]["alpha"], jobs[i]["beta"], jobs[i]["gamma"], jobs[i]["delta"] = prm
        jobs[i]["p_col"], jobs[i]["p_row"] = rng.integers(0, W // 2 - 32), rng.integers(0, H // 2 - 32)
        jobs[i]["p_width"], jobs[i]["p_height"] = w, h
        jobs[i]["ref_off"] = (i % NR) * H * RS
        jobs[i]["pred_off"] = i * 32 * PS
        jobs[i]["dst_off"] = i * 32 * DS
    r0 = 3 + max(bd + 7 - 3 + 2 - 16, 0)
    comp = int(mode > 0)
    cp = dict(round_0=r0, round_1=7 if comp else 14 - r0, is_compound=comp,
              do_average=int(mode >= 2), dist_wtd=int(mode == 3), fwd_offset=11 if mode == 3 else 0,
              bck_offset=5 if mode == 3 else 0)
    t = lambda a: torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a.copy()).cuda()
    tref, tpred, tdst = t(refs), t(pred_in), t(dst_in)
    Wp.warp_affine_batch(tref, W, H, RS, tpred, PS, torch.from_numpy(jobs.view(np.uint8)).cuda(),
                         nj, Wp.conv_params(**cp), bd, conv_dst=tdst, dst_stride=DS,
                         subsampling_x=ss, subsampling_y=ss)
    torch.cuda.synchronize()
    gp = tpred.cpu().numpy().view(pdt)
    gd = tdst.cpu().numpy().view(np.uint16)
    ep, ed = pred_in.copy(), dst_in.copy()
    ocp = dict(do_average=cp["do_average"], round_0=cp["round_0"], round_1=cp["round_1"],
               is_compound=comp, use_dist_wtd_comp_avg=cp["dist_wtd"],
               fwd_offset=cp["fwd_offset"], bck_offset=cp["bck_offset"])
    flat = refs.reshape(-1)
    for i in range(nj):
        jb = jobs[i]
        pv = ep[i * 32:(i + 1) * 32]
        dv = ed[i * 32:(i + 1) * 32]
        rv = flat[int(jb["ref_off"]):int(jb["ref_off"]) + H * RS]
        O.warp_affine(jb["mat"], rv, W, H, RS, pv, int(jb["p_col"]), int(jb["p_row"]),
                      int(jb["p_width"]), int(jb["p_height"]), PS, ss, ss, bd, int(hb), ocp, dv,
                      DS, (int(jb["alpha"]), int(jb["beta"]), int(jb["gamma"]), int(jb["delta"])))
    np.testing.assert_array_equal(gp, ep)
    np.testing.assert_array_equal(gd, ed)
    assert (gp != pred_in).any() or (gd != dst_in).any()
