"""GPU parity against the round-3 reference-executed fixtures (no oracle in
the loop; tests/golden/gen_fixtures.py sections convolve, compound12,
txfeat, trellis2):
  - the six single-reference convolve shims (av1_convolve_{x,y,2d}_sr_hip and
    the highbd forms) = av1_convolve_*_sr_c (convolve.c:76-188,687-787), bd
    8/10/12, 2x2 .. 128x128, five filters incl. 12-tap MULTITAP_SHARP2, with
    the kernel rows taken from the library's own table
    (lavish_interp_kernels);
  - lavish_dist_wtd_convolve_batch and the compound shims with the 12-tap
    kernel (the generic, non-8-tap compound kernel) up to 128x128;
  - lavish_tx_prune_features_batch / lavish_horver_correlation_batch / the
    av1_get_horver_correlation_full_hip shim = get_energy_distribution_finer +
    av1_get_horver_correlation_full_c, float bit patterns (0 ULP);
  - lavish_optimize_b_batch = av1_optimize_b at quant_sharpness 2."""
import ctypes
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return dict(np.load(os.path.join(GOLD, name)))


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_convolve_shims_vs_reference(torch):
    import lavish_dsp.inter as I
    F = _load("fix_convolve.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    oy, ox, pad = (int(v) for v in F["origin"])
    for r in F["rows"]:
        g = lambda k: int(r[J[k]])
        w, h, bd, path = g("w"), g("h"), g("bd"), g("path")
        pdt = np.uint8 if bd == 8 else np.uint16
        SS = w + pad
        src = np.ascontiguousarray(
            F["src"][g("src_off"):g("src_off") + (h + pad) * SS].astype(pdt))
        dst = np.full(w * h, 0x5A, pdt)
        tx = I.interp_kernels(g("filter_x"), w)
        ty = I.interp_kernels(g("filter_y"), h)
        fpx = I.filter_params(tx, tx.shape[1], g("filter_x"))
        fpy = I.filter_params(ty, ty.shape[1], g("filter_y"))
        I.convolve(("", "x", "y", "2d")[path], src, oy * SS + ox, SS, dst, 0, w, w, h, fpx, fpy,
                   g("subpel_x"), g("subpel_y"), g("round_0"), g("round_1"), bd)
        exp = F["dst"][g("dst_off"):g("dst_off") + w * h]
        np.testing.assert_array_equal(dst.astype(np.uint16), exp, err_msg=str(r))


def _cp(Cm, g, conv=None, stride=0):
    from lavish_dsp.inter import ConvolveParams
    d = conv.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)) if conv is not None else None
    return ConvolveParams(int(g("mode") > 0), d, stride, g("round_0"), g("round_1"), 0, 1,
                          int(g("mode") == 2), g("fwd_offset"), g("bck_offset"))


def test_compound_12tap_vs_reference(torch):
    import lavish_dsp.compound as Cm
    import lavish_dsp.inter as I
    F = _load("fix_compound12.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    oy, ox, pad = (int(v) for v in F["origin"])
    for k, r in enumerate(F["rows"]):
        g = lambda n: int(r[J[n]])
        bd, w, h = g("bd"), g("w"), g("h")
        hb = bd > 8
        pdt = np.uint16 if hb else np.uint8
        v = (lambda a: a.view(np.int16)) if hb else (lambda a: a)
        SS = w + pad
        src_np = np.ascontiguousarray(
            F["src"][g("src_off"):g("src_off") + (h + pad) * SS].astype(pdt))
        d0 = g("dst_off")
        fpx, tx = Cm.filter_params(I.interp_kernels(I.MULTITAP_SHARP2, w))
        fpy, ty = Cm.filter_params(I.interp_kernels(I.MULTITAP_SHARP2, h))
        exp_conv, exp_dst = F["conv"][d0:d0 + w * h], F["dst"][d0:d0 + w * h]
        # batch API
        src = torch.from_numpy(v(src_np.copy())).cuda()
        dst = torch.from_numpy(v(F["dst_in"][d0:d0 + w * h].astype(pdt).copy())).cuda()
        conv = torch.from_numpy(F["conv_in"][d0:d0 + w * h].view(np.int16).copy()).cuda()
        job = np.zeros(1, Cm.JOB_DTYPE)
        job["src_off"] = oy * SS + ox
        job["subpel_x_qn"], job["subpel_y_qn"] = g("subpel_x"), g("subpel_y")
        Cm.dist_wtd_convolve_batch(src, SS, dst, w, conv, w, w, h,
                                   torch.from_numpy(job.view(np.uint8)).cuda(), 1, fpx, fpy,
                                   _cp(Cm, g), bd)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(conv.cpu().numpy().view(np.uint16), exp_conv,
                                      err_msg="batch conv %s" % r)
        np.testing.assert_array_equal(dst.cpu().numpy().view(pdt).astype(np.uint16), exp_dst,
                                      err_msg="batch dst %s" % r)
        # per-call shim
        hdst = F["dst_in"][d0:d0 + w * h].astype(pdt).copy()
        hconv = F["conv_in"][d0:d0 + w * h].copy()
        addr = ctypes.c_void_p(src_np.ctypes.data + (oy * SS + ox) * src_np.itemsize)
        Cm.dist_wtd_convolve_shim(g("path"), addr, SS, hdst, w, w, h, fpx, fpy, g("subpel_x"),
                                  g("subpel_y"), _cp(Cm, g, hconv, w), bd)
        np.testing.assert_array_equal(hconv, exp_conv, err_msg="shim conv %s" % r)
        np.testing.assert_array_equal(hdst.astype(np.uint16), exp_dst, err_msg="shim dst %s" % r)


def test_tx_prune_features_vs_reference(torch):
    import lavish_dsp as L
    F = _load("fix_txfeat.npz")
    by_size = {}
    for k, (s, w, h, kind, off) in enumerate(F["rows"]):
        by_size.setdefault(int(s), []).append(k)
    for s, ks in by_size.items():
        w, h = L.TX_W[s], L.TX_H[s]
        # the size's blocks side by side in one plane: block b = fixture row ks[b]
        plane = np.concatenate([F["blocks"][F["rows"][k][4]:F["rows"][k][4] + w * h]
                                .reshape(h, w) for k in ks], axis=1)
        hf, vf = L.tx_prune_features(torch.from_numpy(np.ascontiguousarray(plane)).cuda(), s)
        hc, vc = L.horver_correlation_batch(torch.from_numpy(np.ascontiguousarray(plane)).cuda(),
                                            w, h)
        hf, vf, hc, vc = (t.cpu().numpy() for t in (hf, vf, hc, vc))
        nh = w if w <= 8 else w // 2
        nv = h if h <= 8 else h // 2
        for b, k in enumerate(ks):
            f = F["features"][k].view(np.float32)
            eh = np.concatenate([f[:nh - 1], f[32:33]])
            ev = np.concatenate([f[16:16 + nv - 1], f[33:34]])
            np.testing.assert_array_equal(hf[b][:nh].view(np.int32), eh.view(np.int32), str((s, k)))
            np.testing.assert_array_equal(vf[b][:nv].view(np.int32), ev.view(np.int32), str((s, k)))
            np.testing.assert_array_equal(np.array([hc[b], vc[b]], np.float32).view(np.int32),
                                          F["features"][k][32:34], str((s, k)))
    for k, (w, h, kind, off) in enumerate(F["horver_rows"]):
        blk = np.ascontiguousarray(F["horver_blocks"][off:off + w * h].reshape(h, w))
        got = np.array(L.av1_get_horver_correlation_full(blk, w, w, h), np.float32)
        np.testing.assert_array_equal(got.view(np.int32), F["horver"][k], str((w, h)))
        hc, vc = L.horver_correlation_batch(torch.from_numpy(blk).cuda(), w, h)
        got = np.array([hc.cpu().numpy()[0], vc.cpu().numpy()[0]], np.float32)
        np.testing.assert_array_equal(got.view(np.int32), F["horver"][k], str((w, h)))


def test_optimize_b_sharpness2_vs_reference(torch):
    import lavish_dsp as L
    from lavish_dsp import txb
    F = _load("fix_trellis_s2.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    costs = txb.CoeffCosts(txb.coeff_costs_blob(F["coeff_costs"], F["eob_costs"]))
    keys = ("bd", "tx_size", "tx_type", "qindex", "plane", "is_inter", "sharpness", "rdmult",
            "tx_type_cost")
    groups = {}
    for r in F["rows"]:
        groups.setdefault(tuple(int(r[J[k]]) for k in keys), []).append(r)
    n_checked = changed = 0
    for (bd, s, t, qindex, plane, inter, sharp, rdmult, ttc), rows in groups.items():
        n = L.max_eob(s)
        idx = [int(r[J["index"]]) for r in rows]
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
        tc, qc, dq = (dev(F[k][idx][:, :n]) for k in ("coeff", "qcoeff_in", "dqcoeff_in"))
        eob = dev(np.array([r[J["eob_in"]] for r in rows], np.int16))
        ctx = dev(np.array([[r[J["txb_skip_ctx"]], r[J["dc_sign_ctx"]]] for r in rows], np.int32))
        dqv = O.quant_arrays(O.build_quant(bd, qindex))["dequant"]
        rate, ec = txb.optimize_b_batch(costs, tc, qc, dq, eob, s, t, bd, rdmult, dqv, plane,
                                        inter, sharp, ctx, ttc)
        torch.cuda.synchronize()
        msg = "bd %d size %d type %d q %d plane %d inter %d" % (bd, s, t, qindex, plane, inter)
        np.testing.assert_array_equal(rate.cpu().numpy(), [r[J["rate"]] for r in rows], msg)
        np.testing.assert_array_equal(eob.cpu().numpy().view(np.uint16),
                                      [r[J["eob"]] for r in rows], msg)
        np.testing.assert_array_equal(ec.cpu().numpy(), [r[J["entropy_ctx"]] for r in rows], msg)
        np.testing.assert_array_equal(qc.cpu().numpy(), F["qcoeff"][idx][:, :n], msg)
        np.testing.assert_array_equal(dq.cpu().numpy(), F["dqcoeff"][idx][:, :n], msg)
        changed += int((F["qcoeff"][idx][:, :n] != F["qcoeff_in"][idx][:, :n]).any(1).sum())
        n_checked += len(rows)
    assert n_checked == len(F["rows"]) and changed > n_checked // 4
