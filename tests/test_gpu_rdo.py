"""GPU parity of the 64-point forward transforms and of the C4 fused TX-type
RDO (lavish_rdo_plane, and lavish_rdo_plane_px with pixel-domain
distortion) against the oracle (oracle/oracle_txfm.c,
oracle/oracle_rdo.c): coefficients, eobs, decision records (best type, eob,
rate, satd, distortion, sse, rd cost) and the winner's qcoeff / dqcoeff, all
bit-exact."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

SIZES64 = [4, 11, 12, 17, 18]


@pytest.fixture(scope="module")
def L():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp
    return lavish_dsp


@pytest.mark.parametrize("s", SIZES64)
def test_fwd_txfm2d_64_shims(L, s):
    """Whole W*H output buffer, including the stale words the reference's
    in-place zero + re-pack leaves behind."""
    rng = np.random.default_rng(s)
    W, H = O.TX_W[s], O.TX_H[s]
    for lim in (255, 1023, 4095, 32767):
        blk = rng.integers(-lim, lim + 1, size=(H, W + 3)).astype(np.int16)
        exp = O.fwd_txfm2d(blk, 0, s)
        got = np.full(W * H, 12345, np.int32)
        getattr(L, "av1_fwd_txfm2d_" + L.TX_SIZES[s])(blk, got, W + 3, 0, 8)
        np.testing.assert_array_equal(got, exp, err_msg="lim %d" % lim)


@pytest.mark.parametrize("s", SIZES64)
@pytest.mark.parametrize("bd,kind", [(8, 0), (8, 1), (10, 0), (12, 1)])
def test_txq_plane_64(L, s, bd, kind):
    import torch
    import lavish_dsp.synth as synth
    W, H = O.TX_W[s], O.TX_H[s]
    res = synth.residual_plane(256, 192, bd, seed=s)
    qp = L.build_quant_params(bd, 96, kind)
    out = L.txq_plane(torch.from_numpy(res).cuda(), s, 1, qp, bit_depth=bd, quant_kind=kind)
    qc, dq, eob = O.txq_plane(res, s, 1, O.build_quant(bd, 96), bd=bd, quant_b=bool(kind))
    n = O.max_eob(s)
    nb = (256 // W) * (192 // H)
    np.testing.assert_array_equal(out["qcoeff"].cpu().numpy().reshape(nb, n), qc.reshape(nb, n))
    np.testing.assert_array_equal(out["dqcoeff"].cpu().numpy().reshape(nb, n), dq.reshape(nb, n))
    np.testing.assert_array_equal(out["eob"].cpu().numpy().view(np.uint16).reshape(-1),
                                  eob.reshape(-1))


from _c4ref import planes as _planes, oracle_frame as _oracle_frame  # noqa: E402


# the C4 candidate set plus rectangular sizes
C4_CASES = [(4, 0x1), (3, 0x201), (2, 0xFFFF), (1, 0xFFFF), (0, 0xFFFF), (5, 0xFFFF),
            (9, 0x0201), (13, 0xFFFF), (16, 0x0201), (11, 0x1), (18, 0x1)]


@pytest.mark.parametrize("s,mask", C4_CASES)
@pytest.mark.parametrize("bd", [10, 8, 12])
def test_rdo_plane_vs_oracle(L, s, mask, bd):
    import torch
    src, pred = _planes(bd, 40 + s)
    q = O.build_quant(bd, 128)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    rdmult = 1234 + 17 * s
    exp, eq, ed = O.rdo_plane(src, pred, s, mask, bd, q, rdmult, threads=8)
    out = L.rdo_plane(torch.from_numpy(src.view(np.int16)).cuda(),
                      torch.from_numpy(pred.view(np.int16)).cuda(), s, mask, qp, rdmult, bd)
    got = L.rdo_records(out)
    for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), eq)
    np.testing.assert_array_equal(out["dqcoeff"].cpu().numpy(), ed)
    # more than one type wins somewhere when several are offered
    if bin(mask).count("1") > 2:
        assert len(np.unique(got["best_type"])) > 1


def test_rdo_large_residual_exact_path(L):
    """|src - pred| > 1023 (12-bit content) takes the exact 64-bit path."""
    import torch
    rng = np.random.default_rng(9)
    src = rng.integers(0, 4096, size=(64, 128)).astype(np.uint16)
    pred = rng.integers(0, 4096, size=(64, 128)).astype(np.uint16)
    q = O.build_quant(12, 60)
    qp = L.build_quant_params(12, 60, L.QUANT_FP)
    for s, mask in ((2, 0xFFFF), (4, 1), (3, 0x201)):
        exp, eq, ed = O.rdo_plane(src, pred, s, mask, 12, q, 4321)
        out = L.rdo_plane(torch.from_numpy(src.view(np.int16)).cuda(),
                          torch.from_numpy(pred.view(np.int16)).cuda(), s, mask, qp, 4321, 12)
        got = L.rdo_records(out)
        for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
            np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
        np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), eq)


@pytest.mark.parametrize("bd", [10, 8])
def test_rdo_frame_and_reconstruct(L, bd):
    """Whole C4 frame step (partial last SB row and column) vs the oracle."""
    import torch
    src, pred = _planes(bd, 77, Wp=328, Hp=200)
    masks = dict(L.C4_TYPE_MASKS)
    rdmult = 2000
    per, choice, recon = _oracle_frame(src, pred, bd, masks, rdmult)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    fr = L.RdoFrame(ts)
    L.rdo_frame(ts, tp, fr, L.build_quant_params(bd, 128, L.QUANT_FP), rdmult, bd)
    for s in masks:
        got = L.rdo_records(fr.outs[s])
        for f in ("best_type", "eob", "rdcost"):
            np.testing.assert_array_equal(got[f], per[s][0][f], err_msg="%d %s" % (s, f))
        np.testing.assert_array_equal(fr.outs[s]["dqcoeff"].cpu().numpy(), per[s][2])
    np.testing.assert_array_equal(fr.sb_tx_size.cpu().numpy(), choice)
    np.testing.assert_array_equal(fr.recon.cpu().numpy().view(np.uint16), recon)
    assert len(np.unique(choice)) > 1


# ---- pixel-domain distortion (lavish_rdo_plane_px / lavish_rdo_frame_px) ----

@pytest.mark.parametrize("s,mask", C4_CASES + [(15, 0x0201), (7, 0xFFFF), (14, 0xFFFF)])
@pytest.mark.parametrize("bd", [10, 8, 12])
def test_rdo_plane_px_vs_oracle(L, s, mask, bd):
    import torch
    src, pred = _planes(bd, 90 + s)
    q = O.build_quant(bd, 128)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    rdmult = 1500 + 13 * s
    exp, eq, ed = O.rdo_plane(src, pred, s, mask, bd, q, rdmult, threads=8, px=True)
    out = L.rdo_plane(torch.from_numpy(src.view(np.int16)).cuda(),
                      torch.from_numpy(pred.view(np.int16)).cuda(), s, mask, qp, rdmult, bd,
                      px=True)
    got = L.rdo_records(out)
    for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), eq)
    np.testing.assert_array_equal(out["dqcoeff"].cpu().numpy(), ed)
    # pixel-domain distortion differs from the TX-domain one somewhere
    td, _, _ = O.rdo_plane(src, pred, s, mask, bd, q, rdmult, threads=8)
    assert (td["dist"] != exp["dist"]).any()


def test_rdo_px_high_energy(L):
    """Full-range random content: every block is high-energy, so the
    TX-domain fallbacks (and the TX_64X64 quadrant-energy rule) are taken."""
    import torch
    rng = np.random.default_rng(5)
    for bd in (10, 12):
        mx = (1 << bd) - 1
        src = rng.integers(0, mx + 1, size=(128, 192)).astype(np.uint16)
        pred = rng.integers(0, mx + 1, size=(128, 192)).astype(np.uint16)
        q = O.build_quant(bd, 40)
        qp = L.build_quant_params(bd, 40, L.QUANT_FP)
        for s, mask in ((2, 0xFFFF), (4, 1), (3, 0x201), (0, 0xFFFF), (17, 1)):
            exp, _, _ = O.rdo_plane(src, pred, s, mask, bd, q, 777, px=True)
            out = L.rdo_plane(torch.from_numpy(src.view(np.int16)).cuda(),
                              torch.from_numpy(pred.view(np.int16)).cuda(), s, mask, qp, 777,
                              bd, px=True)
            got = L.rdo_records(out)
            for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
                np.testing.assert_array_equal(got[f], exp[f], err_msg="%d %d %s" % (bd, s, f))


def test_rdo_px_64_rejects_several_types(L):
    import torch
    src, pred = _planes(10, 3)
    qp = L.build_quant_params(10, 128, L.QUANT_FP)
    with pytest.raises(ValueError):
        L.rdo_plane(torch.from_numpy(src.view(np.int16)).cuda(),
                    torch.from_numpy(pred.view(np.int16)).cuda(), 4, 0x201, qp, 100, 10,
                    px=True)


@pytest.mark.parametrize("bd", [10, 8])
def test_rdo_frame_px_and_reconstruct(L, bd):
    import torch
    src, pred = _planes(bd, 78, Wp=328, Hp=200)
    masks = dict(L.C4_TYPE_MASKS)
    rdmult = 2000
    per, choice, recon = _oracle_frame(src, pred, bd, masks, rdmult, px=True)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    fr = L.RdoFrame(ts)
    L.rdo_frame(ts, tp, fr, L.build_quant_params(bd, 128, L.QUANT_FP), rdmult, bd, px=True)
    for s in masks:
        got = L.rdo_records(fr.outs[s])
        for f in ("best_type", "eob", "dist", "sse", "rdcost"):
            np.testing.assert_array_equal(got[f], per[s][0][f], err_msg="%d %s" % (s, f))
        np.testing.assert_array_equal(fr.outs[s]["dqcoeff"].cpu().numpy(), per[s][2])
    np.testing.assert_array_equal(fr.sb_tx_size.cpu().numpy(), choice)
    np.testing.assert_array_equal(fr.recon.cpu().numpy().view(np.uint16), recon)


def test_rdo_frame_px_every_64_point_size(L):
    """All five 64-point sizes in one lavish_rdo_frame_px call: they run on
    concurrent fan-out streams, each with its own scratch plane / job list
    (rdo_plane_px64), and a second call reuses the scratch."""
    import torch
    bd = 10
    src, pred = _planes(bd, 79, Wp=384, Hp=256)
    masks = {4: 0x1, 11: 0x1, 12: 0x1, 17: 0x1, 18: 0x1, 3: 0x201, 2: 0xFFFF}
    rdmult = 1900
    q = O.build_quant(bd, 128)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    fr = L.RdoFrame(ts, type_masks=masks)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    for _ in range(2):
        L.rdo_frame(ts, tp, fr, qp, rdmult, bd, px=True, reconstruct=False)
    torch.cuda.synchronize()
    for s, m in masks.items():
        exp, eq, ed = O.rdo_plane(src, pred, s, m, bd, q, rdmult, threads=8, px=True)
        got = L.rdo_records(fr.outs[s])
        for f in ("best_type", "eob", "dist", "sse", "rdcost"):
            np.testing.assert_array_equal(got[f], exp[f], err_msg="%d %s" % (s, f))
        np.testing.assert_array_equal(fr.outs[s]["dqcoeff"].cpu().numpy(), ed)
