"""GPU parity tests: the HIP transform+quantize path (liblavish_hip.so) against
the CPU oracle, bit-exact.

Structure follows the reference's own tests:
* AV1FwdTxfm2dMatchTest (test/av1_fwd_txfm2d_test.cc:243-297): all-max input
  first, then random blocks, every valid (tx_size, tx_type), bit-exact.
* QuantizeTest (test/quantize_func_test.cc:135-340): random spans, DC-only,
  -8191 fills, CoeffHalfDequant, MultipleQ over qindex; fp and b,
  log_scale 0/1/2, lowbd and highbd; qcoeff, dqcoeff and eob bit-exact.
* plane batches at sizes the oracle finishes in seconds, plus size-independent
  properties (eob/scan consistency, dq = dequant(q), determinism) on a full
  1920x1080 frame.
"""
import numpy as np
import pytest

import _oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SIZES_LE32 = [s for s in range(19) if O.TX_W[s] <= 32 and O.TX_H[s] <= 32]


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import lavish_dsp
    return lavish_dsp


def _mask(s):
    return sum(1 << t for t in range(16) if O.type_valid(s, t))


def _plane(w, h, bd, seed, kind="random"):
    rng = np.random.RandomState(seed)
    m = (1 << bd) - 1
    if kind == "random":
        return rng.randint(-m, m + 1, size=(h, w)).astype(np.int16)
    if kind == "max":
        return np.full((h, w), m, np.int16)
    if kind == "min":
        return np.full((h, w), -m, np.int16)
    if kind == "sparse":
        r = rng.randint(-m, m + 1, size=(h, w))
        r[rng.rand(h, w) < 0.9] = 0
        return r.astype(np.int16)
    if kind == "extreme16":
        return rng.randint(-32768, 32768, size=(h, w)).astype(np.int16)
    raise ValueError(kind)


def _run_plane(L, res, s, mask, bd, qindex, quant_b):
    kind = L.QUANT_B if quant_b else L.QUANT_FP
    qp = L.build_quant_params(bd, qindex, kind)
    dres = torch.from_numpy(res).cuda()
    out = L.txq_plane(dres, s, mask, qp, bit_depth=bd, quant_kind=kind, with_coeff=True)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def _oracle_plane(res, s, mask, bd, qindex, quant_b):
    q = O.build_quant(bd, qindex)
    qc, dq, eob = O.txq_plane(res, s, mask, q, bd=bd, quant_b=quant_b, threads=8)
    # oracle layout [block][slot][n] -> product layout [slot][block][n]
    return qc.transpose(1, 0, 2), dq.transpose(1, 0, 2), eob.T


@pytest.mark.parametrize("s", SIZES_LE32)
@pytest.mark.parametrize("quant_b", [False, True])
def test_txq_plane_parity_lowbd(L, s, quant_b):
    W, H = O.TX_W[s], O.TX_H[s]
    # a plane whose block count is not a multiple of the per-workgroup block
    # count, and whose width leaves a partial (ignored) column of blocks
    pw, ph = 13 * W + W // 2, 7 * H
    mask = _mask(s)
    for kind, qindex, seed in (("max", 128, 1), ("min", 0, 2), ("random", 128, 3),
                               ("random", 255, 4), ("sparse", 32, 5), ("random", 1, 6)):
        res = _plane(pw, ph, 8, seed, kind)
        got = _run_plane(L, res, s, mask, 8, qindex, quant_b)
        qc, dq, eob = _oracle_plane(res, s, mask, 8, qindex, quant_b)
        tag = (O.TX_NAMES[s], kind, qindex, quant_b)
        np.testing.assert_array_equal(got["qcoeff"], qc, err_msg=str(tag))
        np.testing.assert_array_equal(got["dqcoeff"], dq, err_msg=str(tag))
        np.testing.assert_array_equal(got["eob"].view(np.uint16), eob, err_msg=str(tag))


@pytest.mark.parametrize("s", SIZES_LE32)
def test_txq_plane_parity_highbd(L, s):
    W, H = O.TX_W[s], O.TX_H[s]
    mask = _mask(s)
    for bd, quant_b, qindex, kind in ((10, False, 100, "random"), (10, True, 60, "max"),
                                      (12, False, 200, "random"), (12, True, 7, "sparse")):
        res = _plane(9 * W, 5 * H, bd, 11 + bd, kind)
        got = _run_plane(L, res, s, mask, bd, qindex, quant_b)
        qc, dq, eob = _oracle_plane(res, s, mask, bd, qindex, quant_b)
        tag = (O.TX_NAMES[s], bd, quant_b, qindex, kind)
        np.testing.assert_array_equal(got["qcoeff"], qc, err_msg=str(tag))
        np.testing.assert_array_equal(got["dqcoeff"], dq, err_msg=str(tag))
        np.testing.assert_array_equal(got["eob"].view(np.uint16), eob, err_msg=str(tag))


@pytest.mark.parametrize("s", SIZES_LE32)
def test_fwd_txfm2d_coeff_parity(L, s):
    """transform-only output of the batch path, including full-range int16
    input (overflow-wrapping arithmetic must match the reference)."""
    W, H = O.TX_W[s], O.TX_H[s]
    mask = _mask(s)
    for kind in ("random", "extreme16", "max"):
        res = _plane(6 * W, 3 * H, 8, 21, kind)
        qp = L.build_quant_params(8, 100, L.QUANT_FP)
        dres = torch.from_numpy(res).cuda()
        out = L.txq_plane(dres, s, mask, qp, quant_kind=L.QUANT_NONE, with_coeff=True)
        coeff = out["coeff"].cpu().numpy()
        types = [t for t in range(16) if (mask >> t) & 1]
        for bi in range(coeff.shape[1]):
            by, bx = divmod(bi, res.shape[1] // W)
            blk = res[by * H:(by + 1) * H, bx * W:(bx + 1) * W]
            for si, t in enumerate(types):
                np.testing.assert_array_equal(coeff[si, bi], O.fwd_txfm2d(blk, t, s),
                                              err_msg=str((O.TX_NAMES[s], kind, bi, t)))


@pytest.mark.parametrize("s", SIZES_LE32)
def test_fwd_txfm2d_shims(L, s):
    """av1_fwd_txfm2d_WxH_hip per-call shims: all-max block first, then random
    blocks in a strided buffer (AV1FwdTxfm2dMatchTest)."""
    W, H = O.TX_W[s], O.TX_H[s]
    fn = getattr(L, "av1_fwd_txfm2d_" + O.TX_NAMES[s])
    rnd = O.ACMRandom(0xBABA)
    stride = W + 5
    for t in range(16):
        if not O.type_valid(s, t):
            continue
        for it in range(4):
            buf = np.zeros((H, stride), np.int16)
            if it == 0:
                buf[:, :W] = 255
            else:
                buf[:, :W] = np.array([rnd.rand8() - rnd.rand8() for _ in range(W * H)],
                                      np.int16).reshape(H, W)
            out = np.zeros(W * H, np.int32)
            fn(buf.ravel(), out, stride, t, 8)
            np.testing.assert_array_equal(out, O.fwd_txfm2d(buf, t, s),
                                          err_msg=str((O.TX_NAMES[s], t, it)))
    # av1_lowbd_fwd_txfm dispatch
    p = L.TxfmParam(tx_type=0, tx_size=s, lossless=0, bd=8, is_hbd=0, tx_set_type=5, eob=0)
    buf = np.arange(H * stride, dtype=np.int16).reshape(H, stride) % 37 - 18
    out = np.zeros(W * H, np.int32)
    L.av1_lowbd_fwd_txfm(buf.ravel(), out, stride, p)
    np.testing.assert_array_equal(out, O.fwd_txfm2d(buf, 0, s))


QUANT_FNS = [  # (shim name, kind, log_scale, highbd)
    ("av1_quantize_fp", "fp", 0, False), ("av1_quantize_fp_32x32", "fp", 1, False),
    ("av1_quantize_fp_64x64", "fp", 2, False), ("aom_quantize_b", "b", 0, False),
    ("aom_quantize_b_32x32", "b", 1, False), ("aom_quantize_b_64x64", "b", 2, False),
    ("aom_highbd_quantize_b", "b", 0, True), ("aom_highbd_quantize_b_32x32", "b", 1, True),
    ("aom_highbd_quantize_b_64x64", "b", 2, True),
]


@pytest.mark.parametrize("name,kind,ls,highbd", QUANT_FNS)
def test_quantize_shims(L, name, kind, ls, highbd):
    """quantize_func_test.cc fills: random span, DC only, -8191, half dequant,
    multiple q (subset of the 256 qindex sweep)."""
    fn = getattr(L, name)
    tx = {0: 2, 1: 3, 2: 3}[ls]  # 16x16, 32x32 (64x64 uses the 32x32 scan)
    n = O.max_eob(tx) if ls < 2 else 1024
    scan, iscan = L.scan_order(tx, 0)
    bd = 10 if highbd else 8
    rnd = O.ACMRandom(0xBABA)
    for qindex in (0, 1, 37, 128, 200, 255):
        q = O.build_quant(bd, qindex)
        qa = O.quant_arrays(q)
        rnd_arr = qa["round_fp"] if kind == "fp" else qa["round"]
        qt_arr = qa["quant_fp"] if kind == "fp" else qa["quant"]
        for fill in ("random", "dc", "neg8191", "half"):
            c = np.zeros(n, np.int32)
            if fill == "random":
                span = 1 << (7 + bd)
                for i in range(n):
                    c[i] = rnd.pseudo_uniform(2 * span) - span
            elif fill == "dc":
                c[0] = rnd.pseudo_uniform(1 << (8 + bd)) - (1 << (7 + bd))
            elif fill == "neg8191":
                c[:] = -8191
            else:
                c[:] = (qa["dequant"][1] >> 1) * (1 if qindex % 2 else -1)
                c[0] = qa["dequant"][0] >> 1
            qc = np.zeros(n, np.int32)
            dq = np.zeros(n, np.int32)
            eob = np.zeros(1, np.uint16)
            fn(c, n, qa["zbin"], rnd_arr, qt_arr, qa["quant_shift"], qc, dq, qa["dequant"],
               eob, scan, iscan)
            rq, rdq, reob = O.quantize(kind, c, n, q, scan, iscan, ls, highbd=highbd)
            tag = (name, qindex, fill)
            np.testing.assert_array_equal(qc, rq, err_msg=str(tag))
            np.testing.assert_array_equal(dq, rdq, err_msg=str(tag))
            assert int(eob[0]) == reob, tag


@pytest.mark.parametrize("ls", [0, 1, 2])
def test_highbd_quantize_fp_shim(L, ls):
    tx = {0: 2, 1: 3, 2: 3}[ls]
    n = 1024 if ls == 2 else O.max_eob(tx)
    scan, iscan = L.scan_order(tx, 0)
    rng = np.random.RandomState(ls)
    for qindex in (0, 50, 180, 255):
        q = O.build_quant(10, qindex)
        qa = O.quant_arrays(q)
        c = rng.randint(-(1 << 18), 1 << 18, size=n).astype(np.int32)
        c[rng.rand(n) < 0.5] = 0
        qc = np.zeros(n, np.int32)
        dq = np.zeros(n, np.int32)
        eob = np.zeros(1, np.uint16)
        L.av1_highbd_quantize_fp(c, n, qa["zbin"], qa["round_fp"], qa["quant_fp"],
                                 qa["quant_shift"], qc, dq, qa["dequant"], eob, scan, iscan, ls)
        rq, rdq, reob = O.quantize("fp", c, n, q, scan, iscan, ls, highbd=True)
        np.testing.assert_array_equal(qc, rq)
        np.testing.assert_array_equal(dq, rdq)
        assert int(eob[0]) == reob


def test_quantize_batch(L):
    rng = np.random.RandomState(5)
    for tx, t in ((1, 10), (2, 11), (3, 0), (7, 3)):
        n = O.max_eob(tx)
        ls = O.tx_scale(tx)
        scan, iscan = L.scan_order(tx, t)
        coeff = rng.randint(-3000, 3000, size=(37, n)).astype(np.int32)
        for kind, qk in (("fp", L.QUANT_FP), ("b", L.QUANT_B)):
            qp = L.build_quant_params(8, 90, qk)
            q, dq, eob = L.quantize_batch(torch.from_numpy(coeff).cuda(),
                                          torch.from_numpy(scan).cuda(), ls, qp, quant_kind=qk)
            q, dq, eob = q.cpu().numpy(), dq.cpu().numpy(), eob.cpu().numpy().view(np.uint16)
            oq = O.build_quant(8, 90)
            for b in range(coeff.shape[0]):
                rq, rdq, reob = O.quantize(kind, coeff[b], n, oq, scan, iscan, ls)
                np.testing.assert_array_equal(q[b], rq)
                np.testing.assert_array_equal(dq[b], rdq)
                assert eob[b] == reob


def test_full_frame_properties(L):
    """C2 at its full size (1920x1080, qindex 128, every size <= 32 and every
    valid type): size-independent properties plus oracle spot checks."""
    import lavish_dsp.synth as synth
    res = synth.residual_plane(1920, 1080, 8)
    dres = torch.from_numpy(res).cuda()
    qp = L.build_quant_params(8, 128, L.QUANT_FP)
    dq_fp = qp.as_dict()["dequant"]
    rng = np.random.RandomState(0)
    for s in SIZES_LE32:
        W, H = O.TX_W[s], O.TX_H[s]
        mask = _mask(s)
        out = L.txq_plane(dres, s, mask, qp)
        out2 = L.txq_plane(dres, s, mask, qp)
        torch.cuda.synchronize()
        q = out["qcoeff"]
        assert torch.equal(q, out2["qcoeff"]) and torch.equal(out["eob"], out2["eob"])
        qn = q.cpu().numpy()
        dqn = out["dqcoeff"].cpu().numpy()
        eob = out["eob"].cpu().numpy().view(np.uint16)
        types = [t for t in range(16) if (mask >> t) & 1]
        n = O.max_eob(s)
        ls = O.tx_scale(s)
        # dq == sign(q) * ((|q| * dequant) >> log_scale)
        deq = np.full(n, dq_fp[1], np.int64)
        deq[0] = dq_fp[0]
        exp_dq = np.sign(qn) * ((np.abs(qn).astype(np.int64) * deq) >> ls)
        np.testing.assert_array_equal(dqn, exp_dq)
        for si, t in enumerate(types):
            scan, iscan = L.scan_order(s, t)
            pos = iscan.astype(np.int64)
            nz = qn[si] != 0
            last = np.where(nz, pos[None, :] + 1, 0).max(axis=1)
            np.testing.assert_array_equal(eob[si], last)
        # spot-check 24 random blocks against the oracle
        nb = (1920 // W) * (1080 // H)
        oq = O.build_quant(8, 128)
        for bi in rng.randint(0, nb, size=24):
            by, bx = divmod(int(bi), 1920 // W)
            blk = res[by * H:(by + 1) * H, bx * W:(bx + 1) * W]
            for si, t in enumerate(types):
                coeff = O.fwd_txfm2d(blk, t, s)
                scan, iscan = L.scan_order(s, t)
                rq, rdq, reob = O.quantize("fp", coeff, n, oq, scan, iscan, ls)
                np.testing.assert_array_equal(qn[si, bi], rq)
                assert eob[si, bi] == reob


def test_txq_frame_matches_per_size(L):
    """lavish_txq_frame (concurrent per-size kernels) == per-size launches ==
    oracle on a small plane with every size <= 32."""
    res = _plane(256, 96, 8, 77, "random")
    dres = torch.from_numpy(res).cuda()
    qp = L.build_quant_params(8, 140, L.QUANT_FP)
    frame = L.FrameOutputs(dres, SIZES_LE32)
    outs = L.txq_frame(dres, frame, qp)
    torch.cuda.synchronize()
    for s in SIZES_LE32:
        qc, dq, eob = _oracle_plane(res, s, _mask(s), 8, 140, False)
        np.testing.assert_array_equal(outs[s]["qcoeff"].cpu().numpy(), qc)
        np.testing.assert_array_equal(outs[s]["dqcoeff"].cpu().numpy(), dq)
        np.testing.assert_array_equal(outs[s]["eob"].cpu().numpy().view(np.uint16), eob)
