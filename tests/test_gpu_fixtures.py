"""GPU parity against the fixtures produced by executing the reference's own
C function bodies (tests/golden/gen_fixtures.py): the same inputs go through
the HIP path -- the batch C ABI (lavish_txq_plane, lavish_quantize_batch,
lavish_inv_txfm_add_batch) and the per-call RTCD shims -- and the outputs must
equal the reference's, bit for bit.  No oracle in the loop."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TX_W = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
TX_H = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]


@pytest.fixture(scope="module")
def L():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp
    return lavish_dsp


def _load(name):
    return dict(np.load(os.path.join(GOLD, name)))


@pytest.fixture(scope="module")
def FT():
    return _load("fix_txfm.npz")


@pytest.fixture(scope="module")
def FQ():
    return _load("fix_quant.npz")


@pytest.fixture(scope="module")
def FI():
    return _load("fix_inv.npz")


def _types(L, s):
    return [t for t in range(16) if L.tx_type_valid(s, t)]


@pytest.mark.parametrize("s", range(19))
def test_fwd_batch_vs_reference(L, FT, s):
    """lavish_txq_plane (coefficients, no quantization) over a plane made of
    the fixture blocks side by side, every valid type in one launch."""
    import torch
    W, H = TX_W[s], TX_H[s]
    n = L.max_eob(s)
    types = _types(L, s)
    mask = sum(1 << t for t in types)
    k = len(FT["in_%d_%d" % (s, types[0])])
    for j in range(k):
        # one plane per block index: the types see different inputs, so run
        # each type's block j through a one-block-wide plane
        for t in types:
            blk = FT["in_%d_%d" % (s, t)][j]
            res = torch.from_numpy(np.ascontiguousarray(blk)).cuda()
            out = L.txq_plane(res, s, mask, None, quant_kind=L.QUANT_NONE, with_coeff=True)
            torch.cuda.synchronize()
            got = out["coeff"][types.index(t), 0].cpu().numpy()
            np.testing.assert_array_equal(got, FT["out_%d_%d" % (s, t)][j][:n],
                                          err_msg="size %d type %d block %d" % (s, t, j))


@pytest.mark.parametrize("s", range(19))
def test_fwd_shims_vs_reference(L, FT, s):
    """av1_fwd_txfm2d_{WxH}_hip: the whole W*H output buffer the reference
    writes (64-point sizes: zeroed + re-packed in place)."""
    W, H = TX_W[s], TX_H[s]
    fn = getattr(L, "av1_fwd_txfm2d_" + L.TX_SIZES[s])
    for t in _types(L, s):
        for blk, exp, bd in zip(FT["in_%d_%d" % (s, t)], FT["out_%d_%d" % (s, t)],
                                FT["bd_%d_%d" % (s, t)]):
            padded = np.zeros((H, W + 3), np.int16)
            padded[:, :W] = blk
            got = np.full(W * H, 0x5A5A5A5A, np.int32)
            fn(padded, got, W + 3, t, int(bd))
            np.testing.assert_array_equal(got, exp, err_msg="size %d type %d" % (s, t))


def _qp(L, F, bd, q, kind):
    qp = L.QuantParams()
    G = _load("fix_qparams.npz")
    fields = {"zbin": "y_zbin", "quant_shift": "y_quant_shift", "dequant": "y_dequant_QTX",
              "round": "y_round_fp" if kind == "fp" else "y_round",
              "quant": "y_quant_fp" if kind == "fp" else "y_quant"}
    for mine, ref in fields.items():
        row = G["%s_bd%d_sh0" % (ref, bd)][q]
        getattr(qp, mine)[0], getattr(qp, mine)[1] = int(row[0]), int(row[1])
    return qp


def _quant_cases(FQ):
    for ci, (s, ls, hb, isb) in enumerate(FQ["cases"]):
        for q in (0, 32, 128, 255):
            yield ci, int(s), int(ls), bool(hb), bool(isb), 10 if hb else 8, q


def test_quantize_batch_vs_reference(L, FQ):
    """lavish_quantize_batch with the reference's av1_build_quantizer tables
    and DCT_DCT scan: qcoeff, dqcoeff, eob of every fixture block."""
    import torch
    checked = 0
    for ci, s, ls, hb, isb, bd, q in _quant_cases(FQ):
        key = "%d_%d_q%d" % (ci, bd, q)
        coeff = torch.from_numpy(FQ["coeff_" + key]).cuda()
        scan, _ = L.scan_order(s, 0)
        qp = _qp(L, FQ, bd, q, "b" if isb else "fp")
        qc, dq, eob = L.quantize_batch(coeff, torch.from_numpy(scan).cuda(), ls, qp, bit_depth=bd,
                                       quant_kind=L.QUANT_B if isb else L.QUANT_FP)
        torch.cuda.synchronize()
        msg = "%s size %d q %d" % (FQ["case_names"][ci], s, q)
        np.testing.assert_array_equal(qc.cpu().numpy(), FQ["qcoeff_" + key], err_msg=msg)
        np.testing.assert_array_equal(dq.cpu().numpy(), FQ["dqcoeff_" + key], err_msg=msg)
        np.testing.assert_array_equal(eob.cpu().numpy().view(np.uint16), FQ["eob_" + key],
                                      err_msg=msg)
        checked += len(coeff)
    assert checked > 300


def test_quantize_shims_vs_reference(L, FQ):
    """The per-call RTCD shims named like the reference's functions
    (av1_quantize_fp_hip, aom_quantize_b_32x32_hip, ...)."""
    G = _load("fix_qparams.npz")
    for ci, s, ls, hb, isb, bd, q in _quant_cases(FQ):
        name = str(FQ["case_names"][ci])[:-2]  # drop "_c"
        key = "%d_%d_q%d" % (ci, bd, q)
        n = L.max_eob(s)
        scan, iscan = L.scan_order(s, 0)
        row = lambda f: np.ascontiguousarray(G["%s_bd%d_sh0" % (f, bd)][q])
        rnd, qnt = (row("y_round"), row("y_quant")) if isb else (row("y_round_fp"),
                                                                  row("y_quant_fp"))
        for k, c in enumerate(FQ["coeff_" + key]):
            qc = np.full(n, 99, np.int32)
            dq = np.full(n, 99, np.int32)
            eob = np.zeros(1, np.uint16)
            args = [np.ascontiguousarray(c), n, row("y_zbin"), rnd, qnt, row("y_quant_shift"), qc,
                    dq, row("y_dequant_QTX"), eob, scan, iscan]
            if name == "av1_highbd_quantize_fp":
                args.append(ls)
            getattr(L, name)(*args)
            msg = "%s q %d block %d" % (name, q, k)
            np.testing.assert_array_equal(qc, FQ["qcoeff_" + key][k], err_msg=msg)
            np.testing.assert_array_equal(dq, FQ["dqcoeff_" + key][k], err_msg=msg)
            assert eob[0] == FQ["eob_" + key][k], msg


@pytest.mark.parametrize("s", range(19))
def test_inv_batch_vs_reference(L, FI, s):
    """lavish_inv_txfm_add_batch: every fixture block of a (size, type, bd)
    added into its own destination window of one u16 plane."""
    import torch
    W, H = TX_W[s], TX_H[s]
    n = L.max_eob(s)
    for t in _types(L, s):
        key = "%d_%d" % (s, t)
        ins, dsts, outs, bds = FI["in_" + key], FI["dst_" + key], FI["out_" + key], FI["bd_" + key]
        for bd in (8, 10, 12):
            sel = np.nonzero(bds == bd)[0]
            k = len(sel)
            plane = np.concatenate([dsts[i] for i in sel], axis=1)  # [H, k * (W + 5)]
            jobs = np.zeros(k, L.INV_JOB_DTYPE)
            jobs["dst_off"] = np.arange(k) * (W + 5)
            jobs["coeff_off"] = np.arange(k) * n
            jobs["tx_type"] = t
            jobs["eob"] = n
            dq = torch.from_numpy(np.concatenate([ins[i] for i in sel])).cuda()
            dst = torch.from_numpy(plane.view(np.int16).copy()).cuda()
            import lavish_dsp.motion as M
            L.inv_txfm_add_batch(dq, s, M.to_device(jobs), dst, bit_depth=bd)
            got = dst.cpu().numpy().view(np.uint16)
            exp = np.concatenate([outs[i] for i in sel], axis=1)
            np.testing.assert_array_equal(got, exp, err_msg="size %d type %d bd %d" % (s, t, bd))


@pytest.mark.parametrize("s", range(19))
def test_inv_shims_vs_reference(L, FI, s):
    """av1_inv_txfm2d_add_{WxH}_hip on the fixture's u16 destination (stride
    W + 5, only the W x H window may change)."""
    for t in _types(L, s):
        key = "%d_%d" % (s, t)
        for c, dst, exp, bd in zip(FI["in_" + key], FI["dst_" + key], FI["out_" + key],
                                   FI["bd_" + key]):
            d = dst.copy()
            L.av1_inv_txfm2d_add(s, np.ascontiguousarray(c), d, d.shape[1], t, int(bd))
            np.testing.assert_array_equal(d, exp, err_msg="size %d type %d bd %d" % (s, t, bd))


# ---------------------------------------------------------------- pixel --
BLOCK_SIZES = [(128, 128), (128, 64), (64, 128), (64, 64), (64, 32), (32, 64), (32, 32), (32, 16),
               (16, 32), (16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4), (4, 16),
               (16, 4), (8, 32), (32, 8), (16, 64), (64, 16)]
SUBPEL_OFFSETS = [(0, 0), (3, 0), (0, 5), (4, 4), (7, 2)]


@pytest.fixture(scope="module")
def FP():
    return _load("fix_pixel.npz")


@pytest.fixture(scope="module")
def PX():
    import lavish_dsp.pixel as PX
    return PX


@pytest.mark.parametrize("W,H", BLOCK_SIZES)
@pytest.mark.parametrize("bd", [8, 10])
def test_sad_variance_shims_vs_reference(L, PX, FP, W, H, bd):
    k = "%dx%d_bd%d" % (W, H, bd)
    dt = np.uint8 if bd == 8 else np.uint16
    a, b = FP["src_" + k].astype(dt), FP["ref_" + k].astype(dt)
    hb = bd > 8
    ss, rs = a.shape[1], b.shape[1]
    assert PX.sad(W, H, a, ss, b, rs, highbd=hb) == FP["sad_" + k][0]
    assert PX.sad(W, H, a, ss, b, rs, highbd=hb, skip=True) == FP["sadskip_" + k][0]
    flat = b.reshape(-1)
    got4 = PX.sad_x4d(W, H, a, ss, [flat[o:] for o in (0, 1, 3, W + 2)], rs, highbd=hb)
    np.testing.assert_array_equal(got4, FP["sadx4d_" + k])
    assert list(PX.variance(W, H, a, ss, b, rs, bd, hb)) == list(FP["var_" + k])
    got = [PX.sub_pixel_variance(W, H, a, ss, xo, yo, b, rs, bd, hb) for xo, yo in SUBPEL_OFFSETS]
    np.testing.assert_array_equal(np.array(got, np.int64), FP["subvar_" + k])


@pytest.mark.parametrize("bd", [8, 10])
def test_sad_variance_batch_vs_reference(L, PX, FP, bd):
    """lavish_sad_batch / lavish_variance_batch over every block size's
    fixture planes (x4d candidates as four ref offsets of one job)."""
    import torch
    for W, H in BLOCK_SIZES:
        k = "%dx%d_bd%d" % (W, H, bd)
        dt = np.uint8 if bd == 8 else np.int16
        a = torch.from_numpy(FP["src_" + k].astype(np.uint16).astype(dt)).cuda()
        b = torch.from_numpy(FP["ref_" + k].astype(np.uint16).astype(dt)).cuda()
        jobs = np.zeros(1, PX.JOB_DTYPE)
        jobs["ref_off"][0] = (0, 1, 3, W + 2)
        dj = PX.jobs_tensor(jobs, "cuda")
        got = PX.sad_batch(a, b, W, H, dj, nrefs=4).cpu().numpy()[0]
        np.testing.assert_array_equal(got, FP["sadx4d_" + k], err_msg=k)
        got = PX.sad_batch(a, b, W, H, dj, nrefs=1, mode=1).cpu().numpy()[0, 0]
        assert got == FP["sadskip_" + k][0], k
        v = PX.variance_batch(a, b, W, H, dj, kind=0, bit_depth=bd)
        assert [int(v["var"][0]), int(v["sse"][0])] == list(FP["var_" + k]), k
        sj = np.zeros(len(SUBPEL_OFFSETS), PX.JOB_DTYPE)
        sj["xoff"], sj["yoff"] = zip(*SUBPEL_OFFSETS)
        v = PX.variance_batch(a, b, W, H, PX.jobs_tensor(sj, "cuda"), kind=3, bit_depth=bd)
        got = np.stack([v["var"].cpu().numpy(), v["sse"].cpu().numpy()], 1)
        np.testing.assert_array_equal(got, FP["subvar_" + k], err_msg=k)


def test_hadamard_satd_lp_vs_reference(L, PX, FP):
    import torch
    for n in (4, 8, 16, 32):
        for bd in (8, 10):
            k = "%d_bd%d" % (n, bd)
            if "had_" + k not in FP:
                continue
            res = FP["hres_" + k]
            got = PX.hadamard(n, res, res.shape[1], highbd=bd > 8)
            np.testing.assert_array_equal(got, FP["had_" + k], err_msg=k)
            assert PX.satd(got, n * n) == FP["satd_" + k][0]
            if "hadlp_" + k in FP:
                lp = PX.hadamard_lp(n, res, res.shape[1])
                np.testing.assert_array_equal(lp, FP["hadlp_" + k], err_msg=k)
                assert PX.satd_lp(lp, n * n) == FP["satdlp_" + k][0]
                jobs = np.zeros(1, PX.JOB_DTYPE)
                out = PX.hadamard_lp_batch(n, torch.from_numpy(res).cuda(),
                                           PX.jobs_tensor(jobs, "cuda"), n * n)
                np.testing.assert_array_equal(out.cpu().numpy(), FP["hadlp_" + k], err_msg=k)
    # the dual form: two 8x8 lp transforms side by side (avg.c:238-245)
    res = FP["hres_16_bd8"]
    dual = PX.hadamard_lp(8, res, res.shape[1], dual=True)
    np.testing.assert_array_equal(dual[:64], PX.hadamard_lp(8, res, res.shape[1]))
    np.testing.assert_array_equal(dual[64:], PX.hadamard_lp(8, res[:, 8:], res.shape[1]))


def test_block_error_lp_vs_reference(L, PX, FP):
    for n in (16, 64, 256, 1024, 4096):
        c, d = FP["be_c_%d" % n], FP["be_d_%d" % n]
        assert list(PX.block_error(c, d, n)) == list(FP["be_%d" % n])
        for bd in (10, 12):
            assert list(PX.block_error(c, d, n, bd)) == list(FP["behb_%d_bd%d" % (n, bd)])
        assert PX.block_error_lp(FP["belp_c_%d" % n], FP["belp_d_%d" % n], n) == \
            FP["belp_%d" % n][0]


def test_subtract_sse_sums_vs_reference(L, PX, FP):
    for (w, h) in ((4, 4), (8, 4), (16, 16), (7, 5), (64, 64), (32, 8), (128, 128)):
        for bd in (8, 10):
            k = "%dx%d_bd%d" % (w, h, bd)
            dt = np.uint8 if bd == 8 else np.uint16
            src, prd = FP["s_src_" + k].astype(dt), FP["s_pred_" + k].astype(dt)
            exp = FP["sub_" + k]
            diff = np.full(exp.shape, 0x7777, np.int16)
            PX.subtract_block(h, w, diff, diff.shape[1], src, src.shape[1], prd, prd.shape[1],
                              highbd=bd > 8)
            np.testing.assert_array_equal(diff, exp, err_msg=k)
            assert PX.sse(src, src.shape[1], prd, prd.shape[1], w, h, highbd=bd > 8) == \
                FP["sse_" + k][0]
            assert PX.sum_squares_2d_i16(exp, exp.shape[1], w, h) == FP["sumsq_" + k][0]
            # the caller's *sum is accumulated into, as the reference does
            ss, sm = PX.sum_sse_2d_i16(exp, exp.shape[1], w, h, sum_in=7)
            assert [ss, sm - 7] == list(FP["sumsse_" + k])
            assert list(PX.get_blk_sse_sum(exp, exp.shape[1], w, h)) == list(FP["blksse_" + k])


def test_wht_vs_reference(L, PX):
    """Lossless Walsh-Hadamard: the shims, the batch kernels, and the
    lossless branches of av1_lowbd_fwd_txfm / av1_highbd_inv_txfm_add."""
    import torch
    import lavish_dsp.motion as M
    F = _load("fix_wht.npz")
    for blk, exp in zip(F["fwht_in"], F["fwht_out"]):
        np.testing.assert_array_equal(PX.fwht4x4(np.ascontiguousarray(blk), blk.shape[1]), exp)
        got = np.zeros(16, np.int32)
        p = L.TxfmParam(tx_type=0, tx_size=0, lossless=1, bd=8, is_hbd=0, tx_set_type=0, eob=16)
        L.av1_lowbd_fwd_txfm(np.ascontiguousarray(blk), got, blk.shape[1], p)
        np.testing.assert_array_equal(got, exp)
    jobs = np.zeros(len(F["fwht_in"]), PX.JOB_DTYPE)
    jobs["src_off"] = np.arange(len(jobs)) * 7
    jobs["aux_off"] = np.arange(len(jobs)) * 16
    plane = np.concatenate(list(F["fwht_in"]), axis=1)  # [4, 7 * k]
    out = PX.fwht4x4_batch(torch.from_numpy(np.ascontiguousarray(plane)).cuda(),
                           PX.jobs_tensor(jobs, "cuda"), 16 * len(jobs))
    np.testing.assert_array_equal(out.cpu().numpy().reshape(-1, 16), F["fwht_out"])
    for c, d, bd, e16, e1 in zip(F["iwht_in"], F["iwht_dst"], F["iwht_bd"], F["iwht16_out"],
                                 F["iwht1_out"]):
        for full, exp in ((True, e16), (False, e1)):
            dd = d.copy()
            PX.iwht4x4_add(c, dd, dd.shape[1], int(bd), full=full)
            np.testing.assert_array_equal(dd, exp)
            # the same through av1_highbd_inv_txfm_add's lossless TX_4X4 branch
            dd = d.copy()
            p = L.TxfmParam(tx_type=0, tx_size=0, lossless=1, bd=int(bd), is_hbd=1,
                            tx_set_type=0, eob=16 if full else 1)
            L.av1_inv_txfm_add(np.ascontiguousarray(c), dd, dd.shape[1], p)
            np.testing.assert_array_equal(dd, exp)
            # and the batch kernel (eob selects the form)
            j = np.zeros(1, L.INV_JOB_DTYPE)
            j["eob"] = 16 if full else 1
            dst = torch.from_numpy(d.view(np.int16).copy()).cuda()
            PX.iwht4x4_add_batch(torch.from_numpy(np.ascontiguousarray(c)).cuda(),
                                 M.to_device(j), dst, int(bd))
            np.testing.assert_array_equal(dst.cpu().numpy().view(np.uint16), exp)


def test_quick_txfm_vs_reference(L, FT, FP):
    """av1_quick_txfm: Hadamard sizes against the reference's aom_hadamard_*,
    DCT_DCT against its forward transform."""
    for n, s in ((4, 0), (8, 1), (16, 2), (32, 3)):
        res = FP["hres_%d_bd8" % n]
        got = np.zeros(n * n, np.int32)
        L.av1_quick_txfm(1, s, L.BitDepthInfo(8, 0), np.ascontiguousarray(res), res.shape[1], got)
        np.testing.assert_array_equal(got, FP["had_%d_bd8" % n])
        blk = FT["in_%d_0" % s][3]
        got = np.zeros(n * n, np.int32)
        L.av1_quick_txfm(0, s, L.BitDepthInfo(8, 0), np.ascontiguousarray(blk), n, got)
        np.testing.assert_array_equal(got, FT["out_%d_0" % s][3])
