"""The oracle (oracle/*.c) against fixtures produced by executing the
reference's own C function bodies (tests/golden/gen_fixtures.py through
tests/golden/cinterp.py): forward 2-D transforms of every valid (size, type),
av1_build_quantizer's tables, the fp / b quantizers (lowbd and highbd, every
log_scale), and the inverse 2-D transforms + add at bd 8 / 10 / 12 -- all
bit-exact.  This is what pins the 2-D composition (shifts, flips, rect
scaling, 64-point zero + repack), the quantizers and the inverse to the
reference rather than to a reading of it."""
import os

import numpy as np
import pytest

import _oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


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


def _pairs():
    return [(s, t) for s in range(19) for t in range(16) if O.type_valid(s, t)]


def test_fixture_coverage(FT, FI):
    """Every valid (tx_size, tx_type) -- 159 combinations -- is present."""
    p = _pairs()
    assert len(p) == 159
    for s, t in p:
        assert "out_%d_%d" % (s, t) in FT and "out_%d_%d" % (s, t) in FI


@pytest.mark.parametrize("s", range(19))
def test_fwd_txfm2d_vs_reference(FT, s):
    for t in range(16):
        if not O.type_valid(s, t):
            continue
        ins, outs, bds = FT["in_%d_%d" % (s, t)], FT["out_%d_%d" % (s, t)], FT["bd_%d_%d" % (s, t)]
        for blk, exp, bd in zip(ins, outs, bds):
            got = O.fwd_txfm2d(blk, t, s, int(bd))
            np.testing.assert_array_equal(got, exp, err_msg="size %d type %d bd %d" % (s, t, bd))


@pytest.mark.parametrize("bd", [8, 10, 12])
@pytest.mark.parametrize("sharp", [0, 3, -3])
def test_build_quantizer_vs_reference(bd, sharp):
    F = _load("fix_qparams.npz")
    for q in range(256):
        a = O.quant_arrays(O.build_quant(bd, q, sharp))
        for mine, ref in (("quant", "y_quant"), ("quant_shift", "y_quant_shift"),
                          ("zbin", "y_zbin"), ("round", "y_round"), ("quant_fp", "y_quant_fp"),
                          ("round_fp", "y_round_fp"), ("dequant", "y_dequant_QTX")):
            np.testing.assert_array_equal(a[mine], F["%s_bd%d_sh%d" % (ref, bd, sharp)][q, :2],
                                          err_msg="%s q %d" % (mine, q))


def quant_cases(FQ):
    for ci, (s, ls, hb, isb) in enumerate(FQ["cases"]):
        for bd in ((10,) if hb else (8,)):
            for q in (0, 32, 128, 255):
                yield ci, int(s), int(ls), bool(hb), bool(isb), bd, q


def test_quantizers_vs_reference(FQ):
    n_checked = 0
    for ci, s, ls, hb, isb, bd, q in quant_cases(FQ):
        key = "%d_%d_q%d" % (ci, bd, q)
        qq = O.build_quant(bd, q)
        n = O.max_eob(s)
        for k, c in enumerate(FQ["coeff_" + key]):
            qc, dq, eob = O.quantize("b" if isb else "fp", c, n, qq, O.scan(s, 0), O.iscan(s, 0),
                                     ls, highbd=hb)
            msg = "%s size %d q %d block %d" % (FQ["case_names"][ci], s, q, k)
            np.testing.assert_array_equal(qc, FQ["qcoeff_" + key][k], err_msg=msg)
            np.testing.assert_array_equal(dq, FQ["dqcoeff_" + key][k], err_msg=msg)
            assert eob == FQ["eob_" + key][k], msg
            n_checked += 1
    assert n_checked > 300


@pytest.mark.parametrize("s", range(19))
def test_inv_txfm2d_add_vs_reference(FI, s):
    W = O.TX_W[s]
    for t in range(16):
        if not O.type_valid(s, t):
            continue
        key = "%d_%d" % (s, t)
        for c, dst, exp, bd in zip(FI["in_" + key], FI["dst_" + key], FI["out_" + key],
                                   FI["bd_" + key]):
            got = O.inv_txfm2d_add(c, dst, t, s, int(bd))
            np.testing.assert_array_equal(got, exp, err_msg="size %d type %d bd %d" % (s, t, bd))
            assert W + 5 == dst.shape[1]


# ---------------------------------------------------------------- pixel --
BLOCK_SIZES = [(128, 128), (128, 64), (64, 128), (64, 64), (64, 32), (32, 64), (32, 32), (32, 16),
               (16, 32), (16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4), (4, 16),
               (16, 4), (8, 32), (32, 8), (16, 64), (64, 16)]
SUBPEL_OFFSETS = [(0, 0), (3, 0), (0, 5), (4, 4), (7, 2)]


@pytest.fixture(scope="module")
def FP():
    return _load("fix_pixel.npz")


def pixel_planes(FP, W, H, bd):
    k = "%dx%d_bd%d" % (W, H, bd)
    dt = np.uint8 if bd == 8 else np.uint16
    return k, FP["src_" + k].astype(dt), FP["ref_" + k].astype(dt)


@pytest.mark.parametrize("W,H", BLOCK_SIZES)
@pytest.mark.parametrize("bd", [8, 10])
def test_sad_variance_vs_reference(FP, W, H, bd):
    k, a, b = pixel_planes(FP, W, H, bd)
    hb = bd > 8
    ss, rs = a.shape[1], b.shape[1]
    assert O.sad(a, ss, b, rs, W, H, highbd=hb) == FP["sad_" + k][0]
    assert O.sad(a, ss, b, rs, W, H, highbd=hb, skip=True) == FP["sadskip_" + k][0]
    flat = b.reshape(-1)
    got4 = [O.sad(a, ss, flat[o:], rs, W, H, highbd=hb) for o in (0, 1, 3, W + 2)]
    np.testing.assert_array_equal(got4, FP["sadx4d_" + k])
    assert list(O.variance(a, ss, b, rs, W, H, bd, hb)) == list(FP["var_" + k])
    got = [O.sub_pixel_variance(a, ss, xo, yo, b, rs, W, H, bd, hb) for xo, yo in SUBPEL_OFFSETS]
    np.testing.assert_array_equal(np.array(got, np.int64), FP["subvar_" + k])


def test_hadamard_satd_vs_reference(FP):
    for n in (4, 8, 16, 32):
        for bd in (8, 10):
            k = "%d_bd%d" % (n, bd)
            if "had_" + k not in FP:
                continue
            res = FP["hres_" + k]
            got = O.hadamard(n, res, res.shape[1], highbd=bd > 8)
            np.testing.assert_array_equal(got, FP["had_" + k], err_msg=k)
            assert O.satd(got, n * n) == FP["satd_" + k][0]
            if "hadlp_" + k in FP:
                lp = O.hadamard_lp(n, res, res.shape[1])
                np.testing.assert_array_equal(lp, FP["hadlp_" + k], err_msg=k)
                assert O.satd_lp(lp, n * n) == FP["satdlp_" + k][0]


def test_block_error_vs_reference(FP):
    for n in (16, 64, 256, 1024, 4096):
        c, d = FP["be_c_%d" % n], FP["be_d_%d" % n]
        assert list(O.block_error(c, d, n)) == list(FP["be_%d" % n])
        for bd in (10, 12):
            assert list(O.block_error(c, d, n, bd)) == list(FP["behb_%d_bd%d" % (n, bd)])
        assert O.block_error_lp(FP["belp_c_%d" % n], FP["belp_d_%d" % n], n) == FP["belp_%d" % n][0]


def test_subtract_sse_sums_vs_reference(FP):
    for (w, h) in ((4, 4), (8, 4), (16, 16), (7, 5), (64, 64), (32, 8), (128, 128)):
        for bd in (8, 10):
            k = "%dx%d_bd%d" % (w, h, bd)
            dt = np.uint8 if bd == 8 else np.uint16
            src, prd = FP["s_src_" + k].astype(dt), FP["s_pred_" + k].astype(dt)
            exp = FP["sub_" + k]
            diff = np.full(exp.shape, 0x7777, np.int16)
            O.subtract_block(h, w, diff, diff.shape[1], src, src.shape[1], prd, prd.shape[1],
                             highbd=bd > 8)
            np.testing.assert_array_equal(diff, exp, err_msg=k)
            assert O.sse(src, src.shape[1], prd, prd.shape[1], w, h, highbd=bd > 8) == \
                FP["sse_" + k][0]
            assert O.sum_squares_2d_i16(exp, exp.shape[1], w, h) == FP["sumsq_" + k][0]
            sm, ss = O.sum_sse(exp, exp.shape[1], w, h)
            assert [ss, sm] == list(FP["sumsse_" + k])
            assert [sm, ss] == list(FP["blksse_" + k])


def test_wht_vs_reference():
    F = _load("fix_wht.npz")
    for blk, exp in zip(F["fwht_in"], F["fwht_out"]):
        np.testing.assert_array_equal(O.fwht4x4(blk, blk.shape[1]), exp)
    for c, d, bd, e16, e1 in zip(F["iwht_in"], F["iwht_dst"], F["iwht_bd"], F["iwht16_out"],
                                 F["iwht1_out"]):
        np.testing.assert_array_equal(O.iwht4x4_add(c, d, 16, int(bd)), e16)
        np.testing.assert_array_equal(O.iwht4x4_add(c, d, 1, int(bd)), e1)


# -------------------------------------------------------- motion search --
from _mcomp_fix import MS_METHODS, mcomp_groups  # noqa: E402


def test_full_pixel_search_vs_reference():
    """orc_full_pixel_search_batch against av1_full_pixel_search executed from
    the reference (DIAMOND / BIGDIA / FAST_BIGDIA, entropy / L1 / none mv
    cost, downsampled SAD with its quality recheck, cost lists)."""
    F = _load("fix_mcomp.npz")
    stride = F["src"].shape[1]
    n = 0
    for case, bw, bh, epb, spb, rec, rows, J in mcomp_groups(F):
        m, use_cl, ctype, skip, sp = (int(v) for v in case)
        res, cl = O.full_pixel_search_batch(
            F["src"], F["refs"], stride, bw, bh, rec, MS_METHODS[m], sp, ctype, spb, epb,
            F["mvjcost_lp"], F["mvcost_lp"], skip=bool(skip), cost_list=bool(use_cl))
        msg = "case %s %dx%d" % (list(case), bw, bh)
        np.testing.assert_array_equal(res["best_row"], rows[:, J["best_row"]], err_msg=msg)
        np.testing.assert_array_equal(res["best_col"], rows[:, J["best_col"]], err_msg=msg)
        np.testing.assert_array_equal(res["bestsme"], rows[:, J["var"]], err_msg=msg)
        if use_cl:
            np.testing.assert_array_equal(cl, rows[:, J["cl0"]:J["cl4"] + 1], err_msg=msg)
        n += len(rows)
    assert n == len(F["jobs"])


def test_full_pixel_search_methods2_vs_reference():
    """orc_full_pixel_search_batch against av1_full_pixel_search executed from
    the reference for the methods of tests/golden/fix_mcomp2.npz: NSTEP /
    NSTEP_8PT (diamond_search_sad over av1_init_motion_compensation_nstep's
    sites, mcomp.c:452-494), HEX / FAST_HEX and SQUARE (pattern_search,
    mcomp.c:553-653,1258-1289), mesh refinement off."""
    F = _load("fix_mcomp2.npz")
    methods = [str(m).lower() for m in F["methods"]]
    stride = F["src"].shape[1]
    n = 0
    seen = set()
    for case, bw, bh, epb, spb, rec, rows, J in mcomp_groups(F):
        m, use_cl, ctype, skip, sp = (int(v) for v in case)
        res, cl = O.full_pixel_search_batch(
            F["src"], F["refs"], stride, bw, bh, rec, methods[m], sp, ctype, spb, epb,
            F["mvjcost_lp"], F["mvcost_lp"], skip=bool(skip), cost_list=bool(use_cl))
        msg = "case %s %dx%d" % (list(case), bw, bh)
        np.testing.assert_array_equal(res["best_row"], rows[:, J["best_row"]], err_msg=msg)
        np.testing.assert_array_equal(res["best_col"], rows[:, J["best_col"]], err_msg=msg)
        np.testing.assert_array_equal(res["bestsme"], rows[:, J["var"]], err_msg=msg)
        if use_cl:
            np.testing.assert_array_equal(cl, rows[:, J["cl0"]:J["cl4"] + 1], err_msg=msg)
        n += len(rows)
        seen.add(methods[m])
    assert n == len(F["jobs"])
    assert seen == {"nstep", "nstep_8pt", "hex", "fast_hex", "square"}


def test_full_pixel_search_mesh_vs_reference():
    """orc_full_pixel_search_batch_ex against av1_full_pixel_search executed
    from the reference with the exhaustive mesh refinement
    (tests/golden/fix_mcomp3.npz; exhaustive_mesh_search / full_pixel_exhaustive,
    mcomp.c:1529-1680, the tail of av1_full_pixel_search :1818-1893): forced
    by force_mesh_thresh after NSTEP / NSTEP_8PT, run_mesh_search after
    DIAMOND / BIGDIA / FAST_HEX / SQUARE, pruning, the fine interval, the
    intraBC pattern set, the range growth and an illegal pattern."""
    F = _load("fix_mcomp3.npz")
    methods = [str(m).lower() for m in F["methods"]]
    stride = F["src"].shape[1]
    n = moved = 0
    for case, bw, bh, epb, spb, rec, rows, J in mcomp_groups(F):
        m, use_cl, ctype, skip, sp = (int(v) for v in case)
        mesh = O.OrcMeshParams.from_row(F["mesh"][int(rows[0, J["case"]])])
        res, cl = O.full_pixel_search_batch(
            F["src"], F["refs"], stride, bw, bh, rec, methods[m], sp, ctype, spb, epb,
            F["mvjcost_lp"], F["mvcost_lp"], skip=bool(skip), cost_list=bool(use_cl), mesh=mesh)
        plain, _ = O.full_pixel_search_batch(
            F["src"], F["refs"], stride, bw, bh, rec, methods[m], sp, ctype, spb, epb,
            F["mvjcost_lp"], F["mvcost_lp"], skip=bool(skip))
        msg = "case %s %dx%d" % (list(case), bw, bh)
        np.testing.assert_array_equal(res["best_row"], rows[:, J["best_row"]], err_msg=msg)
        np.testing.assert_array_equal(res["best_col"], rows[:, J["best_col"]], err_msg=msg)
        np.testing.assert_array_equal(res["bestsme"], rows[:, J["var"]], err_msg=msg)
        if use_cl:
            np.testing.assert_array_equal(cl, rows[:, J["cl0"]:J["cl4"] + 1], err_msg=msg)
        moved += int(((plain["best_row"] != res["best_row"]) |
                      (plain["best_col"] != res["best_col"])).sum())
        n += len(rows)
    assert n == len(F["jobs"])
    assert moved > 0  # the mesh changed some results


def test_subpel_search_vs_reference():
    """orc_subpel_search_batch against av1_find_best_sub_pixel_tree_pruned
    (_more) executed from the reference, from full-pel results with their
    cost lists (tests/golden/fix_subpel.npz)."""
    from _mcomp_fix import subpel_groups
    F, mc = _load("fix_subpel.npz"), _load("fix_mcomp.npz")
    stride = mc["src"].shape[1]
    n = 0
    for case, bw, bh, epb, rec, cls, rows, J in subpel_groups(F, mc):
        meth, hp, fstop, iters, ctype, use_cl = (int(v) for v in case)
        tab = "hp" if hp else "lp"
        res = O.subpel_search_batch(mc["src"], mc["refs"], stride, bw, bh, rec, meth, fstop,
                                    bool(hp), iters, ctype, epb, mc["mvjcost_" + tab],
                                    mc["mvcost_" + tab], cls if use_cl else None)
        msg = "case %s %dx%d" % (list(case), bw, bh)
        for f in ("best_row", "best_col", "besterr", "distortion", "sse"):
            np.testing.assert_array_equal(res[f].astype(np.int64), rows[:, J[f]],
                                          err_msg=msg + " " + f)
        n += len(rows)
    assert n == len(F["jobs"])


@pytest.mark.parametrize("n", [8, 16, 32])
@pytest.mark.parametrize("bd", [8, 10, 12])
def test_tpl_block_vs_reference(n, bd):
    """orc_tpl_block_batch (one prediction) against tpl_get_satd_cost +
    txfm_quant_rdcost executed from the reference (tests/golden/fix_tpl.npz):
    satd, rate, recon_error, sse and the reconstruction."""
    F = _load("fix_tpl.npz")
    k = "%d_bd%d" % (n, bd)
    dt = np.uint8 if bd == 8 else np.uint16
    for i, (rec, q) in enumerate(zip(F["rec_" + k], F["q_" + k])):
        src = F["src_" + k][i].astype(dt)
        pred = F["pred_" + k][i].astype(dt)[None]
        got, recon, costs = O.tpl_block_batch(src, pred, n, bd, int(q))
        msg = "%s block %d q %d" % (k, i, q)
        assert [got["inter_cost"][0], got["rate_cost"][0], got["recon_error"][0],
                got["sse"][0]] == list(rec), msg
        assert costs[0, 0] == rec[0], msg
        np.testing.assert_array_equal(recon, F["recon_" + k][i].astype(dt), err_msg=msg)


def test_av1_quant_selection_vs_reference():
    """orc_av1_quant_block against skip_trellis_opt_based_on_satd + av1_quant
    executed from the reference (tests/golden/fix_qfacade.npz): the quantizer
    chosen, use_optimize_b, qcoeff, dqcoeff and eob."""
    F = _load("fix_qfacade.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    kinds = set()
    for r in F["rows"]:
        g = lambda k: int(r[J[k]])
        n = O.max_eob(g("tx_size"))
        i = g("index")
        flags, qc, dq, eob = O.av1_quant_block(F["coeff"][i][:n], g("tx_size"), g("tx_type"),
                                               g("bd"), g("qindex"), g("mode"), g("skip_trellis"),
                                               g("threshold"), g("qstep"), g("dc_only"))
        msg = str({k: g(k) for k in J})
        assert flags == g("flags"), msg
        assert eob == g("eob"), msg
        np.testing.assert_array_equal(qc, F["qcoeff"][i][:n], err_msg=msg)
        np.testing.assert_array_equal(dq, F["dqcoeff"][i][:n], err_msg=msg)
        kinds.add(flags)
    assert {0 << 1 | 1, 1 << 1, 2 << 1} <= kinds  # FP+trellis, B, DC all exercised


def test_cost_coeffs_txb_matches_reference():
    """orc_cost_coeffs_txb against av1_cost_coeffs_txb and
    av1_cost_coeffs_txb_laplacian executed from the reference
    (tests/golden/fix_costcoeffs.npz): every tx size, tx types of the 2D /
    horizontal / vertical classes, luma and chroma, eob 0 / 1 / 2 / random /
    max, Golomb-range levels, random cost tables."""
    F = _load("fix_costcoeffs.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    blob = O.coeff_costs_blob(F["coeff_costs"], F["eob_costs"])
    classes = set()
    for r in F["rows"]:
        g = lambda k: int(r[J[k]])
        n = O.max_eob(g("tx_size"))
        q = F["qcoeff"][g("index")][:n]
        args = (blob, q, g("eob"), g("plane"), g("tx_size"), g("tx_type"), g("txb_skip_ctx"),
                g("dc_sign_ctx"), g("tx_type_cost"))
        msg = str({k: g(k) for k in J})
        assert O.cost_coeffs_txb(*args) == g("rate"), msg
        assert O.cost_coeffs_txb(*args, laplacian=True) == g("rate_laplacian"), msg
        classes.add(0 if g("tx_type") < 10 else 1 + (g("tx_type") & 1))
    assert classes == {0, 1, 2}
    assert (F["rows"][:, J["tx_size"]] == np.arange(19)[:, None]).any(axis=1).all()


def test_rdo_rate_oracle_records_are_cost_coeffs():
    """orc_rdo_plane_rate's record rate is orc_cost_coeffs_txb (pinned above)
    of the winning type's qcoeff / eob, and its rd cost is RDCOST of it."""
    import _c4ref
    bd = 10
    src, pred = _c4ref.planes(bd, 3, 128, 64)
    rng = np.random.default_rng(0)
    blob = rng.integers(30, 4000, 10 * O.CC_COEFF_COST + 14 * O.CC_EOB_COST).astype(np.int32)
    ttc = rng.integers(0, 3000, 16).astype(np.int32)
    q = O.build_quant(bd, 128)
    for s, tmask in ((0, 0xFFFF), (2, 0xFFFF), (7, 0xFFFF), (3, 0x201)):
        nb = (128 // O.TX_W[s]) * (64 // O.TX_H[s])
        ctx = np.stack([rng.integers(0, 13, nb), rng.integers(0, 3, nb)], 1).astype(np.int32)
        rec, qc, _ = O.rdo_plane_rate(src, pred, s, tmask, bd, q, 1500, blob, ctx, ttc, threads=4)
        for b in range(nb):
            t = int(rec["best_type"][b])
            r = O.cost_coeffs_txb(blob, qc[b], int(rec["eob"][b]), 0, s, t, int(ctx[b, 0]),
                                  int(ctx[b, 1]), int(ttc[t]))
            assert r == rec["rate"][b]
            assert rec["rdcost"][b] == ((r * 1500 + 256) >> 9) + int(rec["dist"][b]) * 128


def test_optimize_b_matches_reference():
    """orc_optimize_b against av1_optimize_b executed from the reference
    (tests/golden/fix_trellis.npz) on av1_quant's FP output: rate, eob,
    txb_entropy_ctx, qcoeff and dqcoeff, every row."""
    F = _load("fix_trellis.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    blob = O.coeff_costs_blob(F["coeff_costs"], F["eob_costs"])
    changed = skipped = 0
    for r in F["rows"]:
        g = lambda k: int(r[J[k]])
        n = O.max_eob(g("tx_size"))
        i = g("index")
        q = O.quant_arrays(O.build_quant(g("bd"), g("qindex")))
        dqv = q["dequant"]
        e, rate, ec, qc, dq = O.optimize_b(
            blob, F["coeff"][i][:n], F["qcoeff_in"][i][:n], F["dqcoeff_in"][i][:n],
            g("eob_in"), g("plane"), g("tx_size"), g("tx_type"), g("bd"), g("is_inter"),
            g("rdmult"), g("sharpness"), dqv, g("txb_skip_ctx"), g("dc_sign_ctx"),
            g("tx_type_cost"))
        msg = str({k: g(k) for k in J})
        assert (e, rate, ec) == (g("eob"), g("rate"), g("entropy_ctx")), msg
        np.testing.assert_array_equal(qc, F["qcoeff"][i][:n], err_msg=msg)
        np.testing.assert_array_equal(dq, F["dqcoeff"][i][:n], err_msg=msg)
        changed += int((qc != F["qcoeff_in"][i][:n]).any())
        skipped += int(g("eob") == 0 and g("eob_in") > 0)
    assert changed > 100 and skipped > 10


def _warp_case(F, r, J):
    """Inputs of one fix_warp row as the oracle's arguments."""
    g = lambda k: int(r[J[k]])
    W, H, RS, PS, DS = (int(v) for v in F["geom"])
    bd = g("bd")
    hb = bd > 8
    ref = F["refs"][g("ref_index")].astype(np.uint16 if hb else np.uint8)
    mat = [g("m%d" % i) for i in range(6)]
    cp = dict(do_average=int(g("mode") >= 2), round_0=g("round_0"), round_1=g("round_1"),
              is_compound=int(g("mode") > 0), use_dist_wtd_comp_avg=int(g("mode") == 3),
              fwd_offset=g("fwd_offset"), bck_offset=g("bck_offset"))
    prm = tuple(g(k) for k in ("alpha", "beta", "gamma", "delta"))
    return g, W, H, RS, PS, DS, bd, hb, ref, mat, cp, prm


def test_warp_affine_matches_reference():
    """orc_warp_affine against av1_warp_affine_c / av1_highbd_warp_affine_c
    executed from the reference (tests/golden/fix_warp.npz): the prediction
    and the compound buffer of every row (bd 8/10/12, subsampling, cropped
    shapes, single / compound / average / distance-weighted)."""
    F = _load("fix_warp.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    changed = 0
    for k, r in enumerate(F["rows"]):
        g, W, H, RS, PS, DS, bd, hb, ref, mat, cp, prm = _warp_case(F, r, J)
        pred = F["pred_in"][k].astype(np.uint16 if hb else np.uint8).copy()
        dst = F["dst_in"][k].copy()
        O.warp_affine(mat, ref, W, H, RS, pred, g("p_col"), g("p_row"), g("p_width"),
                      g("p_height"), PS, g("ss_x"), g("ss_y"), bd, int(hb), cp, dst, DS, prm)
        np.testing.assert_array_equal(pred.astype(np.uint16), F["pred"][k], err_msg=str(k))
        np.testing.assert_array_equal(dst, F["dst"][k], err_msg=str(k))
        changed += int((F["pred"][k] != F["pred_in"][k]).any() or (F["dst"][k] != F["dst_in"][k]).any())
    assert changed == len(F["rows"])


def test_get_shear_params_matches_reference():
    F = _load("fix_warp.npz")
    for row in F["shear"]:
        ok, prm = O.get_shear_params(row[1:7])
        assert (ok,) + prm == tuple(int(v) for v in (row[0], *row[7:11])), row


def test_dist_wtd_convolve_matches_reference():
    """orc_dist_wtd_convolve against av1_dist_wtd_convolve_{2d_copy,x,y,2d}_c
    and the highbd forms executed from the reference (fix_compound.npz): the
    CONV_BUF and the averaged prediction of every row."""
    F = _load("fix_compound.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    SS, DS, CS, org = (int(v) for v in F["geom"])
    for k, r in enumerate(F["rows"]):
        g = lambda n: int(r[J[n]])
        bd, w, h = g("bd"), g("w"), g("h")
        hb = bd > 8
        src = np.ascontiguousarray(F["src"][g("src_index")].astype(np.uint16 if hb else np.uint8))
        dst = F["dst_in"][k].astype(np.uint16 if hb else np.uint8).copy()
        conv = F["conv_in"][k].copy()
        fx = O.interp_kernel(g("filter_x"), w, g("subpel_x"))
        fy = O.interp_kernel(g("filter_y"), h, g("subpel_y"))
        cp = dict(do_average=int(g("mode") > 0), round_0=g("round_0"), round_1=g("round_1"),
                  is_compound=1, use_dist_wtd_comp_avg=int(g("mode") == 2),
                  fwd_offset=g("fwd_offset"), bck_offset=g("bck_offset"))
        O.dist_wtd_convolve(g("path"), src, SS, dst, DS, w, h, fx, fy, cp, conv, CS, bd, int(hb),
                            src_off=org * SS + org)
        np.testing.assert_array_equal(conv, F["conv"][k], err_msg=str(k))
        np.testing.assert_array_equal(dst.astype(np.uint16), F["dst"][k], err_msg=str(k))


def scale_row(F, k):
    """(getter, conv-param dict) of fix_scale.npz row k."""
    J = {n: i for i, n in enumerate(F["row_fields"])}
    r = F["rows"][k]
    g = lambda n: int(r[J[n]])
    m = g("mode")
    cp = dict(do_average=int(m > 1), round_0=g("round_0"), round_1=g("round_1"),
              is_compound=int(m > 0), use_dist_wtd_comp_avg=int(m == 3),
              fwd_offset=g("fwd_offset"), bck_offset=g("bck_offset"))
    return g, cp


def test_convolve_2d_scale_matches_reference():
    """orc_convolve_2d_scale against av1_convolve_2d_scale_c and
    av1_highbd_convolve_2d_scale_c executed from the reference
    (fix_scale.npz): 1/1024-pel steps 512 .. 2048 and start phases, the five
    filters incl. 12-tap MULTITAP_SHARP2, bd 8 (both forms) / 10 / 12, single
    prediction, compound first pass, plain and distance-weighted average."""
    F = _load("fix_scale.npz")
    SW, DS, CS, org = (int(v) for v in F["geom"])
    modes = set()
    for k in range(len(F["rows"])):
        g, cp = scale_row(F, k)
        hb, bd, w, h = g("highbd"), g("bd"), g("w"), g("h")
        pdt = np.uint16 if hb else np.uint8
        src = np.ascontiguousarray(F["src"][g("src_index")].astype(pdt))
        dst = F["dst_in"][k].astype(pdt).copy()
        conv = F["conv_in"][k].copy()
        fx, fy = O.interp_table(g("filter_x"), w), O.interp_table(g("filter_y"), h)
        assert fx.shape[1] == g("taps_x") and fy.shape[1] == g("taps_y")
        O.convolve_2d_scale(src, SW, dst, DS, w, h, fx, fy, g("subpel_x_qn"), g("x_step_qn"),
                            g("subpel_y_qn"), g("y_step_qn"), cp, conv, CS, bd, hb, src_off=org)
        np.testing.assert_array_equal(conv, F["conv"][k], err_msg=str(k))
        np.testing.assert_array_equal(dst.astype(np.uint16), F["dst"][k], err_msg=str(k))
        modes.add(g("mode"))
    assert modes == {0, 1, 2, 3}


def test_convolve_sr_matches_reference():
    """orc convolve_block against av1_convolve_{x,y,2d}_sr_c and the highbd
    forms executed from the reference (fix_convolve.npz): bd 8/10/12, 2x2 ..
    128x128, the five filters incl. 12-tap MULTITAP_SHARP2."""
    F = _load("fix_convolve.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    oy, ox, pad = (int(v) for v in F["origin"])
    paths = set()
    for r in F["rows"]:
        g = lambda k: int(r[J[k]])
        w, h, bd = g("w"), g("h"), g("bd")
        SS = w + pad
        src = F["src"][g("src_off"):g("src_off") + (h + pad) * SS].reshape(h + pad, SS)
        src = np.ascontiguousarray(src.astype(np.uint8 if bd == 8 else np.uint16))
        fx = O.interp_kernel(g("filter_x"), w, g("subpel_x"))
        fy = O.interp_kernel(g("filter_y"), h, g("subpel_y"))
        got = O.convolve_block(src, oy * SS + ox, SS, w, h, g("path"), fx, fy, g("round_0"),
                               g("round_1"), bd)
        exp = F["dst"][g("dst_off"):g("dst_off") + w * h].reshape(h, w)
        np.testing.assert_array_equal(got.astype(np.int64), exp, err_msg=str(r))
        paths.add((g("path"), g("filter_x") == 4 or g("filter_y") == 4))
    assert len(paths) == 6  # x / y / 2-D, with and without the 12-tap kernel


def test_dist_wtd_convolve_12tap_matches_reference():
    """orc_dist_wtd_convolve against the 12-tap (MULTITAP_SHARP2) compound
    convolutions executed from the reference (fix_compound12.npz)."""
    F = _load("fix_compound12.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    oy, ox, pad = (int(v) for v in F["origin"])
    for r in F["rows"]:
        g = lambda n: int(r[J[n]])
        bd, w, h = g("bd"), g("w"), g("h")
        hb = bd > 8
        SS = w + pad
        src = F["src"][g("src_off"):g("src_off") + (h + pad) * SS]
        src = np.ascontiguousarray(src.astype(np.uint16 if hb else np.uint8))
        d0 = g("dst_off")
        dst = F["dst_in"][d0:d0 + w * h].astype(np.uint16 if hb else np.uint8).copy()
        conv = F["conv_in"][d0:d0 + w * h].copy()
        fx = O.interp_kernel(4, w, g("subpel_x"))
        fy = O.interp_kernel(4, h, g("subpel_y"))
        cp = dict(do_average=int(g("mode") > 0), round_0=g("round_0"), round_1=g("round_1"),
                  is_compound=1, use_dist_wtd_comp_avg=int(g("mode") == 2),
                  fwd_offset=g("fwd_offset"), bck_offset=g("bck_offset"))
        O.dist_wtd_convolve(g("path"), src, SS, dst, w, w, h, fx, fy, cp, conv, w, bd, int(hb),
                            src_off=oy * SS + ox)
        np.testing.assert_array_equal(conv, F["conv"][d0:d0 + w * h], err_msg=str(r))
        np.testing.assert_array_equal(dst.astype(np.uint16), F["dst"][d0:d0 + w * h],
                                      err_msg=str(r))


def _features(F, k):
    """Expected prune_tx_2D feature vectors of fix_txfeat row k."""
    s, w, h = (int(v) for v in F["rows"][k][:3])
    f = F["features"][k].view(np.float32)
    nh = w if w <= 8 else w // 2
    nv = h if h <= 8 else h // 2
    return (np.concatenate([f[:nh - 1], f[32:33]]), np.concatenate([f[16:16 + nv - 1], f[33:34]]))


def test_tx_prune_features_match_reference():
    """orc_tx_prune_features / orc_horver_correlation_full against
    get_energy_distribution_finer + av1_get_horver_correlation_full_c executed
    from the reference (fix_txfeat.npz): float bit patterns, 0 ULP."""
    F = _load("fix_txfeat.npz")
    for k, (s, w, h, kind, off) in enumerate(F["rows"]):
        blk = F["blocks"][off:off + w * h].reshape(h, w)
        hf, vf = O.tx_prune_features(blk, w, h)
        eh, ev = _features(F, k)
        np.testing.assert_array_equal(hf[0][:len(eh)].view(np.int32), eh.view(np.int32))
        np.testing.assert_array_equal(vf[0][:len(ev)].view(np.int32), ev.view(np.int32))
    for k, (w, h, kind, off) in enumerate(F["horver_rows"]):
        blk = F["horver_blocks"][off:off + w * h].reshape(h, w)
        got = np.array(O.horver_full(blk, w, w, h), np.float32).view(np.int32)
        np.testing.assert_array_equal(got, F["horver"][k])


def test_optimize_b_sharpness2_matches_reference():
    """orc_optimize_b against av1_optimize_b executed from the reference at
    quant_sharpness 2 (fix_trellis_s2.npz); the walk changes a good share of
    the blocks there."""
    F = _load("fix_trellis_s2.npz")
    J = {n: i for i, n in enumerate(F["row_fields"])}
    blob = O.coeff_costs_blob(F["coeff_costs"], F["eob_costs"])
    changed = 0
    for r in F["rows"]:
        g = lambda k: int(r[J[k]])
        assert g("sharpness") == 2
        n = O.max_eob(g("tx_size"))
        i = g("index")
        dqv = O.quant_arrays(O.build_quant(g("bd"), g("qindex")))["dequant"]
        e, rate, ec, qc, dq = O.optimize_b(
            blob, F["coeff"][i][:n], F["qcoeff_in"][i][:n], F["dqcoeff_in"][i][:n],
            g("eob_in"), g("plane"), g("tx_size"), g("tx_type"), g("bd"), g("is_inter"),
            g("rdmult"), g("sharpness"), dqv, g("txb_skip_ctx"), g("dc_sign_ctx"),
            g("tx_type_cost"))
        msg = str({k: g(k) for k in J})
        assert (e, rate, ec) == (g("eob"), g("rate"), g("entropy_ctx")), msg
        np.testing.assert_array_equal(qc, F["qcoeff"][i][:n], err_msg=msg)
        np.testing.assert_array_equal(dq, F["dqcoeff"][i][:n], err_msg=msg)
        changed += int((qc != F["qcoeff_in"][i][:n]).any())
    assert changed > len(F["rows"]) // 4, changed


SEARCH_METHOD_NAMES = {0: "diamond", 5: "bigdia", 8: "fast_diamond", 9: "fast_bigdia",
                       10: "vfast_diamond"}


def tplmv_case_inputs(F, ci):
    """Jobs and search settings of fix_tplmv case ci (the fixture's frame)."""
    import lavish_dsp.motion as M
    W, H, border, mvb, nref = (int(v) for v in F["geom"])
    src = F["src"]
    jobs = M.frame_jobs(W, H, src.shape[1], border, src.size, 16, 16, nref, mv_border=mvb)
    meth, rfs, skip, prune, alike = (int(v) for v in F["cases"][ci])
    return jobs, (SEARCH_METHOD_NAMES[meth], rfs, bool(skip), prune, alike), (W // 16, H // 16,
                                                                            nref)


def test_tpl_motion_search_matches_reference():
    """orc_tpl_motion_search against mode_estimation's start-mv selection and
    per-centre motion_estimation executed from the reference text
    (fix_tplmv.npz: every block of a 96x64 frame x 2 references, four tpl_sf
    settings): the tpl mv of every block, the mv limits, and the winning centre
    is one of the reference's (pruned) centres."""
    import lavish_dsp.tpl as T
    F = _load("fix_tplmv.npz")
    fld = {n: i for i, n in enumerate(F["rec_fields"])}
    recs = F["recs"]
    qindex, rdmult, spb, epb, allow_hp = (int(v) for v in F["params"])
    for ci in range(len(F["cases"])):
        jobs, (meth, sp, skip, prune, alike), (cols, rows, nref) = tplmv_case_inputs(F, ci)
        rc = recs[recs[:, fld["case"]] == ci]
        assert len(rc) == len(jobs)
        for f in ("col_min", "col_max", "row_min", "row_max"):
            np.testing.assert_array_equal(jobs[f], rc[:, fld[f]], err_msg=f)
        mvs, fp, cl, cen = O.tpl_motion_search(
            F["src"].reshape(-1), F["refs"].reshape(-1), F["src"].shape[1], jobs, cols, rows,
            nref, meth, sp, skip, prune, alike, spb, epb, F["mvjcost_hp"], F["mvcost_hp"], 0)
        r, c = T.unpack_mv(mvs)
        msg = "case %d" % ci
        np.testing.assert_array_equal(r, rc[:, fld["mv_row"]], err_msg=msg)
        np.testing.assert_array_equal(c, rc[:, fld["mv_col"]], err_msg=msg)
        cr, cc = T.unpack_mv(cen)
        for i in range(len(rc)):
            n = int(rc[i, fld["n_centers"]])
            opts = {(int(rc[i, fld["c%d_row" % q]]), int(rc[i, fld["c%d_col" % q]]))
                    for q in range(n)}
            assert (int(cr[i]), int(cc[i])) in opts, (msg, i)
        # the neighbours matter in this content: some searches start off zero
        assert np.count_nonzero(cen) > 0, msg


def test_rd_select_matches_reference():
    """The C4 composition's cost and type choice (oracle_rdo.c rdcost +
    orc_rd_select, the two lines rdo_rows runs per candidate type) against
    RDCOST and search_tx_type's best-type update executed from the reference
    text (fix_rdselect.npz: 240 lists of 16 candidates, rdmult 1 .. 2^20,
    rates < 2^24, dists < 2^44, planted equal costs): every cost and the
    winning index (the first of strictly lowest cost) agree."""
    F = _load("fix_rdselect.npz")
    ties = 0
    for i in range(len(F["rdmult"])):
        best, rds = O.rd_select(F["rdmult"][i], F["rates"][i], F["dists"][i])
        np.testing.assert_array_equal(rds, F["rds"][i], err_msg="list %d" % i)
        assert best == F["best"][i] and rds[best] == F["best_rd"][i], i
        ties += int(np.count_nonzero(rds == rds[best]) > 1)
    assert ties > 0  # the tie rule was exercised


def test_tpl_motion_search_third_pass_matches_reference():
    """The same with the third-pass candidate (tpl_model.c:687-703): the
    reference ran with cpi->third_pass_ctx set and its CONFIG_THREE_PASS
    thirdpass.c mapping each block to a second-pass mode info
    (fix_tplmv3.npz); the oracle takes each block's adjusted mv as recorded
    there (INVALID_MV where the mode info has no such reference)."""
    import lavish_dsp.tpl as T
    F = _load("fix_tplmv3.npz")
    fld = {n: i for i, n in enumerate(F["rec_fields"])}
    recs = F["recs"]
    qindex, rdmult, spb, epb, allow_hp = (int(v) for v in F["params"])
    valid = 0
    for ci in range(len(F["cases"])):
        jobs, (meth, sp, skip, prune, alike), (cols, rows, nref) = tplmv_case_inputs(F, ci)
        rc = recs[recs[:, fld["case"]] == ci]
        third = np.ascontiguousarray(F["third"][ci], dtype=np.int32)
        valid += int(np.count_nonzero(third.view(np.uint32) != 0x80008000))
        mvs, fp, cl, cen = O.tpl_motion_search(
            F["src"].reshape(-1), F["refs"].reshape(-1), F["src"].shape[1], jobs, cols, rows,
            nref, meth, sp, skip, prune, alike, spb, epb, F["mvjcost_hp"], F["mvcost_hp"], 0,
            third)
        r, c = T.unpack_mv(mvs)
        msg = "case %d" % ci
        np.testing.assert_array_equal(r, rc[:, fld["mv_row"]], err_msg=msg)
        np.testing.assert_array_equal(c, rc[:, fld["mv_col"]], err_msg=msg)
        cr, cc = T.unpack_mv(cen)
        for i in range(len(rc)):
            n = int(rc[i, fld["n_centers"]])
            opts = {(int(rc[i, fld["c%d_row" % q]]), int(rc[i, fld["c%d_col" % q]]))
                    for q in range(n)}
            assert (int(cr[i]), int(cc[i])) in opts, (msg, i)
    assert valid > 0  # some blocks have a third-pass mv for their reference


def test_subpel_tree_upsampled_vs_reference():
    """orc_subpel_search_batch_ex (SUBPEL_TREE) against av1_find_best_sub_pixel_tree
    executed from the reference with subpel_search_type USE_2_TAPS /
    USE_4_TAPS / USE_8_TAPS -- check_better through upsampled_pref_error and
    aom_upsampled_pred_c (tests/golden/fix_subpel_up.npz)."""
    from _mcomp_fix import subpel_groups
    F, mc = _load("fix_subpel_up.npz"), _load("fix_mcomp.npz")
    stride = mc["src"].shape[1]
    n = 0
    moved = 0
    for case, bw, bh, epb, rec, _, rows, J in subpel_groups(F, mc):
        stype, hp, fstop, iters, ctype = (int(v) for v in case)
        tab = "hp" if hp else "lp"
        res = O.subpel_search_batch(mc["src"], mc["refs"], stride, bw, bh, rec, 0, fstop,
                                    bool(hp), iters, ctype, epb, mc["mvjcost_" + tab],
                                    mc["mvcost_" + tab], None, search_type=stype)
        msg = "case %s %dx%d" % (list(case), bw, bh)
        for f in ("best_row", "best_col", "besterr", "distortion", "sse"):
            np.testing.assert_array_equal(res[f].astype(np.int64), rows[:, J[f]],
                                          err_msg=msg + " " + f)
        moved += int(np.count_nonzero((res["best_row"] & 7) | (res["best_col"] & 7)))
        n += len(rows)
    assert n == len(F["jobs"])
    assert moved > n // 2  # most searches end on a sub-pel position
