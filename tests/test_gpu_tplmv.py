"""GPU parity of the TPL motion search with the reference's start-mv
candidates (lavish_tpl_motion_search, a device wavefront over block rows)
against the oracle restatement of mode_estimation's per-reference loop
(oracle/oracle_tpl.c: orc_tpl_motion_search; av1/encoder/tpl_model.c:632-743),
bit-exact: tpl mvs, the winning full-pel search's result and cost list, and
the winning centre.  The oracle's selection logic is pinned to the reference
by tests/golden/fix_tplmv.npz (test_oracle_fixtures.py) and the chained GPU
frame leg below by the same fixture."""
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def T():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp.tpl as T
    return T


CASES = [  # (method, step_param, downsampled sad, prune_starting_mv, skip_alike, third pass)
    ("fast_bigdia", 6, False, 3, 2, False),   # cpu-used >= 5 (speed_features.c:1212-1216)
    ("fast_bigdia", 6, True, 2, 2, False),
    ("diamond", 6, False, 2, 2, True),        # speed 4 search method, with third-pass mvs
    ("bigdia", 0, False, 1, 1, False),
    ("fast_bigdia", 9, True, 0, 0, True),     # no pruning: every distinct centre searched
]


def _run_case(T, W, H, R, border, case, seed, qindex=100, rdmult=1800):
    import torch
    import lavish_dsp.motion as M
    method, sp, skip, prune, alike, third = case
    import lavish_dsp.synth as synth
    src, refs = synth.tpl_motion_planes(W, H, R, border, seed)
    st = src.shape[1]
    cols, rows = W // 16, H // 16
    jobs = M.frame_jobs(W, H, st, border, src.size, 16, 16, R, mv_border=32)
    allow_hp = qindex < 128
    mvj, mvc = M.default_mv_cost_tables(allow_hp)
    spb, epb = M.sad_per_bit(qindex), M.error_per_bit(rdmult)
    tp = None
    if third:
        rng = np.random.default_rng(seed + 5)
        tr = rng.integers(-200, 201, size=len(jobs))
        tc = rng.integers(-200, 201, size=len(jobs))
        tp = T.pack_mv(tr, tc)
        tp[rng.random(len(jobs)) < 0.3] = T.INVALID_MV
    emv, efp, ecl, ecen = O.tpl_motion_search(src.reshape(-1), refs.reshape(-1), st, jobs, cols,
                                              rows, R, method, sp, skip, prune, alike, spb, epb,
                                              mvj, mvc, 0, tp)
    costs = M.MvCosts(mvj, mvc, device="cuda")
    cost = costs.cost_params(spb, epb, M.MV_COST_ENTROPY)
    out = T.tpl_motion_search(torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda(),
                              M.to_device(jobs), cols, rows, R, cost, method, sp, skip, prune,
                              alike, torch.from_numpy(tp).cuda() if tp is not None else None)
    torch.cuda.synchronize()
    assert T.tpl_motion_failures(out) == 0
    gfp = M.results_numpy(out["fp"])
    msg = "case %r" % (case,)
    np.testing.assert_array_equal(out["mvs"].cpu().numpy(), emv, err_msg=msg)
    np.testing.assert_array_equal(out["centers"].cpu().numpy(), ecen, err_msg=msg)
    for f in ("best_row", "best_col", "bestsme", "steps"):
        np.testing.assert_array_equal(gfp[f], efp[f], err_msg=msg + " " + f)
    np.testing.assert_array_equal(out["cl"].cpu().numpy(), ecl, err_msg=msg)
    return emv, ecen


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_tpl_motion_search_vs_oracle(T, ci):
    emv, ecen = _run_case(T, 224, 160, 3, 160, CASES[ci], seed=31 + ci)
    # the neighbour centres matter: some winning centres are not the zero mv
    assert np.count_nonzero(ecen) > 0


def test_tpl_motion_search_1080p(T):
    """The bench configuration (1080p x 7 references, cpu-used 6 tpl_sf) in
    full: every block of every reference bit-exact."""
    _run_case(T, 1920, 1072, 7, 288, CASES[0], seed=5)


def test_tpl_motion_search_rejects(T):
    import ctypes
    import torch
    import lavish_dsp.motion as M
    src = torch.zeros((64, 64), dtype=torch.uint8, device="cuda")
    jobs = M.to_device(M.frame_jobs(16, 16, 64, 24, 64 * 64, 16, 16, 1))
    cost = M.l1_cost_params(M.MV_COST_NONE)
    buf = torch.zeros(64, dtype=torch.int32, device="cuda")

    def rc(method, force_stop, prune=3):
        p = T.TplMvParams(method, 0, 0, prune, 2, force_stop)
        return T._lib.lavish_tpl_motion_search(
            src.data_ptr(), 64, src.data_ptr(), 64, jobs.data_ptr(), 1, 1, 1, ctypes.byref(p),
            ctypes.byref(cost), None, buf.data_ptr(), buf.data_ptr(), None, None,
            buf.data_ptr(), None)
    assert rc(1, M.FULL_PEL) == -4          # NSTEP is not built
    assert rc(9, M.HALF_PEL) == -6          # only subpel_force_stop FULL_PEL
    assert rc(9, M.FULL_PEL, prune=4) == -1


def test_tpl_motion_search_vs_reference(T):
    """lavish_tpl_motion_search against mode_estimation executed from the
    reference text (tests/golden/fix_tplmv.npz), no oracle in the loop: the
    tpl mv of every block of every case."""
    import torch
    import lavish_dsp.motion as M
    from test_oracle_fixtures import _load, tplmv_case_inputs
    F = _load("fix_tplmv.npz")
    fld = {n: i for i, n in enumerate(F["rec_fields"])}
    qindex, rdmult, spb, epb, allow_hp = (int(v) for v in F["params"])
    costs = M.MvCosts(F["mvjcost_hp"], F["mvcost_hp"], device="cuda")
    cost = costs.cost_params(spb, epb, M.MV_COST_ENTROPY)
    src = torch.from_numpy(F["src"]).cuda()
    refs = torch.from_numpy(F["refs"]).cuda()
    for ci in range(len(F["cases"])):
        jobs, (meth, sp, skip, prune, alike), (cols, rows, nref) = tplmv_case_inputs(F, ci)
        out = T.tpl_motion_search(src, refs, M.to_device(jobs), cols, rows, nref, cost, meth, sp,
                                  skip, prune, alike)
        torch.cuda.synchronize()
        assert T.tpl_motion_failures(out) == 0
        r, c = T.unpack_mv(out["mvs"].cpu().numpy())
        rc = F["recs"][F["recs"][:, fld["case"]] == ci]
        np.testing.assert_array_equal(r, rc[:, fld["mv_row"]], err_msg="case %d" % ci)
        np.testing.assert_array_equal(c, rc[:, fld["mv_col"]], err_msg="case %d" % ci)


def test_tpl_motion_search_third_pass_vs_reference(T):
    """With the third-pass candidate: lavish_tpl_motion_search fed each
    block's adjusted third-pass mv against mode_estimation executed from the
    reference with a third_pass_ctx (tests/golden/fix_tplmv3.npz)."""
    import torch
    import lavish_dsp.motion as M
    from test_oracle_fixtures import _load, tplmv_case_inputs
    F = _load("fix_tplmv3.npz")
    fld = {n: i for i, n in enumerate(F["rec_fields"])}
    qindex, rdmult, spb, epb, allow_hp = (int(v) for v in F["params"])
    costs = M.MvCosts(F["mvjcost_hp"], F["mvcost_hp"], device="cuda")
    cost = costs.cost_params(spb, epb, M.MV_COST_ENTROPY)
    src = torch.from_numpy(F["src"]).cuda()
    refs = torch.from_numpy(F["refs"]).cuda()
    for ci in range(len(F["cases"])):
        jobs, (meth, sp, skip, prune, alike), (cols, rows, nref) = tplmv_case_inputs(F, ci)
        third = torch.from_numpy(np.ascontiguousarray(F["third"][ci], dtype=np.int32)).cuda()
        out = T.tpl_motion_search(src, refs, M.to_device(jobs), cols, rows, nref, cost, meth, sp,
                                  skip, prune, alike, third)
        torch.cuda.synchronize()
        assert T.tpl_motion_failures(out) == 0
        r, c = T.unpack_mv(out["mvs"].cpu().numpy())
        rc = F["recs"][F["recs"][:, fld["case"]] == ci]
        np.testing.assert_array_equal(r, rc[:, fld["mv_row"]], err_msg="case %d" % ci)
        np.testing.assert_array_equal(c, rc[:, fld["mv_col"]], err_msg="case %d" % ci)
