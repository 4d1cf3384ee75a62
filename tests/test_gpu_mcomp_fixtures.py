"""GPU parity of lavish_full_pixel_search_batch against av1_full_pixel_search
executed from the reference (tests/golden/fix_mcomp.npz, made by
tests/golden/gen_fixtures.py): DIAMOND, BIGDIA (do_init_search 1) and
FAST_BIGDIA, MV_COST_ENTROPY with the default-context nmv cost tables, L1 and
none, with and without the downsampled-SAD speed feature (and its quality
recheck) and with and without a cost list -- best mv, returned var cost and
the five cost-list entries bit-exact.  No oracle in the loop, except in
test_full_pixel_search_mesh_vs_oracle (wider mesh settings against the
restatement that fix_mcomp3 pins)."""
import os

import numpy as np
import pytest

import _oracle as O
from _mcomp_fix import MS_METHODS, mcomp_groups

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def F():
    return dict(np.load(os.path.join(GOLD, "fix_mcomp.npz")))


@pytest.mark.parametrize("tiled", [False, True])
def test_full_pixel_search_vs_reference(F, tiled):
    """tiled: candidate rows from the LavishRefTiles copy of the references
    (w <= 16; larger blocks take the linear form through the same call)."""
    import torch
    assert torch.cuda.is_available()
    from lavish_dsp import motion as M
    src = torch.from_numpy(F["src"]).cuda()
    refs = torch.from_numpy(np.ascontiguousarray(F["refs"])).cuda()
    tiles = M.RefTiles(refs, src.stride(0)).build() if tiled else None
    costs = M.MvCosts(F["mvjcost_lp"], F["mvcost_lp"])
    n = 0
    for case, bw, bh, epb, spb, rec, rows, J in mcomp_groups(F):
        m, use_cl, ctype, skip, sp = (int(v) for v in case)
        cp = costs.cost_params(spb, epb, ctype)
        out, cl = M.full_pixel_search_batch(src, refs, bw, bh, M.to_device(rec), cp,
                                            MS_METHODS[m], sp, bool(skip), bool(use_cl),
                                            tiles=tiles)
        torch.cuda.synchronize()
        res = M.results_numpy(out)
        msg = "case %s %dx%d" % ([int(v) for v in case], bw, bh)
        np.testing.assert_array_equal(res["best_row"], rows[:, J["best_row"]], err_msg=msg)
        np.testing.assert_array_equal(res["best_col"], rows[:, J["best_col"]], err_msg=msg)
        np.testing.assert_array_equal(res["bestsme"], rows[:, J["var"]], err_msg=msg)
        if use_cl:
            np.testing.assert_array_equal(cl.cpu().numpy(), rows[:, J["cl0"]:J["cl4"] + 1],
                                          err_msg=msg)
        n += len(rows)
    assert n == len(F["jobs"])


@pytest.mark.parametrize("tiled", [False, True])
def test_full_pixel_search_methods2_vs_reference(tiled):
    """The methods of tests/golden/fix_mcomp2.npz (av1_full_pixel_search
    executed from the reference): NSTEP / NSTEP_8PT (the nstep site
    configuration's 8 / 12-point steps, equal-radius step skipping), HEX /
    FAST_HEX and SQUARE pattern searches, with and without cost lists and
    the downsampled SAD -- bit-exact."""
    import torch
    from lavish_dsp import motion as M
    F2 = dict(np.load(os.path.join(GOLD, "fix_mcomp2.npz")))
    methods = [str(m).lower() for m in F2["methods"]]
    src = torch.from_numpy(F2["src"]).cuda()
    refs = torch.from_numpy(np.ascontiguousarray(F2["refs"])).cuda()
    tiles = M.RefTiles(refs, src.stride(0)).build() if tiled else None
    costs = M.MvCosts(F2["mvjcost_lp"], F2["mvcost_lp"])
    n = 0
    for case, bw, bh, epb, spb, rec, rows, J in mcomp_groups(F2):
        m, use_cl, ctype, skip, sp = (int(v) for v in case)
        cp = costs.cost_params(spb, epb, ctype)
        out, cl = M.full_pixel_search_batch(src, refs, bw, bh, M.to_device(rec), cp,
                                            methods[m], sp, bool(skip), bool(use_cl),
                                            tiles=tiles)
        torch.cuda.synchronize()
        res = M.results_numpy(out)
        msg = "%s case %s %dx%d" % (methods[m], [int(v) for v in case], bw, bh)
        np.testing.assert_array_equal(res["best_row"], rows[:, J["best_row"]], err_msg=msg)
        np.testing.assert_array_equal(res["best_col"], rows[:, J["best_col"]], err_msg=msg)
        np.testing.assert_array_equal(res["bestsme"], rows[:, J["var"]], err_msg=msg)
        if use_cl:
            np.testing.assert_array_equal(cl.cpu().numpy(), rows[:, J["cl0"]:J["cl4"] + 1],
                                          err_msg=msg)
        n += len(rows)
    assert n == len(F2["jobs"])


def _mesh(row):
    from lavish_dsp import motion as M
    r = [int(v) for v in row]
    return M.MeshParams.make([(r[6 + 2 * i], r[7 + 2 * i]) for i in range(4)], *r[:6])


@pytest.mark.parametrize("tiled", [False, True])
def test_full_pixel_search_mesh_vs_reference(tiled):
    """lavish_full_pixel_search_batch_mesh against av1_full_pixel_search with
    the exhaustive mesh refinement executed from the reference
    (tests/golden/fix_mcomp3.npz: force_mesh_thresh after NSTEP / NSTEP_8PT,
    run_mesh_search after DIAMOND / BIGDIA / FAST_HEX / SQUARE, pruning, the
    fine interval, the intraBC patterns, range growth, an illegal pattern;
    cost lists, downsampled SAD) -- bit-exact."""
    import torch
    from lavish_dsp import motion as M
    F3 = dict(np.load(os.path.join(GOLD, "fix_mcomp3.npz")))
    methods = [str(m).lower() for m in F3["methods"]]
    src = torch.from_numpy(F3["src"]).cuda()
    refs = torch.from_numpy(np.ascontiguousarray(F3["refs"])).cuda()
    tiles = M.RefTiles(refs, src.stride(0)).build() if tiled else None
    costs = M.MvCosts(F3["mvjcost_lp"], F3["mvcost_lp"])
    n = 0
    for case, bw, bh, epb, spb, rec, rows, J in mcomp_groups(F3):
        m, use_cl, ctype, skip, sp = (int(v) for v in case)
        mesh = _mesh(F3["mesh"][int(rows[0, J["case"]])])
        cp = costs.cost_params(spb, epb, ctype)
        out, cl = M.full_pixel_search_batch(src, refs, bw, bh, M.to_device(rec), cp,
                                            methods[m], sp, bool(skip), bool(use_cl),
                                            tiles=tiles, mesh=mesh)
        torch.cuda.synchronize()
        res = M.results_numpy(out)
        msg = "%s case %s %dx%d" % (methods[m], [int(v) for v in case], bw, bh)
        np.testing.assert_array_equal(res["best_row"], rows[:, J["best_row"]], err_msg=msg)
        np.testing.assert_array_equal(res["best_col"], rows[:, J["best_col"]], err_msg=msg)
        np.testing.assert_array_equal(res["bestsme"], rows[:, J["var"]], err_msg=msg)
        if use_cl:
            np.testing.assert_array_equal(cl.cpu().numpy(), rows[:, J["cl0"]:J["cl4"] + 1],
                                          err_msg=msg)
        n += len(rows)
    assert n == len(F3["jobs"])


MESH_SETS = [  # (patterns, run, force_thresh, prune, diff, fine, intra)
    ([(64, 8), (28, 4), (15, 1), (7, 1)], 1, 0x7FFFFFFF, 0, 4, 0, 0),
    ([(64, 16), (24, 8), (12, 4), (7, 1)], 0, 0, 1, 2, 1, 0),
    ([(9, 3), (7, 1), (0, 0), (0, 0)], 1, 0, 1, 1, 0, 1),
    ([(16, 1), (7, 1), (7, 1), (7, 1)], 0, 1 << 14, 0, 4, 0, 0),
]


@pytest.mark.parametrize("mi", range(len(MESH_SETS)))
@pytest.mark.parametrize("method", ["nstep", "nstep_8pt", "diamond", "fast_bigdia", "hex"])
def test_full_pixel_search_mesh_vs_oracle(mi, method):
    """The mesh refinement after five methods at four mesh settings (every
    fix_mcomp3 job geometry, entropy cost, cost lists, downsampled SAD on
    alternate sizes) against the oracle restatement (pinned to the reference
    by the fixture test above)."""
    import torch
    from lavish_dsp import motion as M
    F3 = dict(np.load(os.path.join(GOLD, "fix_mcomp3.npz")))
    src = torch.from_numpy(F3["src"]).cuda()
    refs = torch.from_numpy(np.ascontiguousarray(F3["refs"])).cuda()
    costs = M.MvCosts(F3["mvjcost_lp"], F3["mvcost_lp"])
    pats, run, thr, prune, diff, fine, intra = MESH_SETS[mi]
    mesh = M.MeshParams.make(pats, run, thr, prune, diff, fine, intra)
    omesh = O.OrcMeshParams(run, thr, prune, diff, fine, intra)
    for i, (r, iv) in enumerate(pats):
        omesh.range[i], omesh.interval[i] = r, iv
    stride = F3["src"].shape[1]
    for k, (case, bw, bh, epb, spb, rec, rows, J) in enumerate(mcomp_groups(F3)):
        skip = k % 2
        cp = costs.cost_params(spb, epb, 0)
        out, cl = M.full_pixel_search_batch(src, refs, bw, bh, M.to_device(rec), cp, method, 1,
                                            bool(skip), True, mesh=mesh)
        torch.cuda.synchronize()
        res = M.results_numpy(out)
        exp, ecl = O.full_pixel_search_batch(F3["src"], F3["refs"], stride, bw, bh, rec, method,
                                             1, 0, spb, epb, F3["mvjcost_lp"], F3["mvcost_lp"],
                                             skip=bool(skip), cost_list=True, mesh=omesh)
        msg = "%s %dx%d" % (method, bw, bh)
        for f in ("best_row", "best_col", "bestsme"):
            np.testing.assert_array_equal(res[f], exp[f], err_msg=msg + " " + f)
        np.testing.assert_array_equal(cl.cpu().numpy(), ecl, err_msg=msg + " cost list")


def test_full_pixel_search_mesh_rejects():
    """A later mesh pass the walk can reach with interval < 1: -6 (the
    reference's loop would not end); an illegal first pattern: the results
    of the search without mesh."""
    import torch
    from lavish_dsp import motion as M
    F3 = dict(np.load(os.path.join(GOLD, "fix_mcomp3.npz")))
    src = torch.from_numpy(F3["src"]).cuda()
    refs = torch.from_numpy(np.ascontiguousarray(F3["refs"])).cuda()
    costs = M.MvCosts(F3["mvjcost_lp"], F3["mvcost_lp"])
    case, bw, bh, epb, spb, rec, rows, J = next(iter(mcomp_groups(F3)))
    cp = costs.cost_params(spb, epb, 0)
    jobs = M.to_device(rec)
    bad = M.MeshParams.make([(64, 8), (28, 0), (15, 1), (7, 1)], run_mesh_search=1)
    with pytest.raises(ValueError):
        M.full_pixel_search_batch(src, refs, bw, bh, jobs, cp, "diamond", 1, mesh=bad)
    noop = M.MeshParams.make([(300, 8), (28, 0), (15, 1), (7, 1)], run_mesh_search=1)
    a, _ = M.full_pixel_search_batch(src, refs, bw, bh, jobs, cp, "diamond", 1, mesh=noop)
    b, _ = M.full_pixel_search_batch(src, refs, bw, bh, jobs, cp, "diamond", 1)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_full_pixel_search_rejects(F):
    """Entropy cost without tables, unknown search methods and bad step
    params are refused (no launch)."""
    import torch
    from lavish_dsp import motion as M
    src = torch.zeros((64, 64), dtype=torch.uint8, device="cuda")
    jobs = M.to_device(np.zeros(1, M.JOB_DTYPE))
    with pytest.raises(ValueError, match="rc=-2"):
        M.full_pixel_search_batch(src, src, 8, 8, jobs, M.MvCostParams(0, 4, 40, 0))
    import ctypes
    # CLAMPED_DIAMOND (3) is not served: refused before any launch
    rc = M._lib.lavish_full_pixel_search_batch(None, 64, None, 64, 8, 8, None, 1, 3, 0,
                                               ctypes.byref(M.l1_cost_params()), 0, None, None,
                                               None)
    assert rc == -4
    with pytest.raises(ValueError, match="rc=-1"):
        M.full_pixel_search_batch(src, src, 8, 8, jobs, M.l1_cost_params(), step_param=11)


def test_subpel_search_vs_reference(F):
    """lavish_find_best_sub_pixel_tree_batch against
    av1_find_best_sub_pixel_tree (USE_2_TAPS_ORIG) / _pruned / _pruned_more executed from the
    reference (tests/golden/fix_subpel.npz): entropy (hp / lp tables), L1 and
    none mv costs, with and without the full-pel cost list, forced_stop and
    iters_per_step variants -- best mv, besterr, distortion, sse bit-exact."""
    import torch
    from lavish_dsp import motion as M
    from _mcomp_fix import subpel_groups
    S = dict(np.load(os.path.join(GOLD, "fix_subpel.npz")))
    src = torch.from_numpy(F["src"]).cuda()
    refs = torch.from_numpy(np.ascontiguousarray(F["refs"])).cuda()
    costs = {t: M.MvCosts(F["mvjcost_" + t], F["mvcost_" + t]) for t in ("lp", "hp")}
    n = 0
    for case, bw, bh, epb, rec, cls, rows, J in subpel_groups(S, F):
        meth, hp, fstop, iters, ctype, use_cl = (int(v) for v in case)
        cp = costs["hp" if hp else "lp"].cost_params(0, epb, ctype)
        out = M.find_best_sub_pixel_tree_batch(
            src, refs, bw, bh, M.to_device(rec), cp, {0: "tree", 1: "pruned", 2: "pruned_more"}[meth],
            fstop, bool(hp), iters, cost_lists=torch.from_numpy(cls).cuda() if use_cl else None)
        torch.cuda.synchronize()
        res = M.subpel_results_numpy(out)
        msg = "case %s %dx%d" % ([int(v) for v in case], bw, bh)
        for f in ("best_row", "best_col", "besterr", "distortion", "sse"):
            np.testing.assert_array_equal(res[f].astype(np.int64), rows[:, J[f]],
                                          err_msg=msg + " " + f)
        n += len(rows)
    assert n == len(S["jobs"])


def test_fullpel_then_subpel_chain(F):
    """The RDO path's chain on the device: full-pel DIAMOND with entropy cost
    and cost list, then pruned_more from its results and cost lists -- equal to
    the same two steps run from the fixture's full-pel answers."""
    import torch
    from lavish_dsp import motion as M
    from _mcomp_fix import MS_METHODS, mcomp_groups
    src = torch.from_numpy(F["src"]).cuda()
    refs = torch.from_numpy(np.ascontiguousarray(F["refs"])).cuda()
    costs = M.MvCosts(F["mvjcost_lp"], F["mvcost_lp"])
    checked = 0
    for case, bw, bh, epb, spb, rec, rows, J in mcomp_groups(F):
        m, use_cl, ctype, skip, sp = (int(v) for v in case)
        if not use_cl or ctype != 0:
            continue
        cp = costs.cost_params(spb, epb, 0)
        fp, cl = M.full_pixel_search_batch(src, refs, bw, bh, M.to_device(rec), cp,
                                           MS_METHODS[m], sp, bool(skip), True)
        # sub-pel jobs: SubpelMvLimits from the block's x->mv_limits and ref_mv
        W, H, BORDER, _ = (int(v) for v in F["geom"])
        srec = rec.copy()
        for i, r in enumerate(rows):
            lim = M.block_mv_limits(((H + 7) & ~7) // 4, ((W + 7) & ~7) // 4, r[J["by"]] // 4,
                                    r[J["bx"]] // 4, bh // 4, bw // 4, BORDER)
            (srec["col_min"][i], srec["col_max"][i], srec["row_min"][i],
             srec["row_max"][i]) = M.subpel_limits(lim, (r[J["ref_mv_row"]], r[J["ref_mv_col"]]))
        chained = M.find_best_sub_pixel_tree_batch(src, refs, bw, bh, M.to_device(srec), cp,
                                                   fullpel=fp, cost_lists=cl)
        srec["start_row"] = rows[:, J["best_row"]] * 8
        srec["start_col"] = rows[:, J["best_col"]] * 8
        ref_cl = torch.from_numpy(np.ascontiguousarray(
            rows[:, J["cl0"]:J["cl4"] + 1].astype(np.int32))).cuda()
        direct = M.find_best_sub_pixel_tree_batch(src, refs, bw, bh, M.to_device(srec), cp,
                                                  cost_lists=ref_cl)
        torch.cuda.synchronize()
        a, b = M.subpel_results_numpy(chained), M.subpel_results_numpy(direct)
        np.testing.assert_array_equal(a, b)
        checked += len(rows)
    assert checked > 50


@pytest.mark.parametrize("stride,rows", [(64, 48), (2240, 9), (100, 7)])
def test_ref_tiles_layout(stride, rows):
    """lavish_ref_tiles_build: field f, strip k, field row fy holds bytes
    [16k, 16k + 32) of buffer row 2 fy + f; zero past the row end / last row."""
    import torch
    from lavish_dsp import motion as M
    rng = np.random.default_rng(stride + rows)
    buf = rng.integers(0, 256, (rows, stride)).astype(np.uint8)
    t = M.RefTiles(torch.from_numpy(buf).cuda(), stride).build()
    torch.cuda.synchronize()
    got = t.data.cpu().numpy()
    ns, fh = (stride + 15) // 16, (rows + 1) // 2
    assert t.desc.field_rows == fh and t.desc.field_bytes == ns * fh * 32
    assert got.size == 2 * ns * fh * 32
    pad = np.zeros((2 * fh, ns * 16 + 32), np.uint8)
    pad[:rows, :stride] = buf
    exp = np.zeros((2, ns, fh, 32), np.uint8)
    for f in range(2):
        for k in range(ns):
            exp[f, k] = pad[f::2, 16 * k:16 * k + 32]
    np.testing.assert_array_equal(got.reshape(2, ns, fh, 32), exp)


def test_subpel_tree_upsampled_vs_reference(F):
    """lavish_find_best_sub_pixel_tree_batch_ex (SUBPEL_TREE, subpel_search_type
    USE_2_TAPS / USE_4_TAPS / USE_8_TAPS) against av1_find_best_sub_pixel_tree
    executed from the reference with the upsampled prediction error
    (tests/golden/fix_subpel_up.npz): best mv, besterr, distortion, sse."""
    import torch
    from lavish_dsp import motion as M
    from _mcomp_fix import subpel_groups
    S = dict(np.load(os.path.join(GOLD, "fix_subpel_up.npz")))
    src = torch.from_numpy(F["src"]).cuda()
    refs = torch.from_numpy(np.ascontiguousarray(F["refs"])).cuda()
    costs = {t: M.MvCosts(F["mvjcost_" + t], F["mvcost_" + t]) for t in ("lp", "hp")}
    n = 0
    for case, bw, bh, epb, rec, _, rows, J in subpel_groups(S, F):
        stype, hp, fstop, iters, ctype = (int(v) for v in case)
        cp = costs["hp" if hp else "lp"].cost_params(0, epb, ctype)
        out = M.find_best_sub_pixel_tree_batch(src, refs, bw, bh, M.to_device(rec), cp, "tree",
                                               fstop, bool(hp), iters, search_type=stype)
        torch.cuda.synchronize()
        res = M.subpel_results_numpy(out)
        msg = "case %s %dx%d" % ([int(v) for v in case], bw, bh)
        for f in ("best_row", "best_col", "besterr", "distortion", "sse"):
            np.testing.assert_array_equal(res[f].astype(np.int64), rows[:, J[f]],
                                          err_msg=msg + " " + f)
        n += len(rows)
    assert n == len(S["jobs"])


@pytest.mark.parametrize("stype", [2, 3])
@pytest.mark.parametrize("bw,bh", [(16, 16), (8, 8), (32, 16), (64, 64), (4, 8)])
def test_subpel_tree_upsampled_vs_oracle(stype, bw, bh):
    """Every block of a 320x192 frame x 2 references (SUBPEL_TREE, USE_4_TAPS /
    USE_8_TAPS, entropy costs, from the DIAMOND full-pel results) against the
    oracle's upsampled error, bit-exact."""
    import torch
    import _oracle as O
    from lavish_dsp import motion as M, synth
    W, H, R, border = 320, 192, 2, 160
    src, refs = synth.motion_planes(W, H, R, border, seed=91 + bw + stype)
    st = src.shape[1]
    jobs = M.frame_jobs(W, H, st, border, src.size, bw, bh, R, ref_mv=(12, -20))
    mvj, mvc = M.default_mv_cost_tables(True)
    fp, _ = O.full_pixel_search_batch(src.reshape(-1), refs.reshape(-1), st, bw, bh, jobs,
                                      "diamond", 2, 0, 4, 40, mvj, mvc, threads=8)
    sj = M.subpel_jobs(W, H, border, bw, bh, jobs, fp, ref_mv=(12, -20))
    exp = O.subpel_search_batch(src.reshape(-1), refs.reshape(-1), st, bw, bh, sj, 0, 0, True,
                                2, 0, 40, mvj, mvc, None, threads=8, search_type=stype)
    costs = M.MvCosts(mvj, mvc)
    out = M.find_best_sub_pixel_tree_batch(
        torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda(), bw, bh, M.to_device(sj),
        costs.cost_params(0, 40, M.MV_COST_ENTROPY), "tree", 0, True, 2, search_type=stype)
    torch.cuda.synchronize()
    got = M.subpel_results_numpy(out)
    for f in ("best_row", "best_col", "besterr", "distortion", "sse"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)


def test_mesh_bench_workload_vs_oracle():
    """bench.py --workload mesh's call (the temporal filter's search: NSTEP,
    MV_COST_L1_HDRES, run_mesh_search on every job, the speed-6 mesh
    patterns, cost lists) on a 1920x128 strip x 7 references against the
    oracle restatement (pinned to av1_full_pixel_search by fix_mcomp3)."""
    import importlib.util
    import torch
    from lavish_dsp import motion as M
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    W, H, R = 1920, 128, 7
    src, refs, st, jobs = b.mesh_setup(W, H, R, 5)
    mesh = M.MeshParams.make(b.MESH_PATTERNS, run_mesh_search=1)
    out, cl = M.full_pixel_search_batch(torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda(),
                                        16, 16, M.to_device(jobs),
                                        M.l1_cost_params(M.MV_COST_L1_HDRES), "nstep", 0, False,
                                        True, mesh=mesh)
    torch.cuda.synchronize()
    om = O.OrcMeshParams(1, 0x7FFFFFFF, 0, 4, 0, 0)
    for i, (r, iv) in enumerate(b.MESH_PATTERNS):
        om.range[i], om.interval[i] = r, iv
    exp, ecl = O.full_pixel_search_batch(src.reshape(-1), refs.reshape(-1), st, 16, 16, jobs,
                                         "nstep", 0, 3, 0, 0, skip=False, cost_list=True,
                                         threads=8, mesh=om)
    res = M.results_numpy(out)
    for f in ("best_row", "best_col", "bestsme"):
        np.testing.assert_array_equal(res[f], exp[f], err_msg=f)
    np.testing.assert_array_equal(cl.cpu().numpy(), ecl)
