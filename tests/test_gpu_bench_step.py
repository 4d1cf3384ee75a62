"""The headline step exactly as bench.py times it, against the oracle.

bench.RdoStep is the object main() times: C3 (the DIAMOND full-pel search of
every 16x16 block x 7 references, downsampled SAD, MV_COST_ENTROPY over the
default nmv tables, cost lists; av1_full_pixel_search, mcomp.c:1755 ->
full_pixel_diamond :1479 -> diamond_search_sad :1318-1477) beside C2
(lavish_txq_frame: every block of the 14 TX sizes <= 32x32 x every valid
type, tx_search.c:2148-2312 -> encodemb.c:295-341).  The default step
("split32") runs C3 on a side stream in at most 384 workgroups
(lavish_set_search_workgroup_cap: the search kernel strides over virtual
workgroups) followed there by C2's 32-point sizes, and the rest of C2 on the
caller's stream; "streams" keeps all of C2 on the caller's stream; "fused"
runs C2 and C3 as one launch (lavish_txq_frame_search: the search's job
groups interleaved among the transform's workgroups) on the caller's
stream.  Two consecutive steps run, then both legs' outputs are compared
with the oracle; the search at workgroup caps {8, 64, 384, 512, 0} and the fused
launch at interleaving strides {1, 3, 10, 40} must give identical results.
"""
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

THREADS = max(1, min(32, os.cpu_count() or 1))


def _bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


@pytest.fixture(scope="module")
def step():
    import torch
    assert torch.cuda.is_available()
    b = _bench()
    R = b.RdoStep()  # the bench's defaults: 1080p, 7 refs, qindex 128, overlapped
    assert R.overlap and R.fused == (b.C3_MODE == "fused") and R.c3_wg_cap == 384
    assert R.split32 == (b.C3_MODE == "split32")
    return b, R


@pytest.fixture(scope="module")
def c2_expected(step):
    b, R = step
    oq = O.build_quant(8, 128)
    return {s: O.txq_plane(R.res_np, s, R.L.valid_type_mask(s), oq, threads=THREADS)
            for s in R.sizes}


@pytest.fixture(scope="module")
def c3_expected(step):
    b, R = step
    mvj, mvc = R.mv_tables
    return O.full_pixel_search_batch(R.src_np.reshape(-1), R.refs_np.reshape(-1), R.ref_stride,
                                     b.C3_BLOCK, b.C3_BLOCK, R.jobs_np, "diamond", 0, b.C3_COST,
                                     R.sad_per_bit, R.error_per_bit, mvj, mvc, skip=b.C3_SKIP,
                                     cost_list=b.C3_CL, threads=THREADS)


def _check_c3(R, exp, exp_cl, what):
    got = R.M.results_numpy(R.c3_out)
    for f in ("best_row", "best_col", "bestsme", "steps"):  # the oracle has no search count
        np.testing.assert_array_equal(got[f], exp[f], err_msg="%s: %s" % (what, f))
    np.testing.assert_array_equal(R.c3_cl.cpu().numpy(), exp_cl, err_msg=what + ": cost list")
    return got


def _poison(R):
    R.c3_out.fill_(0x55)
    R.c3_cl.fill_(-7)
    for out in R.frame.outs.values():
        for t in out.values():
            t.fill_(0x33)


def _check_c2(R, c2_expected, what):
    for s in R.sizes:
        qc, dq, eob = c2_expected[s]
        out = R.frame.outs[s]
        np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), qc.transpose(1, 0, 2),
                                      err_msg="%s: size %d qcoeff" % (what, s))
        np.testing.assert_array_equal(out["dqcoeff"].cpu().numpy(), dq.transpose(1, 0, 2),
                                      err_msg="%s: size %d dqcoeff" % (what, s))
        np.testing.assert_array_equal(out["eob"].cpu().numpy().view(np.uint16), eob.T,
                                      err_msg="%s: size %d eob" % (what, s))


@pytest.mark.parametrize("mode", ["fused", "streams", "split32"])
def test_timed_step_both_legs(step, c2_expected, c3_expected, mode):
    """Two steps as timed (fused: one launch; streams: C3 capped beside C2 on
    two streams; split32: C2's 32-point sizes after C3 on the second stream,
    the rest of C2 on the caller's), then C3's results and cost lists and
    every C2 size's qcoeff / dqcoeff / eob."""
    import torch
    b, R = step
    fused, split = R.fused, R.split32
    R.fused = mode == "fused"
    R.split32 = mode == "split32"
    try:
        _poison(R)
        for _ in range(2):
            R.step()
        torch.cuda.synchronize()
    finally:
        R.fused, R.split32 = fused, split
    assert R.L.status()[0] == 0, R.L.status()
    got = _check_c3(R, *c3_expected, what=mode)
    assert (np.abs(got["best_row"]) + np.abs(got["best_col"]) > 0).mean() > 0.5
    _check_c2(R, c2_expected, mode)


@pytest.mark.parametrize("every", [1, 3, 10, 40])
def test_fused_launch_interleave_sweep(step, c2_expected, c3_expected, every):
    """lavish_txq_frame_search at several interleaving strides (the search's
    units dispatched every `every` units, clamped into the grid): identical
    results."""
    import torch
    b, R = step
    _poison(R)
    R.c3_tiles.build(stream=R.stream)
    R.M.txq_frame_search(R.res, R.frame, R.qp, R.tsrc, R.trefs, R.tjobs, R.c3_cost, R.c3_tiles,
                         R.c3_out, R.c3_cl, every, use_downsampled_sad=b.C3_SKIP,
                         stream=R.stream)
    torch.cuda.synchronize()
    assert R.L.status()[0] == 0, R.L.status()
    _check_c3(R, *c3_expected, what="every %d" % every)
    _check_c2(R, c2_expected, "every %d" % every)


@pytest.mark.parametrize("queued", [True, False])
@pytest.mark.parametrize("cap", [8, 64, 384, 512, 0])
def test_search_workgroup_cap_sweep(step, c3_expected, cap, queued):
    """The capped search -- wave units pulled from the per-XCD queues
    (diamond_lj_dyn_kernel, the default) or the static grid-stride over
    virtual workgroups -- is the uncapped search: identical results at every
    cap, twice in a row (the queues start from zero each launch)."""
    import torch
    b, R = step
    R.M.set_search_workgroup_cap(cap)
    R.M.set_search_schedule(queued)
    try:
        for it in range(2):
            R.c3_out.fill_(0x55)
            R.c3_cl.fill_(-7)
            R.c3(R.stream)
            torch.cuda.synchronize()
            _check_c3(R, *c3_expected, what="cap %d queued %s pass %d" % (cap, queued, it))
    finally:
        R.M.set_search_workgroup_cap(0)
        R.M.set_search_schedule(True)
