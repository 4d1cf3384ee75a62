"""GPU parity of the C3 DIAMOND full-pixel motion search
(lavish_diamond_search_batch) against the oracle's restatement of
av1_full_pixel_search / full_pixel_diamond / diamond_search_sad
(oracle/oracle_mcomp.c): best mv, returned var cost and the number of
diamond steps must match exactly for every (block, reference) job."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

BORDER = 160


@pytest.fixture(scope="module")
def planes():
    import lavish_dsp.synth as synth
    W, H = 480, 272
    src, refs = synth.motion_planes(W, H, 3, BORDER, seed=77)
    return W, H, src, refs


def _run(M, planes, bw, bh, step_param=0, cost=3, skip=False, ref_mv=(0, 0), start=(0, 0),
         sub=1, method="diamond"):
    import torch
    W, H, src, refs = planes
    stride = src.shape[1]
    jobs = M.frame_jobs(W, H, stride, BORDER, src.size, bw, bh, refs.shape[0], ref_mv, start)
    jobs = jobs[::sub]
    ts = torch.from_numpy(src).cuda()
    tr = torch.from_numpy(refs).cuda()
    got = M.results_numpy(M.diamond_search_batch(ts, tr, bw, bh, M.to_device(jobs), step_param,
                                                 cost, skip, method=method))
    exp = O.diamond_batch(src.reshape(-1), refs.reshape(-1), stride, bw, bh, jobs, step_param,
                          cost, skip, threads=8, method=method)
    for f in ("best_row", "best_col", "bestsme", "steps"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    return got


@pytest.fixture(scope="module")
def M():
    import lavish_dsp.motion as M
    return M


@pytest.mark.parametrize("bw,bh", [(16, 16), (8, 8), (32, 32), (64, 64), (4, 4), (16, 8),
                                   (8, 32), (64, 16), (128, 128), (32, 64)])
def test_diamond_sizes(M, planes, bw, bh):
    got = _run(M, planes, bw, bh, sub=1 if bw * bh <= 1024 else 1)
    # the synthetic references are displaced by (3k, -2k): most blocks find it
    assert (np.abs(got["best_row"]) + np.abs(got["best_col"]) > 0).mean() > 0.5


@pytest.mark.parametrize("cost", [1, 2, 3, 4])
def test_diamond_cost_types(M, planes, cost):
    _run(M, planes, 16, 16, cost=cost, ref_mv=(13, -21))


@pytest.mark.parametrize("step_param", [0, 3, 7, 10])
def test_diamond_step_param(M, planes, step_param):
    _run(M, planes, 16, 16, step_param=step_param, start=(2, -3))


@pytest.mark.parametrize("bw,bh", [(16, 16), (32, 32), (8, 16)])
def test_diamond_downsampled_sad(M, planes, bw, bh):
    _run(M, planes, bw, bh, skip=True)


def test_diamond_edges_and_clamped_start(M, planes):
    """Start mvs outside the limits are clamped; blocks on the frame edge
    exercise the per-site range checks (not all_in)."""
    _run(M, planes, 16, 16, start=(-900, 700))
    _run(M, planes, 16, 16, start=(300, -300), ref_mv=(-40, 33))


# ---- FAST_BIGDIA (pattern_search) ----

@pytest.mark.parametrize("bw,bh", [(16, 16), (8, 8), (32, 32), (64, 64), (4, 4), (16, 8),
                                   (8, 32), (128, 128), (4, 16)])
def test_bigdia_sizes(M, planes, bw, bh):
    got = _run(M, planes, bw, bh, step_param=6, method="bigdia")
    assert (np.abs(got["best_row"]) + np.abs(got["best_col"]) > 0).mean() > 0.3


@pytest.mark.parametrize("step_param", [0, 6, 8, 9, 10])
def test_bigdia_step_param(M, planes, step_param):
    _run(M, planes, 16, 16, step_param=step_param, start=(3, -2), method="bigdia")


@pytest.mark.parametrize("cost", [1, 2, 3, 4])
def test_bigdia_cost_types_and_skip(M, planes, cost):
    _run(M, planes, 16, 16, step_param=6, cost=cost, ref_mv=(13, -21), skip=True,
         method="bigdia")


def test_bigdia_edges(M, planes):
    _run(M, planes, 16, 16, step_param=6, start=(-900, 700), method="bigdia")
    _run(M, planes, 32, 32, step_param=8, start=(300, -300), ref_mv=(-40, 33), method="bigdia")
