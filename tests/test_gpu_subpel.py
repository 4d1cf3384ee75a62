"""GPU parity of the sub-pixel refinement (lavish_subpel_search_batch,
av1_find_best_sub_pixel_tree_pruned_more) against the oracle's restatement
(oracle/oracle_subpel.c): best mv, error, distortion and sse bit-exact for
every (block, reference) job, starting from the full-pel DIAMOND results."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

BORDER = 160


@pytest.fixture(scope="module")
def planes():
    import lavish_dsp.synth as synth
    W, H = 480, 272
    src, refs = synth.motion_planes(W, H, 3, BORDER, seed=91)
    return W, H, src, refs


def _run(planes, bw, bh, fs=0, hp=True, iters=1, cost=3, ref_mv=(0, 0)):
    import torch
    import lavish_dsp.motion as M
    W, H, src, refs = planes
    stride = src.shape[1]
    jobs = M.frame_jobs(W, H, stride, BORDER, src.size, bw, bh, refs.shape[0], ref_mv)
    ts, tr = torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda()
    full = M.results_numpy(M.diamond_search_batch(ts, tr, bw, bh, M.to_device(jobs), 0, cost,
                                                  bh >= 16))
    sj = M.subpel_jobs(W, H, BORDER, bw, bh, jobs, full, ref_mv)
    got = M.subpel_results_numpy(M.subpel_search_batch(ts, tr, bw, bh, M.to_device(sj), fs, hp,
                                                       iters, cost))
    exp = O.subpel_batch(src.reshape(-1), refs.reshape(-1), stride, bw, bh, sj, fs, hp, iters,
                         cost, threads=8)
    for f in ("best_row", "best_col", "besterr", "distortion", "sse"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    return got, sj


@pytest.mark.parametrize("bw,bh", [(16, 16), (8, 8), (32, 32), (64, 64), (4, 4), (16, 8),
                                   (8, 32), (64, 16), (128, 128), (32, 64), (4, 16)])
def test_subpel_sizes(planes, bw, bh):
    got, sj = _run(planes, bw, bh)
    moved = (got["best_row"] != sj["start_row"]) | (got["best_col"] != sj["start_col"])
    assert moved.mean() > 0.1


@pytest.mark.parametrize("fs,hp,iters", [(0, False, 1), (1, False, 2), (2, False, 1),
                                         (0, True, 2), (3, False, 1), (1, True, 1)])
def test_subpel_precision_and_iters(planes, fs, hp, iters):
    _run(planes, 16, 16, fs, hp, iters)


@pytest.mark.parametrize("cost", [1, 2, 3, 4])
def test_subpel_cost_types(planes, cost):
    _run(planes, 16, 16, 0, True, 2, cost, ref_mv=(13, -21))


def test_subpel_after_diamond_matches(planes):
    """The device-chained entry point (starts read from the full-pel results
    on the device) equals the host-built jobs."""
    import torch
    import lavish_dsp.motion as M
    W, H, src, refs = planes
    stride = src.shape[1]
    jobs = M.frame_jobs(W, H, stride, BORDER, src.size, 16, 16, refs.shape[0])
    ts, tr = torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda()
    fp = M.diamond_search_batch(ts, tr, 16, 16, M.to_device(jobs), 0, 3, True)
    sj = M.subpel_jobs(W, H, BORDER, 16, 16, jobs, M.results_numpy(fp))
    a = M.subpel_results_numpy(M.subpel_search_batch(ts, tr, 16, 16, M.to_device(sj), 0, False))
    blank = sj.copy()
    blank["start_row"] = blank["start_col"] = 0
    b = M.subpel_results_numpy(M.subpel_after_diamond(ts, tr, 16, 16, M.to_device(blank), fp, 0,
                                                      False))
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("bw,bh", [(16, 16), (8, 8), (64, 64), (4, 4), (128, 128), (32, 8)])
@pytest.mark.parametrize("fs,hp,iters", [(0, True, 2), (0, False, 1), (1, False, 2)])
def test_subpel_tree_vs_oracle(planes, bw, bh, fs, hp, iters):
    """SUBPEL_TREE (av1_find_best_sub_pixel_tree with USE_2_TAPS_ORIG) on the
    general entry point against the oracle, L1 cost around a nonzero ref mv."""
    import torch
    import lavish_dsp.motion as M
    W, H, src, refs = planes
    stride = src.shape[1]
    ref_mv = (13, -21)
    jobs = M.frame_jobs(W, H, stride, BORDER, src.size, bw, bh, refs.shape[0], ref_mv)
    ts, tr = torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda()
    full = M.results_numpy(M.diamond_search_batch(ts, tr, bw, bh, M.to_device(jobs), 0, 3,
                                                  bh >= 16))
    sj = M.subpel_jobs(W, H, BORDER, bw, bh, jobs, full, ref_mv)
    got = M.subpel_results_numpy(M.find_best_sub_pixel_tree_batch(
        ts, tr, bw, bh, M.to_device(sj), M.l1_cost_params(), "tree", fs, hp, iters))
    exp = O.subpel_search_batch(src.reshape(-1), refs.reshape(-1), stride, bw, bh, sj, 0, fs,
                                hp, iters, 3, threads=8)
    for f in ("best_row", "best_col", "besterr", "distortion", "sse"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    moved = (got["best_row"] != sj["start_row"]) | (got["best_col"] != sj["start_col"])
    assert moved.mean() > 0.1
