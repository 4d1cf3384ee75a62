"""CPU checks of the oracle's DIAMOND search restatement
(oracle/oracle_mcomp.c) and of the host-side job construction
(lavish_dsp.motion.mv_limits / frame_jobs).  No reference fixture covers the
search control flow itself (SURVEY.md 8(c) lists none), so beyond the pinned
SAD / variance primitives its parity is checked here through properties the
reference's own code implies."""
import numpy as np
import pytest

import _oracle as O


@pytest.fixture(scope="module")
def setup():
    import lavish_dsp.motion as M
    import lavish_dsp.synth as S
    W, H = 320, 192
    src, refs = S.motion_planes(W, H, 2, 160, seed=5)
    return M, S, W, H, src, refs


def test_mv_limits_formula(setup):
    M = setup[0]
    # av1_set_mv_limits for a 16x16 block at the top-left of a 1080p frame,
    # border 160: rows may reach -(16 + 8) (min2) and (1080 - 16) + 152 (max1)
    mi_rows, mi_cols = 1080 // 4, 1920 // 4
    cmin, cmax, rmin, rmax = M.mv_limits(mi_rows, mi_cols, 0, 0, 4, 4, 160)
    assert (rmin, cmin) == (-24, -24)
    assert rmax == min(1080 - 16 + 152, 1080 + 8, 1023)
    assert cmax == min(1920 - 16 + 152, 1920 + 8, 1023)
    # av1_set_mv_search_range around a ref mv of (-80, 52) 1/8 pel
    cmin, cmax, rmin, rmax = M.mv_limits(mi_rows, mi_cols, 100, 200, 4, 4, 160, (-80, 52))
    assert rmin == max(-(400 + 152), -(416 + 8), ((-80 + 7) >> 3) - 1023)
    assert cmax == min((480 - 204) * 4 + 152, (480 - 200) * 4 + 8, (52 >> 3) + 1023)


def test_diamond_recovers_synthetic_motion(setup):
    M, S, W, H, src, refs = setup
    st = src.shape[1]
    jobs = M.frame_jobs(W, H, st, 160, src.size, 16, 16, 2)
    r = O.diamond_batch(src.reshape(-1), refs.reshape(-1), st, 16, 16, jobs, threads=4)
    n = len(jobs) // 2
    for k in range(2):
        rr = r[k * n:(k + 1) * n]
        # ref_k = current displaced by (3(k+1), -2(k+1)) -> mv (-2(k+1), 3(k+1))
        mvs, cnt = np.unique(np.stack([rr["best_row"], rr["best_col"]], 1), axis=0,
                             return_counts=True)
        assert tuple(mvs[cnt.argmax()]) == (-2 * (k + 1), 3 * (k + 1))
        assert cnt.max() > 0.3 * n
        assert (rr["steps"] >= 11).all()


def test_diamond_invariants(setup):
    """best mv inside the limits; returned cost == variance + L1 mv cost at
    the best mv; MV_COST_NONE on an exact copy finds (0,0) with cost 0."""
    M, S, W, H, src, refs = setup
    st = src.shape[1]
    jobs = M.frame_jobs(W, H, st, 160, src.size, 16, 16, 1)
    r = O.diamond_batch(src.reshape(-1), refs.reshape(-1), st, 16, 16, jobs, threads=4)
    assert ((r["best_row"] >= jobs["row_min"]) & (r["best_row"] <= jobs["row_max"])).all()
    assert ((r["best_col"] >= jobs["col_min"]) & (r["best_col"] <= jobs["col_max"])).all()
    fs, fr = src.reshape(-1), refs.reshape(-1)
    for j in range(0, len(jobs), 17):
        so, ro = int(jobs["src_off"][j]), int(jobs["ref_off"][j])
        br, bc = int(r["best_row"][j]), int(r["best_col"][j])
        a = np.lib.stride_tricks.as_strided(fs[so:], (16, 16), (st, 1))
        b = np.lib.stride_tricks.as_strided(fr[ro + br * st + bc:], (16, 16), (st, 1))
        v, _ = O.variance(a, st, b, st, 16, 16)
        assert r["bestsme"][j] == v + (abs(br * 8) + abs(bc * 8)) // 8  # L1_HDRES, ref mv 0
    same = O.diamond_batch(src.reshape(-1), src.reshape(-1), st, 16, 16,
                           M.frame_jobs(W, H, st, 160, 0, 16, 16, 1), mv_cost_type=4)
    assert (same["best_row"] == 0).all() and (same["best_col"] == 0).all()
    assert (same["bestsme"] == 0).all()
