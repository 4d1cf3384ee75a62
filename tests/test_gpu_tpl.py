"""GPU parity of the TPL block leg (lavish_tpl_block_batch) and of the whole
chained TPL frame leg (full-pel FAST_BIGDIA with entropy costs and a cost
list -> sub-pel with MV_COST_NONE -> EIGHTTAP_REGULAR prediction -> per-block
satd / best reference / quantize error / rate / recon) against the oracle
restatement (oracle/oracle_tpl.c and the pinned motion / prediction
oracles), bit-exact."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def T():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp.tpl as T
    return T


def _planes(W, H, nrefs, bd, seed, flat=False):
    rng = np.random.default_rng(seed)
    m = (1 << bd) - 1
    dt = np.uint8 if bd == 8 else np.uint16
    base = rng.integers(0, m + 1, size=(H, W))
    src = base.astype(dt)
    preds = []
    for k in range(nrefs):
        if flat and k == 0:
            preds.append(src.copy())  # zero residual: eob 0, recon = pred
            continue
        noise = rng.integers(-(8 << (bd - 8)) * (k + 1), (8 << (bd - 8)) * (k + 1) + 1,
                             size=(H, W))
        preds.append(np.clip(base + noise, 0, m).astype(dt))
    return src, np.stack(preds)


def _run(T, src, preds, bsize, bd, qindex):
    import torch
    import lavish_dsp as L
    ts = torch.from_numpy(src.view(np.int16) if bd > 8 else src).cuda()
    tp = torch.from_numpy(preds.view(np.int16) if bd > 8 else preds).cuda()
    qp = L.build_quant_params(bd, qindex, L.QUANT_FP)
    out, recon, costs = T.tpl_block_batch(ts, tp, bsize, bd, qp, ref_costs=True)
    torch.cuda.synchronize()
    rec = recon.cpu().numpy()
    return T.records_numpy(out), rec.view(np.uint16) if bd > 8 else rec, costs.cpu().numpy()


@pytest.mark.parametrize("bsize", [8, 16, 32])
@pytest.mark.parametrize("bd", [8, 10, 12])
def test_tpl_block_batch_vs_oracle(T, bsize, bd):
    for qindex, nrefs, seed in ((0, 1, 1), (60, 3, 2), (128, 2, 3), (255, 4, 4)):
        src, preds = _planes(96, 64, nrefs, bd, seed + bsize + bd, flat=(seed == 2))
        got, grec, gcost = _run(T, src, preds, bsize, bd, qindex)
        exp, erec, ecost = O.tpl_block_batch(src, preds, bsize, bd, qindex)
        msg = "bsize %d bd %d q %d" % (bsize, bd, qindex)
        np.testing.assert_array_equal(gcost, ecost, err_msg=msg)
        for f in exp.dtype.names:
            np.testing.assert_array_equal(got[f], exp[f], err_msg=msg + " " + f)
        np.testing.assert_array_equal(grec, erec, err_msg=msg)


def test_tpl_block_batch_extremes(T):
    """Full-swing residuals (src max, pred 0 and the reverse) at 8 / 10 bit."""
    for bd in (8, 10):
        m = (1 << bd) - 1
        dt = np.uint8 if bd == 8 else np.uint16
        src = np.zeros((32, 64), dt)
        src[:, ::2] = m
        preds = np.stack([m - src, np.zeros_like(src)]).astype(dt)
        got, grec, _ = _run(T, src, preds, 16, bd, 20)
        exp, erec, _ = O.tpl_block_batch(src, preds, 16, bd, 20)
        for f in exp.dtype.names:
            np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
        np.testing.assert_array_equal(grec, erec)


def test_tpl_block_batch_rejects(T):
    import torch
    import lavish_dsp as L
    src = torch.zeros((32, 32), dtype=torch.uint8, device="cuda")
    qp = L.build_quant_params(8, 10, L.QUANT_FP)
    with pytest.raises(ValueError, match="rc=-1"):
        T.tpl_block_batch(src, src, 4, 8, qp)


@pytest.mark.parametrize("neighbours", [True, False])
def test_tpl_frame_chain_vs_oracle(T, neighbours):
    """TplFrame.step (the kernels chained on one stream) against the same
    chain of oracles on a 320x192 frame with 3 references: the full-pel step
    with the reference's neighbour-seeded start mvs (the default,
    orc_tpl_motion_search) or from the zero mv."""
    import torch
    import lavish_dsp.inter as I
    import lavish_dsp.motion as M
    import lavish_dsp.synth as synth
    W, H, R, border, qindex, rdmult = 320, 192, 3, 288, 110, 1500
    if neighbours:
        src, refs = synth.tpl_motion_planes(W, H, R, border, seed=77)
    else:
        src, refs = synth.motion_planes(W, H, R, border, seed=77)
    tf = T.TplFrame(src, refs, W, H, border, qindex, rdmult, neighbour_starts=neighbours)
    out = tf.step()
    torch.cuda.synchronize()
    got = T.records_numpy(out)
    grec = tf.recon.cpu().numpy()
    gcost = tf.costs.cpu().numpy()
    st = src.shape[1]
    mvj, mvc = M.default_mv_cost_tables(tf.allow_hp)
    spb, epb = M.sad_per_bit(qindex), M.error_per_bit(rdmult)
    if neighbours:
        assert T.tpl_motion_failures(tf.mv_out) == 0
        _, fp, cl, _ = O.tpl_motion_search(src.reshape(-1), refs.reshape(-1), st, tf.jobs_np,
                                           W // 16, H // 16, R, "fast_bigdia", 6, False, 3, 2,
                                           spb, epb, mvj, mvc, 0)
    else:
        fp, cl = O.full_pixel_search_batch(src.reshape(-1), refs.reshape(-1), st, 16, 16,
                                           tf.jobs_np, "fast_bigdia", 6, 0, spb, epb, mvj, mvc,
                                           cost_list=True, threads=8)
    gfp = M.results_numpy(tf.fp)
    np.testing.assert_array_equal(gfp["best_row"], fp["best_row"])
    np.testing.assert_array_equal(gfp["best_col"], fp["best_col"])
    sj = M.subpel_jobs(W, H, T.TPL_BORDER, 16, 16, tf.jobs_np, fp)
    sub = O.subpel_search_batch(src.reshape(-1), refs.reshape(-1), st, 16, 16, sj, 2, M.FULL_PEL,
                                tf.allow_hp, 1, M.MV_COST_NONE, 0, None, None, cl, threads=8)
    np.testing.assert_array_equal(M.subpel_results_numpy(tf.sub)["best_row"], sub["best_row"])
    ij = np.concatenate([I.plane_jobs(W, H, 16, 16, (0, 0), ref_off=k * src.size, dst_stride=W)
                         for k in range(R)])
    for k in range(R):
        ij["dst_off"][k * len(ij) // R:(k + 1) * len(ij) // R] += k * W * H
    org = border * st + border
    preds = O.build_inter_pred(refs.reshape(-1, st), org, W, H, 0, 0, 16, 16, ij, (R, H, W),
                               mvs=sub, dst_stride=W)
    np.testing.assert_array_equal(tf.preds.cpu().numpy(), preds)
    exp, erec, ecost = O.tpl_block_batch(src[border:border + H, border:border + W], preds, 16, 8,
                                         qindex)
    np.testing.assert_array_equal(gcost, ecost)
    for f in exp.dtype.names:
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    np.testing.assert_array_equal(grec, erec)
    assert len(set(got["best_ref"])) > 1


@pytest.mark.parametrize("n", [8, 16, 32])
@pytest.mark.parametrize("bd", [8, 10, 12])
def test_tpl_block_batch_vs_reference(T, n, bd):
    """lavish_tpl_block_batch against tpl_get_satd_cost + txfm_quant_rdcost
    executed from the reference (tests/golden/fix_tpl.npz), the blocks of one
    qindex side by side in a plane.  No oracle in the loop."""
    import os
    F = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                  "fix_tpl.npz")))
    k = "%d_bd%d" % (n, bd)
    dt = np.uint8 if bd == 8 else np.uint16
    qs = F["q_" + k]
    for q in sorted(set(qs.tolist())):
        idx = np.nonzero(qs == q)[0]
        src = np.concatenate([F["src_" + k][i] for i in idx], axis=1).astype(dt)
        pred = np.concatenate([F["pred_" + k][i] for i in idx], axis=1).astype(dt)[None]
        got, grec, gcost = _run(T, src, pred, n, bd, int(q))
        exp = F["rec_" + k][idx]
        msg = "%s q %d" % (k, q)
        np.testing.assert_array_equal(got["inter_cost"], exp[:, 0], err_msg=msg)
        np.testing.assert_array_equal(got["rate_cost"], exp[:, 1], err_msg=msg)
        np.testing.assert_array_equal(got["recon_error"], exp[:, 2], err_msg=msg)
        np.testing.assert_array_equal(got["sse"], exp[:, 3], err_msg=msg)
        np.testing.assert_array_equal(
            grec, np.concatenate([F["recon_" + k][i] for i in idx], axis=1).astype(dt), err_msg=msg)
