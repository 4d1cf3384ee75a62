"""GPU parity of lavish_cost_coeffs_txb_batch (the coefficient rate,
SURVEY.md 8(f) rank 4):
  - against av1_cost_coeffs_txb / av1_cost_coeffs_txb_laplacian executed from
    the reference (tests/golden/fix_costcoeffs.npz), every tx size, the three
    tx classes, luma / chroma, eob 0 / 1 / 2 / random / max;
  - against the oracle restatement on large random batches (per-block
    contexts, Golomb-range levels) and on av1_quant_batch's own output (the
    reference's order: av1_quant -> cost_coeffs)."""
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dev():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_cost_coeffs_vs_reference():
    torch = _dev()
    import lavish_dsp as L
    from lavish_dsp import txb
    F = dict(np.load(os.path.join(GOLD, "fix_costcoeffs.npz")))
    J = {n: i for i, n in enumerate(F["row_fields"])}
    costs = txb.CoeffCosts(txb.coeff_costs_blob(F["coeff_costs"], F["eob_costs"]))
    groups = {}
    for r in F["rows"]:
        key = tuple(int(r[J[k]]) for k in ("tx_size", "tx_type", "plane", "tx_type_cost"))
        groups.setdefault(key, []).append(r)
    n_checked = 0
    for (s, t, plane, ttc), rows in groups.items():
        n = L.max_eob(s)
        idx = [int(r[J["index"]]) for r in rows]
        q = torch.from_numpy(np.ascontiguousarray(F["qcoeff"][idx][:, :n])).cuda()
        eob = torch.from_numpy(np.array([r[J["eob"]] for r in rows], np.int16)).cuda()
        ctx = torch.from_numpy(np.array([[r[J["txb_skip_ctx"]], r[J["dc_sign_ctx"]]]
                                         for r in rows], np.int32)).cuda()
        msg = "size %d type %d plane %d" % (s, t, plane)
        for mode, col in ((txb.COEFF_RATE_EXACT, "rate"),
                          (txb.COEFF_RATE_LAPLACIAN, "rate_laplacian")):
            rate = txb.cost_coeffs_txb_batch(costs, q, eob, s, t, plane, ctx, ttc, mode)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(rate.cpu().numpy(), [r[J[col]] for r in rows],
                                          err_msg="%s %s" % (msg, col))
        n_checked += len(rows)
    assert n_checked == len(F["rows"])


def _random_blocks(rng, s, t, nb):
    """Random quantized blocks with a consistent eob (scan position after the
    last nonzero), eob 0 and max included."""
    import lavish_dsp as L
    n = L.max_eob(s)
    scan, _ = L.scan_order(s, t)
    q = np.zeros((nb, n), np.int32)
    eob = rng.integers(0, n + 1, nb)
    eob[0], eob[1 % nb], eob[2 % nb] = 0, n, 1
    # sparse levels, heavier at the start of the scan, a Golomb tail
    lv = rng.choice([0, 0, 0, 1, 1, 2, 3, 5, 9, 14, 15, 40, 200, 3000], size=(nb, n))
    sign = rng.choice([-1, 1], size=(nb, n))
    for b in range(nb):
        e = int(eob[b])
        if e == 0:
            continue
        v = (lv[b, :e] * sign[b, :e]).astype(np.int32)
        if v[e - 1] == 0:
            v[e - 1] = sign[b, e - 1] * (1 + b % 7)
        q[b, scan[:e]] = v
    return q, eob.astype(np.uint16)


@pytest.mark.parametrize("s,t,plane", [(0, 0, 0), (0, 10, 0), (1, 11, 1), (2, 3, 0),
                                       (2, 12, 0), (3, 0, 0), (3, 9, 1), (4, 0, 0), (5, 6, 0),
                                       (6, 15, 0), (9, 0, 1), (12, 0, 0), (13, 14, 0),
                                       (14, 13, 0), (15, 9, 0), (16, 0, 2), (17, 0, 0),
                                       (18, 0, 0)])
def test_cost_coeffs_vs_oracle_random(s, t, plane):
    torch = _dev()
    import lavish_dsp as L
    from lavish_dsp import txb
    rng = np.random.default_rng(1000 + 37 * s + t)
    blob = np.concatenate([rng.integers(0, 5000, 10 * txb.COEFF_COST_CELLS),
                           rng.integers(0, 5000, 14 * txb.EOB_COST_CELLS)]).astype(np.int32)
    costs = txb.CoeffCosts(blob)
    nb = 1500 if L.max_eob(s) >= 512 else 3000
    q, eob = _random_blocks(rng, s, t, nb)
    ctx = np.stack([rng.integers(0, 13, nb), rng.integers(0, 3, nb)], 1).astype(np.int32)
    qd = torch.from_numpy(q).cuda()
    ed = torch.from_numpy(eob.view(np.int16)).cuda()
    cd = torch.from_numpy(ctx).cuda()
    for lap in (False, True):
        want = O.cost_coeffs_txb_batch(blob, q, eob, plane, s, t, ctx, 777, lap)
        got = txb.cost_coeffs_txb_batch(costs, qd, ed, s, t, plane, cd, 777, int(lap))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy(), want, err_msg="lap %d" % lap)
    # no contexts: all {0, 0}
    want = O.cost_coeffs_txb_batch(blob, q, eob, plane, s, t, None, 0, False)
    got = txb.cost_coeffs_txb_batch(costs, qd, ed, s, t, plane)
    np.testing.assert_array_equal(got.cpu().numpy(), want)


def test_cost_coeffs_after_av1_quant():
    """av1_quant_batch -> cost_coeffs_txb_batch on the device, as
    search_tx_type runs them, against the oracle on the same qcoeff / eob."""
    torch = _dev()
    import lavish_dsp as L
    from lavish_dsp import txb
    rng = np.random.default_rng(77)
    blob = rng.integers(0, 4000, txb.COEFF_COSTS_CELLS).astype(np.int32)
    costs = txb.CoeffCosts(blob)
    for s, t in ((0, 0), (1, 3), (2, 0), (3, 0), (4, 0), (7, 10), (10, 9)):
        n = L.max_eob(s)
        c = (rng.laplace(0, 60, (2048, n)) * np.exp(-np.arange(n) / (n / 6))).astype(np.int32)
        cd = torch.from_numpy(c).cuda()
        pq = L.build_plane_quant(8, 100)
        qc, _, eob, _ = L.av1_quant_batch(cd, s, t, 8, pq, L.AV1_QUANT_FP)
        rate = txb.cost_coeffs_txb_batch(costs, qc, eob, s, t, 0, None, 123)
        torch.cuda.synchronize()
        qn, en = qc.cpu().numpy(), eob.cpu().numpy().view(np.uint16)
        assert (en > 0).any()
        want = O.cost_coeffs_txb_batch(blob, qn, en, 0, s, t, None, 123, False)
        np.testing.assert_array_equal(rate.cpu().numpy(), want, err_msg="size %d" % s)


def test_cost_coeffs_rejects():
    torch = _dev()
    from lavish_dsp import txb
    costs = txb.CoeffCosts(np.zeros(txb.COEFF_COSTS_CELLS, np.int32))
    q = torch.zeros((1, 16), dtype=torch.int32, device="cuda")
    e = torch.zeros(1, dtype=torch.int16, device="cuda")
    with pytest.raises(ValueError, match="rc=-4"):
        txb.cost_coeffs_txb_batch(costs, q, e, 0, 0, 0, mode=5)
    with pytest.raises(ValueError, match="rc=-2"):
        txb.cost_coeffs_txb_batch(costs, q, e, 0, 0, plane=3)
