"""GPU parity of lavish_optimize_b_batch (the coefficient trellis,
av1_optimize_b -> av1_optimize_txb):
  - against av1_optimize_b executed from the reference
    (tests/golden/fix_trellis.npz): rate, eob, txb_entropy_ctx, qcoeff and
    dqcoeff of every row, no oracle in the loop;
  - against the oracle restatement on large batches of av1_quant_batch's FP
    output (the use_optimize_b path), every tx-size family."""
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


def test_optimize_b_vs_reference():
    torch = _dev()
    import lavish_dsp as L
    from lavish_dsp import txb
    F = dict(np.load(os.path.join(GOLD, "fix_trellis.npz")))
    J = {n: i for i, n in enumerate(F["row_fields"])}
    costs = txb.CoeffCosts(txb.coeff_costs_blob(F["coeff_costs"], F["eob_costs"]))
    keys = ("bd", "tx_size", "tx_type", "qindex", "plane", "is_inter", "sharpness", "rdmult",
            "tx_type_cost")
    groups = {}
    for r in F["rows"]:
        groups.setdefault(tuple(int(r[J[k]]) for k in keys), []).append(r)
    n_checked = 0
    for (bd, s, t, qindex, plane, inter, sharp, rdmult, ttc), rows in groups.items():
        n = L.max_eob(s)
        idx = [int(r[J["index"]]) for r in rows]
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
        tc = dev(F["coeff"][idx][:, :n])
        qc = dev(F["qcoeff_in"][idx][:, :n])
        dq = dev(F["dqcoeff_in"][idx][:, :n])
        eob = dev(np.array([r[J["eob_in"]] for r in rows], np.int16))
        ctx = dev(np.array([[r[J["txb_skip_ctx"]], r[J["dc_sign_ctx"]]] for r in rows],
                           np.int32))
        dqv = O.quant_arrays(O.build_quant(bd, qindex))["dequant"]
        rate, ec = txb.optimize_b_batch(costs, tc, qc, dq, eob, s, t, bd, rdmult, dqv, plane,
                                        inter, sharp, ctx, ttc)
        torch.cuda.synchronize()
        msg = "bd %d size %d type %d q %d plane %d inter %d sharp %d" % (bd, s, t, qindex, plane,
                                                                           inter, sharp)
        np.testing.assert_array_equal(rate.cpu().numpy(), [r[J["rate"]] for r in rows], msg)
        np.testing.assert_array_equal(eob.cpu().numpy().view(np.uint16),
                                      [r[J["eob"]] for r in rows], msg)
        np.testing.assert_array_equal(ec.cpu().numpy(), [r[J["entropy_ctx"]] for r in rows], msg)
        np.testing.assert_array_equal(qc.cpu().numpy(), F["qcoeff"][idx][:, :n], msg)
        np.testing.assert_array_equal(dq.cpu().numpy(), F["dqcoeff"][idx][:, :n], msg)
        n_checked += len(rows)
    assert n_checked == len(F["rows"])


@pytest.mark.parametrize("s,t", [(0, 0), (0, 10), (1, 3), (2, 0), (2, 11), (3, 0), (3, 9),
                                 (4, 0), (7, 0), (9, 0), (13, 14), (16, 0), (17, 0)])
@pytest.mark.parametrize("bd,sharp", [(8, 0), (10, 0), (10, 2)])
def test_optimize_b_vs_oracle(s, t, bd, sharp):
    torch = _dev()
    import lavish_dsp as L
    from lavish_dsp import txb
    rng = np.random.default_rng(31 * s + t + bd + sharp)
    blob = rng.integers(30, 4000, txb.COEFF_COSTS_CELLS).astype(np.int32)
    costs = txb.CoeffCosts(blob)
    n = L.max_eob(s)
    nb = 512 if n >= 512 else 2048
    # sharpness > 0 scales the trellis rdmult down by 2^sharpness and only
    # lowers levels >= 2 (txb_rdopt.c:326-449): larger levels and a larger
    # rdmult make it act there too (every case below changes some blocks)
    scale, rdmult = (40, 1200) if sharp == 0 else (300, 1200 << 6)
    c = (rng.laplace(0, scale, (nb, n)) * np.exp(-np.arange(n) / (n / 5)) * (1 << (bd - 8)))
    c = c.astype(np.int32)
    qindex = 100
    pq = L.build_plane_quant(bd, qindex)
    qc, dq, eob, _ = L.av1_quant_batch(torch.from_numpy(c).cuda(), s, t, bd, pq, L.AV1_QUANT_FP)
    torch.cuda.synchronize()
    q0, d0, e0 = qc.cpu().numpy(), dq.cpu().numpy(), eob.cpu().numpy().view(np.uint16)
    ctx = np.stack([rng.integers(0, 13, nb), rng.integers(0, 3, nb)], 1).astype(np.int32)
    dqv = O.quant_arrays(O.build_quant(bd, qindex))["dequant"]
    rate, ec = txb.optimize_b_batch(costs, torch.from_numpy(c).cuda(), qc, dq, eob, s, t, bd,
                                    rdmult, dqv, 0, 1, sharp, torch.from_numpy(ctx).cuda(), 321)
    torch.cuda.synchronize()
    gq, gd, ge = qc.cpu().numpy(), dq.cpu().numpy(), eob.cpu().numpy().view(np.uint16)
    gr, gc = rate.cpu().numpy(), ec.cpu().numpy()
    changed = 0
    for b in range(nb):
        e, r, x, oq, od = O.optimize_b(blob, c[b], q0[b], d0[b], int(e0[b]), 0, s, t, bd, 1,
                                       rdmult, sharp, dqv, int(ctx[b, 0]), int(ctx[b, 1]), 321)
        assert (ge[b], gr[b], gc[b]) == (e, r, x), b
        np.testing.assert_array_equal(gq[b], oq)
        np.testing.assert_array_equal(gd[b], od)
        changed += int((oq != q0[b]).any())
    assert changed > 0
