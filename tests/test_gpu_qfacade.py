"""GPU parity of lavish_av1_quant_batch (av1_quant + search_tx_type's satd
gate) against skip_trellis_opt_based_on_satd + av1_quant
executed from the reference (tests/golden/fix_qfacade.npz): quantizer
chosen, use_optimize_b, qcoeff, dqcoeff, eob.  No oracle in the loop."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_av1_quant_batch_vs_reference():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp as L
    F = dict(np.load(os.path.join(GOLD, "fix_qfacade.npz")))
    J = {n: i for i, n in enumerate(F["row_fields"])}
    # blocks sharing every call parameter go in one batch (dc_only per block)
    groups = {}
    for r in F["rows"]:
        key = tuple(int(r[J[k]]) for k in ("bd", "tx_size", "tx_type", "qindex", "mode",
                                           "skip_trellis", "threshold", "qstep"))
        groups.setdefault(key, []).append(r)
    n_checked = 0
    for (bd, s, t, qindex, mode, st, thr, qstep), rows in groups.items():
        n = L.max_eob(s)
        idx = [int(r[J["index"]]) for r in rows]
        coeff = torch.from_numpy(np.ascontiguousarray(F["coeff"][idx][:, :n])).cuda()
        dc = torch.from_numpy(np.array([r[J["dc_only"]] for r in rows], np.uint8)).cuda()
        pq = L.build_plane_quant(bd, qindex)
        qc, dq, eob, flags = L.av1_quant_batch(coeff, s, t, bd, pq, mode, st, thr, qstep, dc)
        torch.cuda.synchronize()
        msg = "bd %d size %d q %d mode %d skip %d thr %d" % (bd, s, qindex, mode, st, thr)
        np.testing.assert_array_equal(flags.cpu().numpy(), [r[J["flags"]] for r in rows],
                                      err_msg=msg)
        np.testing.assert_array_equal(eob.cpu().numpy().view(np.uint16),
                                      [r[J["eob"]] for r in rows], err_msg=msg)
        np.testing.assert_array_equal(qc.cpu().numpy(), F["qcoeff"][idx][:, :n], err_msg=msg)
        np.testing.assert_array_equal(dq.cpu().numpy(), F["dqcoeff"][idx][:, :n], err_msg=msg)
        n_checked += len(rows)
    assert n_checked == len(F["rows"])


def test_av1_quant_batch_rejects():
    import torch
    import lavish_dsp as L
    c = torch.zeros((1, 16), dtype=torch.int32, device="cuda")
    pq = L.build_plane_quant(8, 10)
    with pytest.raises(ValueError, match="rc=-3"):
        L.av1_quant_batch(c, 0, 0, 8, pq, 7)
    with pytest.raises(ValueError, match="rc=-2"):
        L.av1_quant_batch(c, 0, 0, 9, pq, 0)
