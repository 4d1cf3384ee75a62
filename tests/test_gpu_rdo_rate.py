"""GPU parity of C4 ranked by the coefficient rate (lavish_rdo_plane_rate:
search_tx_type's cost_coeffs, av1_cost_coeffs_txb, instead of the TPL
rate_estimator) against the oracle (orc_rdo_plane_rate, whose rate is
orc_cost_coeffs_txb, pinned to the reference by fix_costcoeffs.npz): records
and the winner's coefficients bit-exact; the records' rate equals
lavish_cost_coeffs_txb_batch on the winner."""
import numpy as np
import pytest

import _oracle as O
from _c4ref import planes as _planes

pytestmark = pytest.mark.gpu

# the C4 candidate sets plus rectangular and 1-D-class sizes
CASES = [(0, 0xFFFF), (1, 0xFFFF), (2, 0xFFFF), (3, 0x201), (4, 0x1), (5, 0xFFFF), (6, 0xFFFF),
         (7, 0xFFFF), (9, 0x201), (11, 0x1), (13, 0xFFFF), (14, 0xFFFF), (16, 0x201),
         (17, 0x1), (18, 0x1)]


@pytest.fixture(scope="module")
def L():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp
    return lavish_dsp


def _tables(seed):
    """Cost tables in the magnitude av1_fill_coeff_costs produces (a few
    hundred to a few thousand 1/512-bit units)."""
    from lavish_dsp import txb
    rng = np.random.default_rng(seed)
    return rng.integers(30, 4000, txb.COEFF_COSTS_CELLS).astype(np.int32)


@pytest.mark.parametrize("s,tmask", CASES)
@pytest.mark.parametrize("bd", [10, 8])
def test_rdo_rate_vs_oracle(L, s, tmask, bd):
    import torch
    from lavish_dsp import txb
    src, pred = _planes(bd, 90 + s)
    nb = (src.shape[1] // O.TX_W[s]) * (src.shape[0] // O.TX_H[s])
    rng = np.random.default_rng(s * 3 + bd)
    blob = _tables(s + 100 * bd)
    ctx = np.stack([rng.integers(0, 13, nb), rng.integers(0, 3, nb)], 1).astype(np.int32)
    ttc = rng.integers(0, 3000, 16).astype(np.int32)
    q = O.build_quant(bd, 128)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    exp, eq, ed = O.rdo_plane_rate(src, pred, s, tmask, bd, q, 1500, blob, ctx, ttc, threads=8)
    costs = txb.CoeffCosts(blob)
    out = txb.rdo_plane_rate(torch.from_numpy(src.view(np.int16)).cuda(),
                             torch.from_numpy(pred.view(np.int16)).cuda(), s, tmask, qp, 1500,
                             costs, torch.from_numpy(ctx).cuda(), ttc, bit_depth=bd)
    got = L.rdo_records(out)
    for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), eq)
    np.testing.assert_array_equal(out["dqcoeff"].cpu().numpy(), ed)
    # the rate differs from the rate_estimator ranking somewhere
    plain, _, _ = O.rdo_plane(src, pred, s, tmask, bd, q, 1500, threads=8)
    assert (plain["rate"] != exp["rate"]).any()
    # the records' rate is the coefficient rate of the winner
    for t in np.unique(got["best_type"]):
        sel = np.nonzero(got["best_type"] == t)[0]
        qc = out["qcoeff"][torch.from_numpy(sel).cuda()].contiguous()
        eob = torch.from_numpy(got["eob"][sel].astype(np.int16)).cuda()
        c = torch.from_numpy(ctx[sel]).cuda()
        r = txb.cost_coeffs_txb_batch(costs, qc, eob, s, int(t), 0, c, int(ttc[t]))
        np.testing.assert_array_equal(r.cpu().numpy(), got["rate"][sel])


def test_rdo_rate_masked(L):
    """Per-block allowed masks / search orders with the coefficient rate."""
    import torch
    from lavish_dsp import txb
    bd, s = 10, 2
    src, pred = _planes(bd, 7)
    src[:32, :128] = pred[:32, :128]  # ties: the order decides
    nb = (src.shape[1] // 16) * (src.shape[0] // 16)
    rng = np.random.default_rng(5)
    masks = rng.integers(0, 1 << 16, size=nb).astype(np.uint16)
    masks[::7] = 0
    maps = np.stack([rng.permutation(16) for _ in range(nb)]).astype(np.uint8)
    blob = _tables(11)
    q = O.build_quant(bd, 128)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    exp, eq, ed = O.rdo_plane_rate(src, pred, s, 0xFFFF, bd, q, 1500, blob, None, None, masks,
                                   maps, threads=8)
    out = txb.rdo_plane_rate(torch.from_numpy(src.view(np.int16)).cuda(),
                             torch.from_numpy(pred.view(np.int16)).cuda(), s, 0xFFFF, qp, 1500,
                             txb.CoeffCosts(blob), block_mask=torch.from_numpy(
                                 masks.view(np.int16)).cuda(),
                             block_map=torch.from_numpy(maps).cuda(), bit_depth=bd)
    got = L.rdo_records(out)
    for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), eq)
