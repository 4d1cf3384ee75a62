"""GPU parity of C4 with search_tx_type's per-block allowed_tx_mask and
search order (lavish_rdo_plane_masked) against the oracle's loop over
txk_map (oracle/oracle_rdo.c orc_rdo_plane_masked), and of the chained
device pipeline residual -> prune_tx_2D -> masked RDO."""
import json
import os

import numpy as np
import pytest

import _oracle as O
from _c4ref import planes as _planes

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
T = json.load(open(os.path.join(HERE, "golden", "ref_tables.json")))
NN, TH = T["tx_type_nn"], T["prune_2d_thresholds"]
AGGR = [None, (4, 1), (6, 3), (9, 6), (9, 6), (12, 9)]


@pytest.fixture(scope="module")
def L():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp
    return lavish_dsp


def _cmp(got, exp, eq, ed, out):
    for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), eq)
    np.testing.assert_array_equal(out["dqcoeff"].cpu().numpy(), ed)


@pytest.mark.parametrize("s", [0, 1, 2, 5, 7, 3])
@pytest.mark.parametrize("px", [False, True])
def test_masked_random_orders(L, s, px):
    """Random per-block masks and permuted search orders; flat regions make
    many types tie, so the order decides."""
    import torch
    bd = 10
    src, pred = _planes(bd, 60 + s)
    src[:32, :128] = pred[:32, :128]  # zero residual: every type ties
    src[32:48, :64] = pred[32:48, :64] + 3
    nb = (src.shape[1] // O.TX_W[s]) * (src.shape[0] // O.TX_H[s])
    rng = np.random.default_rng(s)
    masks = rng.integers(0, 1 << 16, size=nb).astype(np.uint16)
    masks[::7] = 0  # zero mask: DCT_DCT only
    maps = np.stack([rng.permutation(16) for _ in range(nb)]).astype(np.uint8)
    maps[::5, 12:] = 255  # orders that list fewer types
    q = O.build_quant(bd, 128)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    tmask = 0xFFFF if s != 3 else 0x0201
    exp, eq, ed = O.rdo_plane_masked(src, pred, s, tmask, bd, q, 1500, masks, maps, px,
                                     threads=8)
    out = L.rdo_plane_masked(torch.from_numpy(src.view(np.int16)).cuda(),
                             torch.from_numpy(pred.view(np.int16)).cuda(), s, tmask, qp, 1500,
                             torch.from_numpy(masks.view(np.int16)).cuda(),
                             torch.from_numpy(maps).cuda(), bd, px)
    got = L.rdo_records(out)
    live = exp["rdcost"] != np.iinfo(np.int64).max  # blocks left with an allowed type
    assert live.mean() > 0.5
    # every block, including the ones with no candidate (tmask 0x0201 leaves
    # many): TX_TYPE_INVALID, eob 0, INT64_MAX cost, zero coefficients
    if s == 3:
        assert (~live).sum() > 0
    assert (exp["best_type"][~live] == 255).all() and (exp["eob"][~live] == 0).all()
    _cmp(got, exp, eq, ed, out)


def test_dead_blocks_reconstruct(L):
    """Blocks without a candidate cost INT64_MAX: the SB sums saturate (no
    wrap), so such an SB never picks that size, as in the oracle."""
    import torch
    bd = 10
    src, pred = _planes(bd, 17)
    sizes = {3: 0x0201, 2: 0xFFFF}
    nb3 = (src.shape[1] // 32) * (src.shape[0] // 32)
    masks = np.full(nb3, 0x0002, np.uint16)  # ADST_DCT only: never in {DCT, IDTX}
    masks[::3] = 0
    q = O.build_quant(bd, 128)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    o3 = L.rdo_plane_masked(ts, tp, 3, sizes[3], qp, 1500,
                            torch.from_numpy(masks.view(np.int16)).cuda(), None, bd)
    o2 = L.rdo_plane(ts, tp, 2, sizes[2], qp, 1500, bd)
    e3, q3, d3 = O.rdo_plane_masked(src, pred, 3, sizes[3], bd, q, 1500, masks, None, threads=8)
    e2, q2, d2 = O.rdo_plane(src, pred, 2, sizes[2], bd, q, 1500, threads=8)
    _cmp(L.rdo_records(o3), e3, q3, d3, o3)
    recon = torch.empty_like(ts)
    sbt = torch.empty(((src.shape[1] + 63) // 64) * ((src.shape[0] + 63) // 64), dtype=torch.uint8,
                      device="cuda")
    L.rdo_reconstruct([3, 2], {3: o3, 2: o2}, tp, recon, sbt, bd)
    torch.cuda.synchronize()
    er, esb = O.rdo_reconstruct([3, 2], [e3, e2], [d3, d2], pred, bd)
    np.testing.assert_array_equal(sbt.cpu().numpy(), esb)
    np.testing.assert_array_equal(recon.cpu().numpy().view(np.uint16), er)
    assert (esb == 2).mean() > 0.5


def test_masked_null_equals_plain(L):
    import torch
    bd = 8
    src, pred = _planes(bd, 5)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    a = L.rdo_plane(torch.from_numpy(src.view(np.int16)).cuda(),
                    torch.from_numpy(pred.view(np.int16)).cuda(), 1, 0xFFFF, qp, 999, bd)
    b = L.rdo_plane_masked(torch.from_numpy(src.view(np.int16)).cuda(),
                           torch.from_numpy(pred.view(np.int16)).cuda(), 1, 0xFFFF, qp, 999,
                           None, None, bd)
    np.testing.assert_array_equal(L.rdo_records(a), L.rdo_records(b))


@pytest.mark.parametrize("s", [0, 1, 2, 5, 7])
@pytest.mark.parametrize("mode", [1, 4])
def test_prune_then_rdo_pipeline(L, s, mode):
    """residual -> lavish_prune_tx_2d_batch -> lavish_rdo_plane_masked on the
    device, vs the oracle's prune_tx_2D + search_tx_type loop."""
    import torch
    import lavish_dsp.txprune as P
    bd = 10
    src, pred = _planes(bd, 80 + s)
    res = (src.astype(np.int32) - pred.astype(np.int32)).astype(np.int16)
    set_type = 4  # EXT_TX_SET_DTT9_IDTX_1DDCT (inter, 16x16 and below)
    tmask = 0x0FFF  # that set's 12 types: the 9 DTT9 pairs, IDTX, V_DCT, H_DCT
    hc = P.nn_config(**{k: NN["hor"][s][k] for k in ("num_inputs", "num_outputs")},
                     hidden=NN["hor"][s]["hidden"], weights=NN["hor"][s]["weights"],
                     bias=NN["hor"][s]["bias"])
    vc = P.nn_config(**{k: NN["ver"][s][k] for k in ("num_inputs", "num_outputs")},
                     hidden=NN["ver"][s]["hidden"], weights=NN["ver"][s]["weights"],
                     bias=NN["ver"][s]["bias"])
    tsrc = torch.from_numpy(src.view(np.int16)).cuda()
    tpred = torch.from_numpy(pred.view(np.int16)).cuda()
    tres = torch.from_numpy(res).cuda()
    mask, maps = P.prune_tx_2d(tres, s, set_type, mode, hc, vc, allowed_default=tmask)
    qp = L.build_quant_params(bd, 128, L.QUANT_FP)
    out = L.rdo_plane_masked(tsrc, tpred, s, tmask, qp, 1800, mask, maps, bd)
    got = L.rdo_records(out)
    em, emap = O.prune_tx_2d(res, O.TX_W[s], O.TX_H[s], set_type, mode, TH[s], NN["hor"][s],
                             NN["ver"][s], None, tmask)
    np.testing.assert_array_equal(mask.cpu().numpy().view(np.uint16), em)
    np.testing.assert_array_equal(maps.cpu().numpy(), emap)
    q = O.build_quant(bd, 128)
    exp, eq, ed = O.rdo_plane_masked(src, pred, s, tmask, bd, q, 1800, em, emap, threads=8)
    _cmp(got, exp, eq, ed, out)
    # pruning removed candidates; the winner is always among the kept ones
    assert (em != tmask).mean() > 0.05
    assert all((int(m) >> int(t)) & 1 for m, t in zip(em, got["best_type"]))
