"""GPU parity of prune_tx_2D (lavish_prune_tx_2d_batch), av1_nn_predict_c
batches and the av1_nn_predict shim against the oracle's restatement
(oracle/oracle_txfeat.c), on the reference's own models and thresholds
(tests/golden/ref_tables.json): masks and search orders bit-exact, network
outputs bit-exact (single precision, same operation order; the tolerance is
0 ULP)."""
import json
import os

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
T = json.load(open(os.path.join(HERE, "golden", "ref_tables.json")))
NN, TH = T["tx_type_nn"], T["prune_2d_thresholds"]
MODEL_SIZES = [s for s in range(19) if NN["hor"][s] is not None]
TXW = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
TXH = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]
AGGR = [None, (4, 1), (6, 3), (9, 6), (9, 6), (12, 9)]


def _cfg(d):
    import lavish_dsp.txprune as P
    return P.nn_config(d["num_inputs"], d["num_outputs"], d["hidden"], d["weights"], d["bias"])


def _plane(W, H, seed, lim=200):
    rng = np.random.default_rng(seed)
    res = rng.integers(-lim, lim + 1, size=(H, W)).astype(np.int16)
    # smooth / structured blocks too: horizontal and vertical ramps, flat, zero
    res[:H // 4, :] = (np.arange(W)[None, :] % 37 - 18).astype(np.int16)
    res[H // 4:H // 2, :W // 2] = (np.arange(H // 4)[:, None] % 23 - 11).astype(np.int16)
    res[H // 2:H // 2 + 8, W // 2:] = 0
    return res


def _run(s, set_type, mode, seed, masks=True):
    import torch
    import lavish_dsp.txprune as P
    bw, bh = TXW[s], TXH[s]
    W, H = bw * 16, bh * 16
    res = _plane(W, H, seed)
    nb = (W // bw) * (H // bh)
    rng = np.random.default_rng(seed + 1)
    ain = rng.integers(1, 1 << 16, size=nb).astype(np.uint16) if masks else None
    hc, vc = _cfg(NN["hor"][s]), _cfg(NN["ver"][s])
    tain = None if ain is None else torch.from_numpy(ain.view(np.int16)).cuda()
    out, maps = P.prune_tx_2d(torch.from_numpy(res).cuda(), s, set_type, mode, hc, vc, tain)
    torch.cuda.synchronize()
    eo, em = O.prune_tx_2d(res, bw, bh, set_type, mode, TH[s], NN["hor"][s], NN["ver"][s], ain)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), eo)
    np.testing.assert_array_equal(maps.cpu().numpy(), em)
    return eo, ain


@pytest.mark.parametrize("s", MODEL_SIZES)
@pytest.mark.parametrize("set_type,mode", [(5, 1), (5, 2), (5, 3), (5, 4), (5, 5), (4, 1),
                                           (4, 3), (4, 4), (4, 5)])
def test_prune_tx_2d(s, set_type, mode):
    if set_type == 5 and s == 2 and AGGR[mode][0] >= len(TH[s]):
        pytest.skip("16x16 has no EXT_TX_SET_ALL16 threshold at this aggressiveness")
    eo, ain = _run(s, set_type, mode, seed=s * 31 + set_type * 7 + mode)
    assert ((eo & ~ain) == 0).all() and (eo != 0).all()
    assert (eo != ain).mean() > 0.2  # it prunes


@pytest.mark.parametrize("s", [0, 2, 7])
def test_prune_default_mask(s):
    _run(s, 4, 4, seed=5 + s, masks=False)


def test_prune_passthrough_and_rejects():
    import torch
    import lavish_dsp.txprune as P
    res = torch.from_numpy(_plane(64, 64, 3)).cuda()
    hc, vc = _cfg(NN["hor"][0]), _cfg(NN["ver"][0])
    for st, md, h, v in ((3, 2, hc, vc), (5, 0, hc, vc), (5, 2, None, None)):
        out, maps = P.prune_tx_2d(res, 0, st, md, h, v, allowed_default=0x0F0F)
        assert (out.cpu().numpy().view(np.uint16) == 0x0F0F).all()
        assert (maps.cpu().numpy() == np.arange(16)).all()
    with pytest.raises(ValueError):  # 16x16 with ALL16 at mode 5: beyond the threshold row
        P.prune_tx_2d(res, 2, 5, 5, _cfg(NN["hor"][2]), _cfg(NN["ver"][2]))
    with pytest.raises(ValueError):  # model with 2 outputs
        bad = P.nn_config(4, 2, [8], [np.zeros(32), np.zeros(16)], [np.zeros(8), np.zeros(2)])
        P.prune_tx_2d(res, 0, 5, 1, bad, bad)


@pytest.mark.parametrize("s", MODEL_SIZES)
@pytest.mark.parametrize("d", ["hor", "ver"])
def test_nn_predict_batch_and_shim(s, d):
    import torch
    import lavish_dsp.txprune as P
    cfg = NN[d][s]
    c = _cfg(cfg)
    rng = np.random.default_rng(s * 2 + (d == "ver"))
    x = rng.random((300, cfg["num_inputs"])).astype(np.float32)
    for rp in (True, False):
        got = P.nn_predict_batch(torch.from_numpy(x).cuda(), c, rp).cpu().numpy()
        exp = np.stack([O.nn_predict(v, cfg, rp) for v in x])
        np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(P.av1_nn_predict(x[0], c, True), O.nn_predict(x[0], cfg, True))


def test_nn_predict_deep_random_model():
    # a 3-hidden-layer model with 128-wide layers (the NN_MAX bounds)
    import torch
    import lavish_dsp.txprune as P
    rng = np.random.default_rng(77)
    sizes = [20, 128, 64, 128, 7]
    w = [rng.standard_normal(sizes[i] * sizes[i + 1]).astype(np.float32) * 0.2
         for i in range(4)]
    b = [rng.standard_normal(sizes[i + 1]).astype(np.float32) * 0.1 for i in range(4)]
    cfgd = {"num_inputs": 20, "num_outputs": 7, "hidden": [128, 64, 128], "weights": w, "bias": b}
    c = P.nn_config(20, 7, [128, 64, 128], w, b)
    x = rng.standard_normal((64, 20)).astype(np.float32)
    got = P.nn_predict_batch(torch.from_numpy(x).cuda(), c, False).cpu().numpy()
    exp = np.stack([O.nn_predict(v, O.nn_config(cfgd), False) for v in x])
    np.testing.assert_array_equal(got, exp)
