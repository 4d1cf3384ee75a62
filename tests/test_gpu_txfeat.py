"""GPU parity of the TX-pruning features (lavish_horver_correlation_batch,
lavish_tx_prune_features_batch, the av1_get_horver_correlation_full_hip shim)
against the oracle's restatement (oracle/oracle_txfeat.c).  Floating point:
the reference's own SIMD-vs-C test allows 1e-6 absolute
(test/horver_correlation_test.cc:70-73) and north_star 1 ULP; the GPU keeps the
reference's operation order with IEEE single precision, so the bar checked
here is both (and the values are expected to be identical)."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

SIZES = [(4, 4), (8, 8), (16, 16), (32, 32), (64, 64), (128, 128), (4, 16), (16, 4), (8, 32),
         (32, 8), (16, 64), (64, 16), (4, 8), (8, 4), (8, 16), (16, 8), (16, 32), (32, 16),
         (32, 64), (64, 32), (64, 128), (128, 64)]


def _ulp(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


@pytest.fixture(scope="module")
def L():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp
    return lavish_dsp


@pytest.mark.parametrize("w,h", SIZES)
def test_horver_batch_random(L, w, h):
    """The reference test's input: (Rand16 % 4096) - 2048, every block size."""
    import torch
    rng = np.random.default_rng(w * 131 + h)
    nbx, nby = max(1, 256 // w), max(1, 256 // h)
    res = rng.integers(-2048, 2048, size=(nby * h, nbx * w)).astype(np.int16)
    hc, vc = L.horver_correlation_batch(torch.from_numpy(res).cuda(), w, h)
    hc, vc = hc.cpu().numpy(), vc.cpu().numpy()
    W = res.shape[1]
    for b in range(nbx * nby):
        by, bx = divmod(b, nbx)
        blk = np.ascontiguousarray(res[by * h:(by + 1) * h, bx * w:(bx + 1) * w])
        eh, ev = O.horver_full(blk, w, w, h)
        assert abs(float(hc[b]) - float(eh)) <= 1e-6 and _ulp(hc[b], eh) <= 1, (b, hc[b], eh)
        assert abs(float(vc[b]) - float(ev)) <= 1e-6 and _ulp(vc[b], ev) <= 1, (b, vc[b], ev)
    assert W == nbx * w


@pytest.mark.parametrize("w,h", [(16, 16), (64, 64), (128, 128), (4, 8)])
def test_horver_shim_and_extremes(L, w, h):
    buf = np.full((128, 128), 4095, np.int16)  # ExtremeValues
    assert L.av1_get_horver_correlation_full(buf, 128, w, h) == (1.0, 1.0)
    rng = np.random.default_rng(7)
    buf = rng.integers(-2048, 2048, size=(128, 128)).astype(np.int16)
    got = L.av1_get_horver_correlation_full(buf, 128, w, h)
    exp = O.horver_full(buf, 128, w, h)
    assert _ulp(got[0], exp[0]) <= 1 and _ulp(got[1], exp[1]) <= 1


@pytest.mark.parametrize("s", [0, 1, 2, 5, 6, 7, 8, 13, 14, 3, 9, 16])
def test_tx_prune_features_plane(L, s):
    """Every TX size prune_tx_2D can see, on a synthetic residual plane with
    flat (zero-energy) blocks mixed in."""
    import torch
    import lavish_dsp.synth as synth
    res = synth.residual_plane(192, 96, 10, seed=40 + s)
    res[:32, :64] = 0
    res[32:48, 64:96] = 77
    hf, vf = L.tx_prune_features(torch.from_numpy(res).cuda(), s)
    ef, evf = O.tx_prune_features(res, L.TX_W[s], L.TX_H[s])
    hf, vf = hf.cpu().numpy(), vf.cpu().numpy()
    assert (_ulp(hf, ef) <= 1).all() and (_ulp(vf, evf) <= 1).all()
    np.testing.assert_allclose(hf, ef, rtol=0, atol=1e-6)
    np.testing.assert_allclose(vf, evf, rtol=0, atol=1e-6)
    # bit-exact in practice
    assert (hf.view(np.int32) == ef.view(np.int32)).mean() == 1.0
