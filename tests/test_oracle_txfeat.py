"""CPU checks of the oracle's TX-pruning features (oracle/oracle_txfeat.c):
av1_get_horver_correlation_full and get_energy_distribution_finer.  The
reference's test (test/horver_correlation_test.cc) compares SIMD against C
only, so the restatement is pinned by known answers: flat blocks and the
test's ExtremeValues input (all 4095) take the zero-variance branch (1.0),
rows that repeat give a vertical correlation of 1, a horizontal ramp a
horizontal correlation of 1, a checkerboard 0 (clamped), and the energy
projection of a uniform block is uniform."""
import numpy as np
import pytest

import _oracle as O

SIZES = [(4, 4), (8, 8), (16, 16), (32, 32), (64, 64), (128, 128), (4, 16), (16, 4), (8, 32),
         (32, 8), (16, 64), (64, 16), (4, 8), (8, 4), (8, 16), (16, 8), (16, 32), (32, 16),
         (32, 64), (64, 32), (64, 128), (128, 64)]


@pytest.mark.parametrize("w,h", SIZES)
def test_horver_known_answers(w, h):
    flat = np.full((h, 128), 4095, np.int16)                      # ExtremeValues
    assert O.horver_full(flat, 128, w, h) == (1.0, 1.0)
    rows = np.tile(np.arange(128, dtype=np.int16) * 7 - 300, (h, 1))
    hc, vc = O.horver_full(rows, 128, w, h)
    assert vc == 1.0 and abs(hc - 1.0) <= 1e-6                   # repeated rows, ramp
    chk = np.where(np.indices((h, 128)).sum(0) % 2 == 0, 1000, -1000).astype(np.int16)
    hc, vc = O.horver_full(chk, 128, w, h)
    assert hc == 0.0 and vc == 0.0                                # anti-correlated -> 0


def test_energy_distribution_uniform_and_zero():
    for bw, bh in ((4, 4), (8, 8), (16, 16), (8, 16), (16, 4)):
        ew, eh = (bw if bw <= 8 else bw // 2), (bh if bh <= 8 else bh // 2)
        hf, vf = O.tx_prune_features(np.full((bh, bw), 9, np.int16), bw, bh)
        np.testing.assert_allclose(hf[0, :ew - 1], 1.0 / ew, rtol=1e-6)
        np.testing.assert_allclose(vf[0, :eh - 1], 1.0 / eh, rtol=1e-6)
        hz, vz = O.tx_prune_features(np.zeros((bh, bw), np.int16), bw, bh)
        np.testing.assert_array_equal(hz[0, :ew - 1], np.float32(1.0) / np.float32(ew))
        assert hz[0, ew - 1] == 1.0 and vz[0, eh - 1] == 1.0     # zero variance
        assert (hz[0, ew:] == 0).all() and (vz[0, eh:] == 0).all()


def test_random_features_in_range():
    rng = np.random.default_rng(3)
    res = rng.integers(-2048, 2048, size=(64, 64)).astype(np.int16)
    hf, vf = O.tx_prune_features(res, 16, 16)
    assert ((hf[:, 7] >= 0) & (hf[:, 7] <= 1.0000001)).all()
    assert (hf[:, :7].sum(1) < 1).all() and (hf[:, :7] >= 0).all()
