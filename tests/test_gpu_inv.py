"""GPU parity of the inverse transform + reconstruction (SURVEY.md section 8
row a17) against the oracle's inv_txfm2d_add restatement (oracle/oracle_inv.c,
pinned by tests/test_oracle_golden.py): every TX size x valid TX type, bit
depths 8/10/12, per-call shims (av1_inv_txfm2d_add_*, av1_inv_txfm_add,
av1_highbd_inv_txfm_add) and the batch API with mixed types per tile and
eob == 0 blocks, including coefficients at the clamp limits."""
import ctypes

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp
    return lavish_dsp


def _coeffs(rng, s, bd, kind):
    n = O.max_eob(s)
    if kind == "random":      # typical dequantized magnitudes
        c = rng.integers(-(1 << (bd + 3)), 1 << (bd + 3), size=n)
        c[rng.random(n) < 0.6] = 0
    elif kind == "extreme":   # beyond the bd+8 row clamp: exercises every clamp
        c = rng.choice([-(1 << (bd + 9)), (1 << (bd + 9)) - 1, 0], size=n)
    else:                     # DC only
        c = np.zeros(n, np.int64)
        c[0] = rng.integers(-(1 << (bd + 6)), 1 << (bd + 6))
    return c.astype(np.int32)


@pytest.mark.parametrize("s", list(range(19)))
def test_inv_txfm2d_add_shims(L, s):
    rng = np.random.default_rng(100 + s)
    W, H = O.TX_W[s], O.TX_H[s]
    for bd in (8, 10, 12):
        for t in range(16):
            if not O.type_valid(s, t):
                continue
            for kind in ("random", "extreme", "dc"):
                c = _coeffs(rng, s, bd, kind)
                dst = rng.integers(0, 1 << bd, size=(H, W + 5)).astype(np.uint16)
                exp = O.inv_txfm2d_add(c, dst, t, s, bd)
                got = dst.copy()
                L.av1_inv_txfm2d_add(s, c, got, W + 5, t, bd)
                np.testing.assert_array_equal(got, exp, err_msg="s=%d t=%d bd=%d %s"
                                              % (s, t, bd, kind))


@pytest.mark.parametrize("s", [0, 1, 2, 3, 4, 5, 9, 12, 13, 17])
def test_inv_txfm_add_txfmparam(L, s):
    rng = np.random.default_rng(7 + s)
    W, H = O.TX_W[s], O.TX_H[s]
    for t in range(16):
        if not O.type_valid(s, t):
            continue
        c = _coeffs(rng, s, 8, "random")
        dst8 = rng.integers(0, 256, size=(H, W)).astype(np.uint8)
        exp = O.inv_txfm2d_add(c, dst8.astype(np.uint16), t, s, 8).astype(np.uint8)
        p = L.TxfmParam(tx_type=t, tx_size=s, lossless=0, bd=8, is_hbd=0, tx_set_type=0, eob=1)
        got = dst8.copy()
        L.av1_inv_txfm_add(c, got, W, p)
        np.testing.assert_array_equal(got, exp)
        dst16 = rng.integers(0, 1024, size=(H, W)).astype(np.uint16)
        p = L.TxfmParam(tx_type=t, tx_size=s, lossless=0, bd=10, is_hbd=1, tx_set_type=0, eob=1)
        got = dst16.copy()
        L.av1_inv_txfm_add(c, got, W, p)
        np.testing.assert_array_equal(got, O.inv_txfm2d_add(c, dst16, t, s, 10))


@pytest.mark.parametrize("s", [0, 1, 2, 3, 4, 6, 8, 10, 11, 14, 15, 18])
@pytest.mark.parametrize("bd", [8, 10])
def test_inv_batch_mixed_types(L, s, bd):
    """Jobs over a plane, random valid type per block (tiles mix types: the
    waterfall path), 1/8 of the blocks with eob == 0 (must stay untouched)."""
    import torch
    rng = np.random.default_rng(s * 31 + bd)
    W, H = O.TX_W[s], O.TX_H[s]
    n = O.max_eob(s)
    PW, PH = 256, 128
    nbx, nby = PW // W, PH // H
    nj = nbx * nby
    plane = rng.integers(0, 1 << bd, size=(PH, PW)).astype(np.uint8 if bd == 8 else np.uint16)
    valid = [t for t in range(16) if O.type_valid(s, t)]
    jobs = np.zeros(nj, L.INV_JOB_DTYPE)
    coeff = np.concatenate([_coeffs(rng, s, bd, "random" if j % 5 else "extreme")
                            for j in range(nj)])
    order = rng.permutation(nj)   # blocks in a random order: no tile is raster-contiguous
    for j, blk in enumerate(order):
        by, bx = divmod(int(blk), nbx)
        jobs[j] = (by * H * PW + bx * W, j * n, valid[rng.integers(len(valid))],
                   0 if rng.random() < 0.125 else 1)
    exp = plane.astype(np.uint16).copy()
    for j in range(nj):
        if jobs["eob"][j] == 0:
            continue
        off = int(jobs["dst_off"][j])
        y, x = divmod(off, PW)
        blk = exp[y:y + H, x:x + W].copy()
        exp[y:y + H, x:x + W] = O.inv_txfm2d_add(coeff[j * n:(j + 1) * n], blk,
                                                 int(jobs["tx_type"][j]), s, bd)
    tplane = torch.from_numpy(plane.view(np.int16) if bd > 8 else plane).cuda()
    L.inv_txfm_add_batch(torch.from_numpy(coeff).cuda(), s,
                         torch.from_numpy(jobs.view(np.uint8).copy()).cuda(), tplane, bd)
    got = tplane.cpu().numpy()
    got = got.view(np.uint16) if bd > 8 else got.astype(np.uint16)
    np.testing.assert_array_equal(got, exp)
