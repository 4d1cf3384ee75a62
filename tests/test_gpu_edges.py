"""Edge cases on the GPU path, as the reference's tests exercise them: planes
with no full block, ragged planes (partial last tile / block row), empty job
lists, per-size maximum-magnitude residuals, and argument rejection (the
C ABI returns a negative code; the host wrappers raise)."""
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


def test_plane_without_full_blocks(L):
    import torch
    res = torch.zeros((12, 30), dtype=torch.int16, device="cuda")
    qp = L.build_quant_params(8, 128, L.QUANT_FP)
    out = L.txq_plane(res, 3, L.valid_type_mask(3), qp)  # 32x32 on a 30x12 plane
    assert out["qcoeff"].shape[1] == 0
    torch.cuda.synchronize()
    assert L.status()[0] == 0


@pytest.mark.parametrize("s", [0, 2, 5, 9, 16])
def test_ragged_plane_matches_oracle(L, s):
    """Width / height not multiples of the block size: only full blocks,
    and a partial last tile of blocks inside a wave."""
    import torch
    import lavish_dsp.synth as synth
    W, H = 100 + 3 * s, 70 + s
    res = synth.residual_plane(W, H, 8, seed=500 + s)
    mask = L.valid_type_mask(s)
    qp = L.build_quant_params(8, 100, L.QUANT_FP)
    out = L.txq_plane(torch.from_numpy(res).cuda(), s, mask, qp)
    qc, dq, eob = O.txq_plane(res, s, mask, O.build_quant(8, 100))
    np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), qc.transpose(1, 0, 2))
    np.testing.assert_array_equal(out["dqcoeff"].cpu().numpy(), dq.transpose(1, 0, 2))
    np.testing.assert_array_equal(out["eob"].cpu().numpy().view(np.uint16), eob.T)


@pytest.mark.parametrize("s", [0, 1, 2, 3, 9, 13])
def test_extreme_residuals(L, s):
    """+-255 checkerboards and constant +-255 / +-1023 blocks (the shapes
    the reference's max-input transform tests use) at 8 and 10 bits."""
    import torch
    W, H = L.TX_W[s], L.TX_H[s]
    for bd, lim in ((8, 255), (10, 1023)):
        tiles = []
        for v in (lim, -lim):
            tiles.append(np.full((H, W), v, np.int16))
            chk = np.indices((H, W)).sum(0) % 2
            tiles.append(np.where(chk == 0, v, -v).astype(np.int16))
        res = np.ascontiguousarray(np.concatenate(tiles, axis=1))
        mask = L.valid_type_mask(s)
        qp = L.build_quant_params(bd, 0, L.QUANT_FP)
        out = L.txq_plane(torch.from_numpy(res).cuda(), s, mask, qp, bit_depth=bd)
        qc, dq, eob = O.txq_plane(res, s, mask, O.build_quant(bd, 0), bd=bd)
        np.testing.assert_array_equal(out["qcoeff"].cpu().numpy(), qc.transpose(1, 0, 2))
        np.testing.assert_array_equal(out["dqcoeff"].cpu().numpy(), dq.transpose(1, 0, 2))


def test_empty_job_lists(L):
    import torch
    import lavish_dsp.motion as M
    src = torch.zeros((64, 64), dtype=torch.uint8, device="cuda")
    empty = torch.zeros(0, dtype=torch.uint8, device="cuda")
    M.diamond_search_batch(src, src, 16, 16, empty)
    M.subpel_search_batch(src, src, 16, 16, empty)
    dst = torch.zeros((16, 16), dtype=torch.int16, device="cuda")
    L.inv_txfm_add_batch(torch.zeros(256, dtype=torch.int32, device="cuda"), 2, empty, dst, 10)
    torch.cuda.synchronize()
    assert L.status()[0] == 0


def test_rejected_arguments(L):
    import torch
    res = torch.zeros((64, 64), dtype=torch.int16, device="cuda")
    qp = L.build_quant_params(8, 128, L.QUANT_FP)
    with pytest.raises(ValueError):
        L.txq_plane(res, 19, 1, qp)                  # no such TX size
    with pytest.raises(ValueError):
        L.txq_plane(res, 3, 1 << 4, qp)              # FLIPADST_DCT is not valid at 32x32
    with pytest.raises(ValueError):
        L.rdo_plane(res, res, 2, 1, qp, 100, 9)      # bit depth 9
    import lavish_dsp.motion as M
    src = torch.zeros((64, 64), dtype=torch.uint8, device="cuda")
    jobs = M.to_device(np.zeros(1, M.JOB_DTYPE))
    with pytest.raises(ValueError):
        M.diamond_search_batch(src, src, 12, 12, jobs)   # not an encoder block size
    with pytest.raises(ValueError):
        M.diamond_search_batch(src, src, 16, 16, jobs, mv_cost_type=0)  # MV_COST_ENTROPY
    sj = M.to_device(np.zeros(1, M.SUBPEL_JOB_DTYPE))
    with pytest.raises(ValueError):
        M.subpel_search_batch(src, src, 16, 16, sj, iters_per_step=3)
    torch.cuda.synchronize()
    assert L.status()[0] == 0
