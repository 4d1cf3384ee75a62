"""The coefficient rate on the MI355X backend:
lavish_cost_coeffs_txb_batch replaces av1_cost_coeffs_txb /
av1_cost_coeffs_txb_laplacian (av1/encoder/txb_rdopt.c:599-660) for a batch
of blocks of one (tx_size, tx_type, plane), against the MACROBLOCK's
coeff_costs tables (CoeffCosts, av1/encoder/block.h:806-811) held on the
device."""
import ctypes

import numpy as np

from . import _lib, _stream_ptr, max_eob

_vp, _i32 = ctypes.c_void_p, ctypes.c_int32

COEFF_RATE_EXACT = 0
COEFF_RATE_LAPLACIAN = 1
COEFF_COST_CELLS = 944  # int32 cells of one LV_MAP_COEFF_COST
EOB_COST_CELLS = 22     # LV_MAP_EOB_COST
COEFF_COSTS_CELLS = 10 * COEFF_COST_CELLS + 14 * EOB_COST_CELLS

_lib.lavish_cost_coeffs_txb_batch.argtypes = [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _i32,
                                              _i32, _vp, _vp]
_lib.lavish_cost_coeffs_txb_batch.restype = _i32


def coeff_costs_blob(coeff_costs, eob_costs):
    """CoeffCosts as one flat int32 array: coeff_costs [5][2] x 944 cells
    (txb_skip_cost, base_eob_cost, base_cost, eob_extra_cost, dc_sign_cost,
    lps_cost), then eob_costs [7][2] x 22."""
    a = np.ascontiguousarray(coeff_costs, np.int32).reshape(-1)
    b = np.ascontiguousarray(eob_costs, np.int32).reshape(-1)
    assert a.size == 10 * COEFF_COST_CELLS and b.size == 14 * EOB_COST_CELLS
    return np.concatenate([a, b])


class CoeffCosts:
    """MACROBLOCK::coeff_costs on the device (upload once per frame / cdf
    update)."""

    def __init__(self, blob, device="cuda"):
        import torch
        blob = np.ascontiguousarray(blob, np.int32).reshape(-1)
        assert blob.size == COEFF_COSTS_CELLS
        self.t = torch.from_numpy(blob).to(device)


def cost_coeffs_txb_batch(costs, qcoeff, eob, tx_size, tx_type, plane=0, txb_ctx=None,
                          tx_type_cost=0, mode=COEFF_RATE_EXACT, out=None, stream=None):
    """lavish_cost_coeffs_txb_batch.  qcoeff: device int32 [nblocks, n]
    (n = max_eob(tx_size)); eob: device int16/uint16 [nblocks]; txb_ctx:
    None or device int32 [nblocks, 2] (txb_skip_ctx, dc_sign_ctx).  Returns
    the int32 [nblocks] rates."""
    import torch
    n = max_eob(tx_size)
    assert qcoeff.dtype == torch.int32 and qcoeff.is_contiguous() and qcoeff.shape[-1] == n
    nb = qcoeff.numel() // n
    assert eob.dtype in (torch.int16, torch.uint16) and eob.numel() >= nb and eob.is_cuda
    if txb_ctx is not None:
        assert txb_ctx.dtype == torch.int32 and txb_ctx.is_contiguous()
        assert txb_ctx.numel() >= 2 * nb
    if out is None:
        out = torch.empty(nb, dtype=torch.int32, device=qcoeff.device)
    rc = _lib.lavish_cost_coeffs_txb_batch(
        _vp(costs.t.data_ptr()), _vp(qcoeff.data_ptr()), _vp(eob.data_ptr()), nb, plane,
        tx_size, tx_type, _vp(txb_ctx.data_ptr()) if txb_ctx is not None else None,
        tx_type_cost, mode, _vp(out.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_cost_coeffs_txb_batch rejected its arguments (rc=%d)" % rc)
    return out
