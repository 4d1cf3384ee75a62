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


_lib.lavish_rdo_plane_rate.argtypes = [_vp, _vp, _i32, _i32, _i32, _i32, ctypes.c_uint32, _i32,
                                       _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
_lib.lavish_rdo_plane_rate.restype = _i32


def rdo_plane_rate(src, pred, tx_size, type_mask, qp, rdmult, costs, txb_ctx=None,
                   tx_type_costs=None, block_mask=None, block_map=None, bit_depth=10, out=None,
                   stream=None):
    """lavish_rdo_plane_rate: C4 (TX-domain distortion) ranked by the
    coefficient rate.  costs: CoeffCosts; txb_ctx: None or device int32
    [nblocks, 2]; tx_type_costs: None or 16 ints (get_tx_type_cost per type);
    masks as rdo_plane_masked."""
    import torch
    from . import TX_H, TX_W, rdo_out
    assert src.dtype == torch.int16 and pred.dtype == torch.int16
    assert src.is_cuda and pred.is_cuda and src.shape == pred.shape
    assert src.stride(1) == 1 and pred.stride(0) == src.stride(0)
    H, W = src.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    if txb_ctx is not None:
        assert txb_ctx.is_cuda and txb_ctx.dtype == torch.int32 and txb_ctx.is_contiguous()
        assert tuple(txb_ctx.shape) == (nb, 2)
    if block_mask is not None:
        assert block_mask.is_cuda and block_mask.dtype in (torch.int16, torch.uint16)
        assert block_mask.is_contiguous() and tuple(block_mask.shape) == (nb,)
    if block_map is not None:
        assert block_map.is_cuda and block_map.dtype == torch.uint8
        assert block_map.is_contiguous() and tuple(block_map.shape) == (nb, 16)
    ttc = None
    if tx_type_costs is not None:
        ttc = np.ascontiguousarray(tx_type_costs, np.int32)
        assert ttc.shape == (16,)
    if out is None:
        out = rdo_out(src, tx_size)
    p = lambda t: None if t is None else _vp(t.data_ptr())
    rc = _lib.lavish_rdo_plane_rate(
        _vp(src.data_ptr()), _vp(pred.data_ptr()), src.stride(0), W, H, tx_size, type_mask,
        bit_depth, ctypes.byref(qp), rdmult, _vp(costs.t.data_ptr()), p(txb_ctx),
        None if ttc is None else ttc.ctypes.data_as(_vp), p(block_mask), p(block_map),
        _vp(out["records"].data_ptr()), _vp(out["qcoeff"].data_ptr()),
        _vp(out["dqcoeff"].data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_rdo_plane_rate rejected its arguments (rc=%d)" % rc)
    return out


_lib.lavish_optimize_b_batch.argtypes = [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32,
                                         _i32, _i32, _i32, _vp, _vp, _i32, _vp, _vp, _vp]
_lib.lavish_optimize_b_batch.restype = _i32


def optimize_b_batch(costs, tcoeff, qcoeff, dqcoeff, eob, tx_size, tx_type, bit_depth, rdmult,
                     dequant, plane=0, is_inter=1, sharpness=0, txb_ctx=None, tx_type_cost=0,
                     rate=None, entropy_ctx=None, stream=None):
    """lavish_optimize_b_batch (av1_optimize_b): qcoeff / dqcoeff / eob are
    updated in place (device int32 [nblocks, n], int16 / uint16 [nblocks]);
    dequant = (dc, ac) dequantizer values.  Returns (rate, entropy_ctx)."""
    import torch
    n = max_eob(tx_size)
    for t in (tcoeff, qcoeff, dqcoeff):
        assert t.dtype == torch.int32 and t.is_contiguous() and t.shape[-1] == n and t.is_cuda
    nb = qcoeff.numel() // n
    assert tcoeff.numel() == qcoeff.numel() == dqcoeff.numel()
    assert eob.dtype in (torch.int16, torch.uint16) and eob.numel() >= nb and eob.is_cuda
    if txb_ctx is not None:
        assert txb_ctx.dtype == torch.int32 and txb_ctx.is_contiguous()
        assert txb_ctx.numel() >= 2 * nb and txb_ctx.is_cuda
    if rate is None:
        rate = torch.empty(nb, dtype=torch.int32, device=qcoeff.device)
    if entropy_ctx is None:
        entropy_ctx = torch.empty(nb, dtype=torch.uint8, device=qcoeff.device)
    dq = np.ascontiguousarray(dequant, np.int16)
    assert dq.shape == (2,)
    rc = _lib.lavish_optimize_b_batch(
        _vp(costs.t.data_ptr()), _vp(tcoeff.data_ptr()), _vp(qcoeff.data_ptr()),
        _vp(dqcoeff.data_ptr()), _vp(eob.data_ptr()), nb, plane, tx_size, tx_type, bit_depth,
        is_inter, rdmult, sharpness, dq.ctypes.data_as(_vp),
        _vp(txb_ctx.data_ptr()) if txb_ctx is not None else None, tx_type_cost,
        _vp(rate.data_ptr()), _vp(entropy_ctx.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_optimize_b_batch rejected its arguments (rc=%d)" % rc)
    return rate, entropy_ctx
