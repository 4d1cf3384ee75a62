"""C3 full-pixel DIAMOND motion search on the MI355X backend
(lavish_diamond_search_batch) plus the host-side job construction the
reference does per block before calling av1_full_pixel_search:
av1_set_mv_limits (av1/encoder/mcomp.h:225-258) and av1_set_mv_search_range
(av1/encoder/mcomp.c:206-234)."""
import ctypes

import numpy as np

from . import _lib, _stream_ptr

JOB_DTYPE = np.dtype([("src_off", "<i8"), ("ref_off", "<i8"), ("start_row", "<i2"),
                      ("start_col", "<i2"), ("ref_mv_row", "<i2"), ("ref_mv_col", "<i2"),
                      ("col_min", "<i2"), ("col_max", "<i2"), ("row_min", "<i2"),
                      ("row_max", "<i2")], align=True)
RESULT_DTYPE = np.dtype([("best_row", "<i2"), ("best_col", "<i2"), ("bestsme", "<i4"),
                         ("steps", "<i4"), ("searches", "<i4")], align=True)
assert JOB_DTYPE.itemsize == 32 and RESULT_DTYPE.itemsize == 16

MV_COST_L1_LOWRES, MV_COST_L1_MIDRES, MV_COST_L1_HDRES, MV_COST_NONE = 1, 2, 3, 4
MI_SIZE = 4
AOM_INTERP_EXTEND = 4
MAX_FULL_PEL_VAL = (1 << 10) - 1   # mcomp.h: (1 << (MAX_MVSEARCH_STEPS - 1)) - 1
MV_LOW, MV_UPP = -(1 << 14), 1 << 14

_vp, _i32 = ctypes.c_void_p, ctypes.c_int32
_lib.lavish_diamond_search_batch.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _i32, _i32,
                                             _i32, _i32, _vp, _vp]
_lib.lavish_diamond_search_batch.restype = _i32


def mv_limits(mi_rows, mi_cols, mi_row, mi_col, mi_height, mi_width, border, ref_mv=(0, 0)):
    """(col_min, col_max, row_min, row_max) as av1_set_mv_limits followed by
    av1_set_mv_search_range(ref_mv) (ref_mv in 1/8 pel, (row, col))."""
    e2 = 2 * AOM_INTERP_EXTEND
    row_min = max(-(mi_row * MI_SIZE + border - e2), -((mi_row + mi_height) * MI_SIZE + e2))
    row_max = min((mi_rows - mi_row - mi_height) * MI_SIZE + border - e2,
                  (mi_rows - mi_row) * MI_SIZE + e2)
    col_min = max(-(mi_col * MI_SIZE + border - e2), -((mi_col + mi_width) * MI_SIZE + e2))
    col_max = min((mi_cols - mi_col - mi_width) * MI_SIZE + border - e2,
                  (mi_cols - mi_col) * MI_SIZE + e2)
    r, c = ref_mv
    cmin = max(((c + 7) >> 3) - MAX_FULL_PEL_VAL, (MV_LOW >> 3) + 1)
    rmin = max(((r + 7) >> 3) - MAX_FULL_PEL_VAL, (MV_LOW >> 3) + 1)
    cmax = min((c >> 3) + MAX_FULL_PEL_VAL, (MV_UPP >> 3) - 1)
    rmax = min((r >> 3) + MAX_FULL_PEL_VAL, (MV_UPP >> 3) - 1)
    col_min, row_min = max(col_min, cmin), max(row_min, rmin)
    col_max, row_max = min(col_max, cmax), min(row_max, rmax)
    return col_min, max(col_min, col_max), row_min, max(row_min, row_max)


def frame_jobs(width, height, stride, border, plane_bytes, bw, bh, nrefs, ref_mv=(0, 0),
               start_mv=(0, 0)):
    """Jobs for every full bw x bh block of a width x height frame against
    each of nrefs padded reference planes (plane k at k * plane_bytes), in
    reference-major, raster block order.  Padded planes: origin at
    (border, border), `stride` bytes per row."""
    mi_rows = ((height + 7) & ~7) // MI_SIZE   # aligned to 8 px like mi_params
    mi_cols = ((width + 7) & ~7) // MI_SIZE
    nbx, nby = width // bw, height // bh
    n = nbx * nby
    one = np.zeros(n, JOB_DTYPE)
    ys = np.repeat(np.arange(nby) * bh, nbx)
    xs = np.tile(np.arange(nbx) * bw, nby)
    one["src_off"] = (ys + border) * stride + xs + border
    lim = np.array([mv_limits(mi_rows, mi_cols, y // MI_SIZE, x // MI_SIZE, bh // MI_SIZE,
                              bw // MI_SIZE, border, ref_mv) for y, x in zip(ys, xs)])
    one["col_min"], one["col_max"], one["row_min"], one["row_max"] = lim.T
    one["start_row"], one["start_col"] = start_mv
    one["ref_mv_row"], one["ref_mv_col"] = ref_mv
    jobs = np.concatenate([one] * nrefs)
    jobs["ref_off"] = np.concatenate([one["src_off"] + k * plane_bytes for k in range(nrefs)])
    return jobs


def to_device(arr, device="cuda"):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy()).to(device)


def diamond_search_batch(src, ref, w, h, jobs, step_param=0, mv_cost_type=MV_COST_L1_HDRES,
                         use_downsampled_sad=False, out=None, stream=None):
    """src: uint8 device tensor (padded plane, 2-D), ref: uint8 device tensor
    holding the reference planes (any shape, contiguous, same stride); jobs:
    device byte tensor of JOB_DTYPE records.  Returns a device byte tensor of
    RESULT_DTYPE records (view with results_numpy)."""
    import torch
    assert src.dtype == torch.uint8 and ref.dtype == torch.uint8
    assert src.is_contiguous() and ref.is_contiguous(), "planes must be C-contiguous"
    nj = jobs.numel() // JOB_DTYPE.itemsize
    if out is None:
        out = torch.empty(nj * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=src.device)
    rc = _lib.lavish_diamond_search_batch(_vp(src.data_ptr()), src.stride(0),
                                          _vp(ref.data_ptr()), src.stride(0), w, h,
                                          _vp(jobs.data_ptr()), nj, step_param, mv_cost_type,
                                          int(use_downsampled_sad), _vp(out.data_ptr()),
                                          _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_diamond_search_batch rejected its arguments (rc=%d)" % rc)
    return out


def results_numpy(out):
    return out.cpu().numpy().view(RESULT_DTYPE)
