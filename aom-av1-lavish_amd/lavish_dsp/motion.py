"""C3 full-pixel DIAMOND motion search and the sub-pixel refinement that
follows it on the MI355X backend (lavish_diamond_search_batch,
lavish_subpel_search_batch) plus the host-side job construction the
reference does per block: av1_set_mv_limits (av1/encoder/mcomp.h:225-258),
av1_set_mv_search_range (av1/encoder/mcomp.c:206-234) and
av1_set_subpel_mv_search_range (av1/encoder/mcomp.h:357-373)."""
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

MV_COST_ENTROPY, MV_COST_L1_LOWRES, MV_COST_L1_MIDRES, MV_COST_L1_HDRES, MV_COST_NONE = range(5)
# SEARCH_METHODS (av1/encoder/mcomp_structs.h:56-86) the full-pel search takes
# (all of them but CLAMPED_DIAMOND)
SEARCH_METHODS = {"diamond": 0, "nstep": 1, "nstep_8pt": 2, "hex": 4, "bigdia": 5, "square": 6,
                  "fast_hex": 7, "fast_diamond": 8, "fast_bigdia": 9, "vfast_diamond": 10}
MV_MAX = (1 << 14) - 1
MI_SIZE = 4
AOM_INTERP_EXTEND = 4
MAX_FULL_PEL_VAL = (1 << 10) - 1   # mcomp.h: (1 << (MAX_MVSEARCH_STEPS - 1)) - 1
MV_LOW, MV_UPP = -(1 << 14), 1 << 14

_vp, _i32 = ctypes.c_void_p, ctypes.c_int32
_lib.lavish_diamond_search_batch.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _i32, _i32,
                                             _i32, _i32, _vp, _vp]
_lib.lavish_diamond_search_batch.restype = _i32
_lib.lavish_fast_bigdia_search_batch.argtypes = _lib.lavish_diamond_search_batch.argtypes
_lib.lavish_fast_bigdia_search_batch.restype = _i32


class MvCostParams(ctypes.Structure):
    """LavishMvCostParams: MV_COST_PARAMS with device table pointers."""
    _fields_ = [("mv_cost_type", ctypes.c_int32), ("sad_per_bit", ctypes.c_int32),
                ("error_per_bit", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("mvjcost", ctypes.c_void_p), ("mvcost", ctypes.c_void_p * 2)]


_lib.lavish_full_pixel_search_batch.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _i32,
                                                _i32, _i32, ctypes.POINTER(MvCostParams), _i32,
                                                _vp, _vp, _vp]
_lib.lavish_full_pixel_search_batch.restype = _i32


class RefTilesDesc(ctypes.Structure):
    """LavishRefTiles (include/lavish_dsp.h)."""
    _fields_ = [("data", ctypes.c_void_p), ("field_bytes", ctypes.c_int64),
                ("field_rows", ctypes.c_int32), ("stride", ctypes.c_int32)]


_lib.lavish_ref_tiles_bytes.argtypes = [_i32, _i32]
_lib.lavish_ref_tiles_bytes.restype = ctypes.c_int64
_lib.lavish_ref_tiles_build.argtypes = [_vp, _i32, _i32, _vp, ctypes.POINTER(RefTilesDesc), _vp]
_lib.lavish_ref_tiles_build.restype = _i32
_lib.lavish_full_pixel_search_batch_tiled.argtypes = [
    _vp, _i32, _vp, _i32, ctypes.POINTER(RefTilesDesc), _i32, _i32, _vp, _i32, _i32, _i32,
    ctypes.POINTER(MvCostParams), _i32, _vp, _vp, _vp]
_lib.lavish_full_pixel_search_batch_tiled.restype = _i32


class MeshParams(ctypes.Structure):
    """LavishMeshParams: the mesh fields of FULLPEL_MOTION_SEARCH_PARAMS
    (av1/encoder/mcomp.h:114-123) and the pattern set mesh_patterns
    [is_intra_mode] as (range, interval) pairs."""
    _fields_ = [("run_mesh_search", ctypes.c_int32), ("force_mesh_thresh", ctypes.c_int32),
                ("prune_mesh_search", ctypes.c_int32),
                ("mesh_search_mv_diff_threshold", ctypes.c_int32),
                ("fine_search_interval", ctypes.c_int32), ("is_intra_mode", ctypes.c_int32),
                ("range", ctypes.c_int32 * 4), ("interval", ctypes.c_int32 * 4)]

    @classmethod
    def make(cls, patterns, run_mesh_search=0, force_mesh_thresh=0x7FFFFFFF,
             prune_mesh_search=0, mesh_search_mv_diff_threshold=4, fine_search_interval=0,
             is_intra_mode=0):
        m = cls(run_mesh_search, force_mesh_thresh, prune_mesh_search,
                mesh_search_mv_diff_threshold, fine_search_interval, is_intra_mode)
        for i, (r, iv) in enumerate(patterns):
            m.range[i], m.interval[i] = r, iv
        return m


_lib.lavish_full_pixel_search_batch_mesh.argtypes = [
    _vp, _i32, _vp, _i32, ctypes.POINTER(RefTilesDesc), _i32, _i32, _vp, _i32, _i32, _i32,
    ctypes.POINTER(MvCostParams), _i32, ctypes.POINTER(MeshParams), _vp, _vp, _vp]
_lib.lavish_full_pixel_search_batch_mesh.restype = _i32
if hasattr(_lib, "lavish_set_search_workgroup_cap"):  # (older experiment builds lack it)
    _lib.lavish_set_search_workgroup_cap.argtypes = [_i32]
    _lib.lavish_set_search_workgroup_cap.restype = _i32
if hasattr(_lib, "lavish_set_search_schedule"):
    _lib.lavish_set_search_schedule.argtypes = [_i32]
    _lib.lavish_set_search_schedule.restype = _i32


class RefTiles:
    """The searches' candidate-row copy of a device u8 reference buffer
    (lavish_ref_tiles_build): every row of `ref` viewed as rows x stride.
    build() refreshes it (asynchronously, on `stream`) after the buffer
    changes."""

    def __init__(self, ref, stride=None):
        import torch
        assert ref.dtype == torch.uint8 and ref.is_contiguous()
        self.ref = ref
        self.stride = int(stride if stride is not None else ref.shape[-1])
        self.rows = ref.numel() // self.stride
        n = _lib.lavish_ref_tiles_bytes(self.stride, self.rows)
        if n <= 0:
            raise ValueError("lavish_ref_tiles_bytes rejected (%d, %d)" % (self.stride, self.rows))
        self.data = torch.empty(n, dtype=torch.uint8, device=ref.device)
        self.desc = RefTilesDesc()

    def build(self, stream=None):
        rc = _lib.lavish_ref_tiles_build(_vp(self.ref.data_ptr()), self.stride, self.rows,
                                         _vp(self.data.data_ptr()), ctypes.byref(self.desc),
                                         _stream_ptr(stream))
        if rc != 0:
            raise ValueError("lavish_ref_tiles_build rejected its arguments (rc=%d)" % rc)
        return self


class MvCosts:
    """Device copy of an nmv cost context (x->mv_costs): mvjcost int32[4] and
    mvcost int32[2][2 * MV_MAX + 1] as av1_build_nmv_cost_table lays them
    out; cost_params() makes the LavishMvCostParams for a search."""

    def __init__(self, mvjcost, mvcost, device="cuda"):
        import torch
        mvcost = np.ascontiguousarray(mvcost, np.int32)
        if mvcost.shape != (2, 2 * MV_MAX + 1) or np.shape(mvjcost) != (4,):
            raise ValueError("mvjcost[4] and mvcost[2][%d] expected" % (2 * MV_MAX + 1))
        self.mvjcost = torch.from_numpy(np.ascontiguousarray(mvjcost, np.int32)).to(device)
        self.mvcost = torch.from_numpy(mvcost).to(device)

    def cost_params(self, sad_per_bit, error_per_bit, mv_cost_type=MV_COST_ENTROPY):
        c = MvCostParams(mv_cost_type, sad_per_bit, error_per_bit, 0)
        c.mvjcost = self.mvjcost.data_ptr()
        row = self.mvcost.stride(0) * 4
        c.mvcost[0] = self.mvcost.data_ptr() + 4 * MV_MAX
        c.mvcost[1] = self.mvcost.data_ptr() + row + 4 * MV_MAX
        c._owner = self  # the device tables live as long as the parameters
        return c


def set_search_workgroup_cap(workgroups):
    """lavish_set_search_workgroup_cap: at most `workgroups` workgroups for
    the 16x16 DIAMOND search (0: no cap) -- a scheduling knob for running the
    search beside other streams' work; results do not depend on it."""
    rc = _lib.lavish_set_search_workgroup_cap(int(workgroups))
    if rc:
        raise ValueError("lavish_set_search_workgroup_cap(%r): %d" % (workgroups, rc))


def set_search_schedule(queued):
    """lavish_set_search_schedule: a capped search pulls its wave units from
    per-XCD queues (True, the default) or strides statically (False);
    results do not depend on it."""
    rc = _lib.lavish_set_search_schedule(1 if queued else 0)
    if rc:
        raise ValueError("lavish_set_search_schedule(%r): %d" % (queued, rc))


def default_mv_cost_tables(allow_hp=False):
    """(mvjcost[4], mvcost[2][2 * MV_MAX + 1]) of av1_build_nmv_cost_table over
    the default nmv context at the frame's mv precision (package data made by
    tests/golden/gen_fixtures.py nmv from the reference's own function)."""
    import os
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data",
                             "nmv_cost_default.npz"))
    t = "hp" if allow_hp else "lp"
    return d["mvjcost_" + t], d["mvcost_" + t]


def sad_per_bit(qindex, bit_depth=8):
    """av1_set_sad_per_bit (av1/encoder/rd.c:336-346, 507-513):
    (int)(0.0418 * q + 2.4107), q = av1_convert_qindex_to_q = ac_quant / 4."""
    from . import build_quant_params
    q = int(build_quant_params(bit_depth, qindex).dequant[1]) / 4.0
    if bit_depth == 10:
        q /= 4.0
    elif bit_depth == 12:
        q /= 16.0
    return int(0.0418 * q + 2.4107)


def error_per_bit(rdmult):
    """av1_set_error_per_bit (av1/encoder/rd.h:305-307)."""
    return max(rdmult >> 6, 1)


def l1_cost_params(mv_cost_type=MV_COST_L1_HDRES):
    return MvCostParams(mv_cost_type, 0, 0, 0)


def block_mv_limits(mi_rows, mi_cols, mi_row, mi_col, mi_height, mi_width, border):
    """x->mv_limits: (col_min, col_max, row_min, row_max) of av1_set_mv_limits
    (full pel)."""
    e2 = 2 * AOM_INTERP_EXTEND
    row_min = max(-(mi_row * MI_SIZE + border - e2), -((mi_row + mi_height) * MI_SIZE + e2))
    row_max = min((mi_rows - mi_row - mi_height) * MI_SIZE + border - e2,
                  (mi_rows - mi_row) * MI_SIZE + e2)
    col_min = max(-(mi_col * MI_SIZE + border - e2), -((mi_col + mi_width) * MI_SIZE + e2))
    col_max = min((mi_cols - mi_col - mi_width) * MI_SIZE + border - e2,
                  (mi_cols - mi_col) * MI_SIZE + e2)
    return col_min, col_max, row_min, row_max


def subpel_limits(lim, ref_mv=(0, 0)):
    """av1_set_subpel_mv_search_range (mcomp.h:357-373): SubpelMvLimits (1/8
    pel) from x->mv_limits and ref_mv ((row, col), 1/8 pel)."""
    col_min, col_max, row_min, row_max = lim
    max_mv = MAX_FULL_PEL_VAL * 8
    r, c = ref_mv
    minc = max(col_min * 8, c - max_mv)
    maxc = min(col_max * 8, c + max_mv)
    minr = max(row_min * 8, r - max_mv)
    maxr = min(row_max * 8, r + max_mv)
    maxc, maxr = max(minc, maxc), max(minr, maxr)
    return (max(MV_LOW + 1, minc), min(MV_UPP - 1, maxc), max(MV_LOW + 1, minr),
            min(MV_UPP - 1, maxr))


def mv_limits(mi_rows, mi_cols, mi_row, mi_col, mi_height, mi_width, border, ref_mv=(0, 0)):
    """(col_min, col_max, row_min, row_max) as av1_set_mv_limits followed by
    av1_set_mv_search_range(ref_mv) (ref_mv in 1/8 pel, (row, col))."""
    col_min, col_max, row_min, row_max = block_mv_limits(mi_rows, mi_cols, mi_row, mi_col,
                                                         mi_height, mi_width, border)
    r, c = ref_mv
    cmin = max(((c + 7) >> 3) - MAX_FULL_PEL_VAL, (MV_LOW >> 3) + 1)
    rmin = max(((r + 7) >> 3) - MAX_FULL_PEL_VAL, (MV_LOW >> 3) + 1)
    cmax = min((c >> 3) + MAX_FULL_PEL_VAL, (MV_UPP >> 3) - 1)
    rmax = min((r >> 3) + MAX_FULL_PEL_VAL, (MV_UPP >> 3) - 1)
    col_min, row_min = max(col_min, cmin), max(row_min, rmin)
    col_max, row_max = min(col_max, cmax), min(row_max, rmax)
    return col_min, max(col_min, col_max), row_min, max(row_min, row_max)


def frame_jobs(width, height, stride, border, plane_bytes, bw, bh, nrefs, ref_mv=(0, 0),
               start_mv=(0, 0), mv_border=None):
    """Jobs for every full bw x bh block of a width x height frame against
    each of nrefs padded reference planes (plane k at k * plane_bytes), in
    reference-major, raster block order.  Padded planes: origin at
    (border, border), `stride` bytes per row.  mv_border: the border the mv
    limits allow (av1_set_mv_limits; default the padding, TPL uses
    tpl_data->border_in_pixels = 32, tpl_model.c:155-156)."""
    mi_rows = ((height + 7) & ~7) // MI_SIZE   # aligned to 8 px like mi_params
    mi_cols = ((width + 7) & ~7) // MI_SIZE
    nbx, nby = width // bw, height // bh
    n = nbx * nby
    one = np.zeros(n, JOB_DTYPE)
    ys = np.repeat(np.arange(nby) * bh, nbx)
    xs = np.tile(np.arange(nbx) * bw, nby)
    one["src_off"] = (ys + border) * stride + xs + border
    mb = border if mv_border is None else mv_border
    lim = np.array([mv_limits(mi_rows, mi_cols, y // MI_SIZE, x // MI_SIZE, bh // MI_SIZE,
                              bw // MI_SIZE, mb, ref_mv) for y, x in zip(ys, xs)])
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
                         use_downsampled_sad=False, out=None, stream=None, method="diamond"):
    """src: uint8 device tensor (padded plane, 2-D), ref: uint8 device tensor
    holding the reference planes (any shape, contiguous, same stride); jobs:
    device byte tensor of JOB_DTYPE records.  Returns a device byte tensor of
    RESULT_DTYPE records (view with results_numpy).  method "bigdia":
    lavish_fast_bigdia_search_batch (search_method FAST_BIGDIA)."""
    import torch
    assert src.dtype == torch.uint8 and ref.dtype == torch.uint8
    assert src.is_contiguous() and ref.is_contiguous(), "planes must be C-contiguous"
    nj = jobs.numel() // JOB_DTYPE.itemsize
    if out is None:
        out = torch.empty(nj * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=src.device)
    fn = (_lib.lavish_fast_bigdia_search_batch if method == "bigdia"
          else _lib.lavish_diamond_search_batch)
    rc = fn(_vp(src.data_ptr()), src.stride(0), _vp(ref.data_ptr()), src.stride(0), w, h,
            _vp(jobs.data_ptr()), nj, step_param, mv_cost_type, int(use_downsampled_sad),
            _vp(out.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_diamond_search_batch rejected its arguments (rc=%d)" % rc)
    return out


def full_pixel_search_batch(src, ref, w, h, jobs, cost, method="diamond", step_param=0,
                            use_downsampled_sad=False, cost_list=False, out=None,
                            cost_lists=None, stream=None, tiles=None, mesh=None):
    """lavish_full_pixel_search_batch (av1_full_pixel_search): planes and jobs
    as diamond_search_batch, cost a MvCostParams (MvCosts.cost_params or
    l1_cost_params); mesh a MeshParams: lavish_full_pixel_search_batch_mesh
    (the exhaustive mesh refinement).  Returns (RESULT_DTYPE byte tensor,
    int32 [n, 5] cost lists or None)."""
    import torch
    assert src.dtype == torch.uint8 and ref.dtype == torch.uint8
    assert src.is_contiguous() and ref.is_contiguous(), "planes must be C-contiguous"
    nj = jobs.numel() // JOB_DTYPE.itemsize
    if out is None:
        out = torch.empty(nj * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=src.device)
    if cost_list and cost_lists is None:
        cost_lists = torch.empty((nj, 5), dtype=torch.int32, device=src.device)
    if tiles is not None:
        assert tiles.ref.data_ptr() == ref.data_ptr() and tiles.stride == src.stride(0)
    if mesh is not None:
        rc = _lib.lavish_full_pixel_search_batch_mesh(
            _vp(src.data_ptr()), src.stride(0), _vp(ref.data_ptr()), src.stride(0),
            ctypes.byref(tiles.desc) if tiles is not None else None, w, h, _vp(jobs.data_ptr()),
            nj, SEARCH_METHODS[method], step_param, ctypes.byref(cost),
            int(use_downsampled_sad), ctypes.byref(mesh), _vp(out.data_ptr()),
            _vp(cost_lists.data_ptr()) if cost_list else None, _stream_ptr(stream))
    elif tiles is not None:  # RefTiles of `ref`: candidate rows from the tiled copy
        rc = _lib.lavish_full_pixel_search_batch_tiled(
            _vp(src.data_ptr()), src.stride(0), _vp(ref.data_ptr()), src.stride(0),
            ctypes.byref(tiles.desc), w, h, _vp(jobs.data_ptr()), nj, SEARCH_METHODS[method],
            step_param, ctypes.byref(cost), int(use_downsampled_sad), _vp(out.data_ptr()),
            _vp(cost_lists.data_ptr()) if cost_list else None, _stream_ptr(stream))
    else:
        rc = _lib.lavish_full_pixel_search_batch(
            _vp(src.data_ptr()), src.stride(0), _vp(ref.data_ptr()), src.stride(0), w, h,
            _vp(jobs.data_ptr()), nj, SEARCH_METHODS[method], step_param, ctypes.byref(cost),
            int(use_downsampled_sad), _vp(out.data_ptr()),
            _vp(cost_lists.data_ptr()) if cost_list else None, _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_full_pixel_search_batch rejected its arguments (rc=%d)" % rc)
    return out, (cost_lists if cost_list else None)


_lib.lavish_txq_frame_search.argtypes = [
    _vp, _i32, _i32, _i32, ctypes.c_uint32, _vp, _i32, _i32, _vp, _vp, _vp, _vp,
    _vp, _i32, _vp, _i32, ctypes.POINTER(RefTilesDesc), _vp, _i32, _i32,
    ctypes.POINTER(MvCostParams), _i32, _vp, _vp, _i32, _vp]
_lib.lavish_txq_frame_search.restype = _i32


def txq_frame_search(residual, frame_out, qp, src, ref, jobs, cost, tiles, out, cost_lists,
                     every, step_param=0, use_downsampled_sad=True, bit_depth=8,
                     quant_kind=None, stream=None):
    """lavish_txq_frame_search: lavish_txq_frame over `frame_out`'s sizes and
    the 16x16 DIAMOND full_pixel_search_batch (tiled references, cost lists
    into `cost_lists` when given) in one launch, a search unit every `every`
    units of the dispatch order.  The tiles must already be built."""
    import torch
    import lavish_dsp as L
    assert residual.dtype == torch.int16 and residual.stride(1) == 1
    assert src.dtype == torch.uint8 and ref.dtype == torch.uint8 and src.is_contiguous()
    assert tiles.ref.data_ptr() == ref.data_ptr() and tiles.stride == src.stride(0)
    H, W = residual.shape
    nj = jobs.numel() // JOB_DTYPE.itemsize
    qk = L.QUANT_FP if quant_kind is None else quant_kind
    rc = _lib.lavish_txq_frame_search(
        _vp(residual.data_ptr()), residual.stride(0), W, H, frame_out.size_mask, frame_out.tm,
        bit_depth, qk, ctypes.byref(qp), frame_out.q, frame_out.dq, frame_out.eob,
        _vp(src.data_ptr()), src.stride(0), _vp(ref.data_ptr()), src.stride(0),
        ctypes.byref(tiles.desc), _vp(jobs.data_ptr()), nj, step_param, ctypes.byref(cost),
        int(use_downsampled_sad), _vp(out.data_ptr()),
        _vp(cost_lists.data_ptr()) if cost_lists is not None else None, int(every),
        _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_txq_frame_search rejected its arguments (rc=%d)" % rc)
    return frame_out.outs, out


def results_numpy(out):
    return out.cpu().numpy().view(RESULT_DTYPE)


# ------------------------------------------------------- sub-pixel search --
SUBPEL_JOB_DTYPE = np.dtype([("src_off", "<i8"), ("ref_off", "<i8"), ("start_row", "<i2"),
                             ("start_col", "<i2"), ("ref_mv_row", "<i2"), ("ref_mv_col", "<i2"),
                             ("col_min", "<i2"), ("col_max", "<i2"), ("row_min", "<i2"),
                             ("row_max", "<i2")], align=True)
SUBPEL_RESULT_DTYPE = np.dtype([("best_row", "<i2"), ("best_col", "<i2"), ("besterr", "<u4"),
                                ("distortion", "<i4"), ("sse", "<u4")], align=True)
assert SUBPEL_JOB_DTYPE.itemsize == 32 and SUBPEL_RESULT_DTYPE.itemsize == 16
EIGHTH_PEL, QUARTER_PEL, HALF_PEL, FULL_PEL = 0, 1, 2, 3

_lib.lavish_subpel_search_batch.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _i32, _i32,
                                            _i32, _i32, _i32, _vp, _vp]
_lib.lavish_subpel_search_batch.restype = _i32
_lib.lavish_subpel_search_after_diamond.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _vp,
                                                    _i32, _i32, _i32, _i32, _i32, _vp, _vp]
_lib.lavish_subpel_search_after_diamond.restype = _i32


def subpel_jobs(width, height, border, bw, bh, fullpel_jobs, fullpel_results, ref_mv=(0, 0)):
    """Sub-pixel jobs continuing the full-pel jobs of frame_jobs (same order):
    start = the full-pel best x 8, SubpelMvLimits from the block's
    x->mv_limits and ref_mv."""
    mi_rows = ((height + 7) & ~7) // MI_SIZE
    mi_cols = ((width + 7) & ~7) // MI_SIZE
    nbx, nby = width // bw, height // bh
    ys = np.repeat(np.arange(nby) * bh, nbx)
    xs = np.tile(np.arange(nbx) * bw, nby)
    lim = np.array([subpel_limits(block_mv_limits(mi_rows, mi_cols, y // MI_SIZE, x // MI_SIZE,
                                                  bh // MI_SIZE, bw // MI_SIZE, border), ref_mv)
                    for y, x in zip(ys, xs)])
    nrefs = len(fullpel_jobs) // len(lim)
    lim = np.concatenate([lim] * nrefs)
    out = np.zeros(len(fullpel_jobs), SUBPEL_JOB_DTYPE)
    out["src_off"] = fullpel_jobs["src_off"]
    out["ref_off"] = fullpel_jobs["ref_off"]
    out["start_row"] = fullpel_results["best_row"].astype(np.int32) * 8
    out["start_col"] = fullpel_results["best_col"].astype(np.int32) * 8
    out["ref_mv_row"], out["ref_mv_col"] = ref_mv
    out["col_min"], out["col_max"], out["row_min"], out["row_max"] = lim.T
    return out


def subpel_search_batch(src, ref, w, h, jobs, forced_stop=EIGHTH_PEL, allow_hp=False,
                        iters_per_step=1, mv_cost_type=MV_COST_L1_HDRES, out=None, stream=None):
    """lavish_subpel_search_batch over device planes (as diamond_search_batch)
    and a device byte tensor of SUBPEL_JOB_DTYPE records; returns a device
    byte tensor of SUBPEL_RESULT_DTYPE records."""
    import torch
    assert src.dtype == torch.uint8 and ref.dtype == torch.uint8
    assert src.is_contiguous() and ref.is_contiguous(), "planes must be C-contiguous"
    nj = jobs.numel() // SUBPEL_JOB_DTYPE.itemsize
    if out is None:
        out = torch.empty(nj * SUBPEL_RESULT_DTYPE.itemsize, dtype=torch.uint8,
                          device=src.device)
    rc = _lib.lavish_subpel_search_batch(_vp(src.data_ptr()), src.stride(0),
                                         _vp(ref.data_ptr()), src.stride(0), w, h,
                                         _vp(jobs.data_ptr()), nj, forced_stop, int(allow_hp),
                                         iters_per_step, mv_cost_type, _vp(out.data_ptr()),
                                         _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_subpel_search_batch rejected its arguments (rc=%d)" % rc)
    return out


def subpel_after_diamond(src, ref, w, h, jobs, fullpel, forced_stop=EIGHTH_PEL, allow_hp=False,
                         iters_per_step=1, mv_cost_type=MV_COST_L1_HDRES, out=None,
                         stream=None):
    """lavish_subpel_search_after_diamond: as subpel_search_batch with every
    job starting at the device-resident full-pel result `fullpel` (the
    RESULT_DTYPE bytes diamond_search_batch returned)."""
    import torch
    nj = jobs.numel() // SUBPEL_JOB_DTYPE.itemsize
    assert fullpel.numel() >= nj * RESULT_DTYPE.itemsize
    if out is None:
        out = torch.empty(nj * SUBPEL_RESULT_DTYPE.itemsize, dtype=torch.uint8,
                          device=src.device)
    rc = _lib.lavish_subpel_search_after_diamond(
        _vp(src.data_ptr()), src.stride(0), _vp(ref.data_ptr()), src.stride(0), w, h,
        _vp(jobs.data_ptr()), _vp(fullpel.data_ptr()), nj, forced_stop, int(allow_hp),
        iters_per_step, mv_cost_type, _vp(out.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_subpel_search_after_diamond rejected its arguments (rc=%d)" % rc)
    return out


SUBPEL_METHODS = {"tree": 0, "pruned": 1, "pruned_more": 2}   # SUBPEL_SEARCH_METHODS
_lib.lavish_find_best_sub_pixel_tree_batch.argtypes = [
    _vp, _i32, _vp, _i32, _i32, _i32, _vp, _vp, _i32, _i32, _i32, _i32, _i32,
    ctypes.POINTER(MvCostParams), _vp, _vp, _vp]
_lib.lavish_find_best_sub_pixel_tree_batch.restype = _i32
_lib.lavish_find_best_sub_pixel_tree_batch_ex.argtypes = [
    _vp, _i32, _vp, _i32, _i32, _i32, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32,
    ctypes.POINTER(MvCostParams), _vp, _vp, _vp]
_lib.lavish_find_best_sub_pixel_tree_batch_ex.restype = _i32
# SUBPEL_SEARCH_TYPE (av1/common/filter.h:45-50)
USE_2_TAPS_ORIG, USE_2_TAPS, USE_4_TAPS, USE_8_TAPS = range(4)


def find_best_sub_pixel_tree_batch(src, ref, w, h, jobs, cost, method="pruned_more",
                                   forced_stop=EIGHTH_PEL, allow_hp=False, iters_per_step=1,
                                   fullpel=None, cost_lists=None, out=None, stream=None,
                                   search_type=USE_2_TAPS_ORIG):
    """lavish_find_best_sub_pixel_tree_batch_ex: av1_find_best_sub_pixel_tree
    ("tree"; the bilinear error with search_type USE_2_TAPS_ORIG / USE_2_TAPS,
    the upsampled prediction's with USE_4_TAPS / USE_8_TAPS), _pruned or
    _pruned_more with any mv cost (MvCostParams) and the full-pel cost lists
    (device int32 [n, 5] or None); fullpel: device RESULT_DTYPE bytes to start
    from (or None: the jobs' start fields)."""
    import torch
    assert src.dtype == torch.uint8 and ref.dtype == torch.uint8
    assert src.is_contiguous() and ref.is_contiguous(), "planes must be C-contiguous"
    nj = jobs.numel() // SUBPEL_JOB_DTYPE.itemsize
    if fullpel is not None:
        assert fullpel.numel() >= nj * RESULT_DTYPE.itemsize
    if cost_lists is not None:
        assert cost_lists.dtype == torch.int32 and cost_lists.numel() >= 5 * nj
    if out is None:
        out = torch.empty(nj * SUBPEL_RESULT_DTYPE.itemsize, dtype=torch.uint8,
                          device=src.device)
    rc = _lib.lavish_find_best_sub_pixel_tree_batch_ex(
        _vp(src.data_ptr()), src.stride(0), _vp(ref.data_ptr()), src.stride(0), w, h,
        _vp(jobs.data_ptr()), None if fullpel is None else _vp(fullpel.data_ptr()), nj,
        SUBPEL_METHODS[method], search_type, forced_stop, int(allow_hp), iters_per_step,
        ctypes.byref(cost),
        None if cost_lists is None else _vp(cost_lists.data_ptr()), _vp(out.data_ptr()),
        _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_find_best_sub_pixel_tree_batch rejected its arguments (rc=%d)"
                         % rc)
    return out


def subpel_results_numpy(out):
    return out.cpu().numpy().view(SUBPEL_RESULT_DTYPE)
