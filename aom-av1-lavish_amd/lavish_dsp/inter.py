"""Single-reference inter prediction on the MI355X backend
(lavish_build_inter_pred_batch / _after_subpel) and the per-call convolve
shims (av1_convolve_{x,y,2d}_sr_hip, their highbd forms, aom_convolve_copy_hip).

The batch form is av1_enc_build_one_inter_predictor
(av1/encoder/reconinter_enc.c:47-51) for many blocks at once: the caller's
per-block work (mv, filter pair, block position) becomes one
INTER_JOB_DTYPE record, exactly the arguments build_inter_predictors
(av1/common/reconinter_template.inc) hands to it for TRANSLATION_PRED,
UNIFORM_SINGLE, unscaled references."""
import ctypes

import numpy as np

from . import _lib, _stream_ptr

INTER_JOB_DTYPE = np.dtype([("ref_off", "<i8"), ("dst_off", "<i8"), ("pix_row", "<i4"),
                            ("pix_col", "<i4"), ("mv_row", "<i2"), ("mv_col", "<i2"),
                            ("filter_x", "u1"), ("filter_y", "u1"), ("pad", "u1", (2,))],
                           align=True)
assert INTER_JOB_DTYPE.itemsize == 32

# InterpFilter (av1/common/filter.h:30-43)
EIGHTTAP_REGULAR, EIGHTTAP_SMOOTH, MULTITAP_SHARP, BILINEAR, MULTITAP_SHARP2 = range(5)
AOM_BORDER_IN_PIXELS = 288

_vp, _i32, _pd = ctypes.c_void_p, ctypes.c_int32, ctypes.c_ssize_t
_lib.lavish_build_inter_pred_batch.argtypes = [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                               _vp, _i32, _vp, _i32, _i32, _i32, _vp]
_lib.lavish_build_inter_pred_batch.restype = _i32
_lib.lavish_build_inter_pred_after_subpel.argtypes = [_vp, _i32, _i32, _i32, _i32, _i32, _i32,
                                                      _i32, _vp, _vp, _i32, _vp, _i32, _i32,
                                                      _i32, _vp]
_lib.lavish_build_inter_pred_after_subpel.restype = _i32


class InterpFilterParams(ctypes.Structure):
    """Layout of InterpFilterParams (av1/common/filter.h:105-109)."""
    _fields_ = [("filter_ptr", ctypes.POINTER(ctypes.c_int16)), ("taps", ctypes.c_uint16),
                ("interp_filter", ctypes.c_uint8)]


class ConvolveParams(ctypes.Structure):
    """Layout of ConvolveParams (av1/common/convolve.h:21-32)."""
    _fields_ = [("do_average", ctypes.c_int), ("dst", ctypes.POINTER(ctypes.c_uint16)),
                ("dst_stride", ctypes.c_int), ("round_0", ctypes.c_int),
                ("round_1", ctypes.c_int), ("plane", ctypes.c_int),
                ("is_compound", ctypes.c_int), ("use_dist_wtd_comp_avg", ctypes.c_int),
                ("fwd_offset", ctypes.c_int), ("bck_offset", ctypes.c_int)]


_FP = ctypes.POINTER(InterpFilterParams)
_CP = ctypes.POINTER(ConvolveParams)
_lib.av1_convolve_2d_sr_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _FP, _i32, _i32,
                                        _CP]
_lib.av1_convolve_x_sr_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _i32, _CP]
_lib.av1_convolve_y_sr_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _i32]
_lib.av1_highbd_convolve_2d_sr_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _FP, _i32,
                                               _i32, _CP, _i32]
_lib.av1_highbd_convolve_x_sr_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _i32, _CP,
                                              _i32]
_lib.av1_highbd_convolve_y_sr_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _i32, _i32]
_lib.aom_convolve_copy_hip.argtypes = [_vp, _pd, _vp, _pd, _i32, _i32]
_lib.aom_highbd_convolve_copy_hip.argtypes = [_vp, _pd, _vp, _pd, _i32, _i32]
for _n in ("av1_convolve_2d_sr_hip", "av1_convolve_x_sr_hip", "av1_convolve_y_sr_hip",
           "av1_highbd_convolve_2d_sr_hip", "av1_highbd_convolve_x_sr_hip",
           "av1_highbd_convolve_y_sr_hip", "aom_convolve_copy_hip",
           "aom_highbd_convolve_copy_hip"):
    getattr(_lib, _n).restype = None
_lib.lavish_interp_kernels.argtypes = [_i32, _i32, _vp]
_lib.lavish_interp_kernels.restype = _i32


def interp_kernels(interp_filter, size):
    """The library's kernel table for av1_get_interp_filter_params_with_block_size
    (av1/common/filter.h:253-259): int16 [16, taps] (lavish_interp_kernels)."""
    out = np.zeros(16 * 12, np.int16)
    taps = _lib.lavish_interp_kernels(interp_filter, size, out.ctypes.data)
    if taps < 0:
        raise ValueError("lavish_interp_kernels(%d, %d) rejected" % (interp_filter, size))
    return out[:16 * taps].reshape(16, taps)


def conv_rounds(bd):
    """get_conv_params_no_round(0, plane, NULL, 0, 0, bd) -> (round_0, round_1)
    (av1/common/convolve.h:63-84)."""
    r0, r1 = 3, 14 - 3
    ibr = bd + 7 - r0 + 2
    if ibr > 16:
        r0 += ibr - 16
        r1 -= ibr - 16
    return r0, r1


def plane_jobs(width, height, bw, bh, mvs, filters=(EIGHTTAP_REGULAR, EIGHTTAP_REGULAR),
               ref_off=0, dst_stride=None):
    """One job per full bw x bh block of a width x height plane (raster order):
    mvs is an (nblocks, 2) array of (row, col) 1/8-pel MVs or a single pair;
    filters a (filter_x, filter_y) pair or an (nblocks, 2) array.  The
    prediction of block (by, bx) lands at its own position in a dst plane of
    stride dst_stride (default width)."""
    nbx, nby = width // bw, height // bh
    n = nbx * nby
    ds = width if dst_stride is None else dst_stride
    jobs = np.zeros(n, INTER_JOB_DTYPE)
    by, bx = np.divmod(np.arange(n), nbx)
    jobs["pix_row"], jobs["pix_col"] = by * bh, bx * bw
    jobs["ref_off"] = ref_off
    jobs["dst_off"] = by * bh * ds + bx * bw
    mv = np.broadcast_to(np.asarray(mvs, np.int16).reshape(-1, 2), (n, 2))
    jobs["mv_row"], jobs["mv_col"] = mv[:, 0], mv[:, 1]
    f = np.broadcast_to(np.asarray(filters, np.uint8).reshape(-1, 2), (n, 2))
    jobs["filter_x"], jobs["filter_y"] = f[:, 0], f[:, 1]
    return jobs


def build_inter_pred_batch(ref, ref_origin, ref_width, ref_height, w, h, jobs, dst=None,
                           dst_stride=None, bit_depth=8, ss=(0, 0), mvs=None, stream=None):
    """lavish_build_inter_pred_batch over a device reference plane (uint8, or
    uint16 / int16 holding u16 pixels; 2-D, bordered) whose frame origin (buf0) is element offset
    ref_origin; jobs: device byte tensor of INTER_JOB_DTYPE records (their
    ref_off is added to ref_origin).  mvs: optional device byte tensor of
    SUBPEL_RESULT records (lavish_build_inter_pred_after_subpel).  Returns the
    dst tensor (allocated as ref_height x ref_width when None)."""
    import torch
    assert ref.dtype in (torch.uint8, torch.uint16, torch.int16) and ref.is_contiguous()
    highbd = int(ref.element_size() == 2)  # int16 tensors carry u16 planes bit for bit
    es = ref.element_size()
    if dst is None:
        dst = torch.zeros((ref_height, ref_width), dtype=ref.dtype, device=ref.device)
    ds = dst.stride(0) if dst_stride is None else dst_stride
    nj = jobs.numel() // INTER_JOB_DTYPE.itemsize
    base = _vp(ref.data_ptr() + ref_origin * es)
    if mvs is None:
        rc = _lib.lavish_build_inter_pred_batch(base, ref.stride(0), ref_width, ref_height,
                                                ss[0], ss[1], w, h, _vp(jobs.data_ptr()), nj,
                                                _vp(dst.data_ptr()), ds, bit_depth, highbd,
                                                _stream_ptr(stream))
    else:
        rc = _lib.lavish_build_inter_pred_after_subpel(base, ref.stride(0), ref_width,
                                                       ref_height, ss[0], ss[1], w, h,
                                                       _vp(jobs.data_ptr()),
                                                       _vp(mvs.data_ptr()), nj,
                                                       _vp(dst.data_ptr()), ds, bit_depth,
                                                       highbd, _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_build_inter_pred_batch rejected its arguments (rc=%d)" % rc)
    return dst


def filter_params(table, taps, interp_filter=0):
    """An InterpFilterParams over a (16, taps) int16 numpy kernel table (kept
    alive on the returned object)."""
    t = np.ascontiguousarray(table, np.int16)
    fp = InterpFilterParams(t.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), taps,
                            interp_filter)
    fp._keep = t
    return fp


def convolve(kind, src, src_off, src_stride, dst, dst_off, dst_stride, w, h, fpx=None,
             fpy=None, subpel_x=0, subpel_y=0, round_0=3, round_1=11, bd=8):
    """Per-call RTCD shim on host numpy planes: kind in "2d", "x", "y",
    "copy"; uint16 planes select the highbd function."""
    hb = src.dtype == np.uint16
    es = src.itemsize
    s = _vp(src.ctypes.data + src_off * es)
    d = _vp(dst.ctypes.data + dst_off * es)
    cp = ConvolveParams(0, None, 0, round_0, round_1, 0, 0, 0, 0, 0)
    px = ctypes.byref(fpx) if fpx is not None else None
    py = ctypes.byref(fpy) if fpy is not None else None
    if kind == "2d":
        if hb:
            _lib.av1_highbd_convolve_2d_sr_hip(s, src_stride, d, dst_stride, w, h, px, py,
                                               subpel_x, subpel_y, ctypes.byref(cp), bd)
        else:
            _lib.av1_convolve_2d_sr_hip(s, src_stride, d, dst_stride, w, h, px, py, subpel_x,
                                        subpel_y, ctypes.byref(cp))
    elif kind == "x":
        if hb:
            _lib.av1_highbd_convolve_x_sr_hip(s, src_stride, d, dst_stride, w, h, px, subpel_x,
                                              ctypes.byref(cp), bd)
        else:
            _lib.av1_convolve_x_sr_hip(s, src_stride, d, dst_stride, w, h, px, subpel_x,
                                       ctypes.byref(cp))
    elif kind == "y":
        if hb:
            _lib.av1_highbd_convolve_y_sr_hip(s, src_stride, d, dst_stride, w, h, py, subpel_y,
                                              bd)
        else:
            _lib.av1_convolve_y_sr_hip(s, src_stride, d, dst_stride, w, h, py, subpel_y)
    elif kind == "copy":
        if hb:
            _lib.aom_highbd_convolve_copy_hip(s, src_stride, d, dst_stride, w, h)
        else:
            _lib.aom_convolve_copy_hip(s, src_stride, d, dst_stride, w, h)
    else:
        raise ValueError(kind)
