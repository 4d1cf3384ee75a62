"""Compound (CONV_BUF) convolutions on the MI355X backend (SURVEY.md 8(f)
rank 2): lavish_dist_wtd_convolve_batch replaces the
av1_dist_wtd_convolve_{2d_copy,x,y,2d}_c family and its highbd forms
(av1/common/convolve.c:291-489,790-988) for a batch of blocks; the eight
av1_*dist_wtd_convolve*_hip functions are the per-call RTCD shims."""
import ctypes

import numpy as np

from . import _lib, _stream_ptr
from .inter import ConvolveParams, InterpFilterParams

_vp, _i32 = ctypes.c_void_p, ctypes.c_int32
_FP = ctypes.POINTER(InterpFilterParams)
_CP = ctypes.POINTER(ConvolveParams)

JOB_DTYPE = np.dtype([("src_off", "<i8"), ("dst_off", "<i8"), ("conv_off", "<i8"),
                      ("subpel_x_qn", "<i4"), ("subpel_y_qn", "<i4")])
assert JOB_DTYPE.itemsize == 32

_lib.lavish_dist_wtd_convolve_batch.argtypes = [_vp, _i32, _vp, _i32, _vp, _i32, _i32, _i32, _vp,
                                                _i32, _FP, _FP, _CP, _i32, _i32, _vp]
_lib.lavish_dist_wtd_convolve_batch.restype = _i32
_lib.av1_dist_wtd_convolve_2d_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _FP, _i32,
                                              _i32, _CP]
_lib.av1_dist_wtd_convolve_x_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _i32, _CP]
_lib.av1_dist_wtd_convolve_y_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _i32, _CP]
_lib.av1_dist_wtd_convolve_2d_copy_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _CP]
_lib.av1_highbd_dist_wtd_convolve_2d_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _FP,
                                                     _i32, _i32, _CP, _i32]
_lib.av1_highbd_dist_wtd_convolve_x_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _i32,
                                                    _CP, _i32]
_lib.av1_highbd_dist_wtd_convolve_y_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _i32,
                                                    _CP, _i32]
_lib.av1_highbd_dist_wtd_convolve_2d_copy_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _CP,
                                                          _i32]


def filter_params(table):
    """InterpFilterParams over a host int16 [16, taps] kernel table (kept
    alive by the caller)."""
    t = np.ascontiguousarray(table, np.int16)
    return InterpFilterParams(t.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), t.shape[1], 0), t


def dist_wtd_convolve_batch(src, src_stride, dst, dst_stride, conv, conv_stride, w, h, jobs,
                            njobs, fpx, fpy, cp, bit_depth=8, stream=None):
    """lavish_dist_wtd_convolve_batch on device tensors (u8, or int16 views
    of u16 samples; conv an int16 view of the CONV_BUF)."""
    highbd = src.element_size() == 2
    rc = _lib.lavish_dist_wtd_convolve_batch(
        _vp(src.data_ptr()), src_stride, _vp(dst.data_ptr()) if dst is not None else None,
        dst_stride, _vp(conv.data_ptr()), conv_stride, w, h, _vp(jobs.data_ptr()), njobs,
        ctypes.byref(fpx), ctypes.byref(fpy), ctypes.byref(cp), bit_depth, int(highbd),
        _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_dist_wtd_convolve_batch rejected its arguments (rc=%d)" % rc)


def dist_wtd_convolve_shim(path, src, src_stride, dst, dst_stride, w, h, fpx, fpy, sx, sy, cp,
                           bd=8):
    """One of the eight av1_*dist_wtd_convolve*_hip shims on host arrays
    (src: the flat array positioned at the block via ctypes address)."""
    hb = dst.dtype == np.uint16
    p = "av1_highbd_" if hb else "av1_"
    d = dst.ctypes.data_as(_vp)
    extra = (bd,) if hb else ()
    if path == 0:
        getattr(_lib, p + "dist_wtd_convolve_2d_copy_hip")(src, src_stride, d, dst_stride, w, h,
                                                          ctypes.byref(cp), *extra)
    elif path == 1:
        getattr(_lib, p + "dist_wtd_convolve_x_hip")(src, src_stride, d, dst_stride, w, h,
                                                    ctypes.byref(fpx), sx, ctypes.byref(cp),
                                                    *extra)
    elif path == 2:
        getattr(_lib, p + "dist_wtd_convolve_y_hip")(src, src_stride, d, dst_stride, w, h,
                                                    ctypes.byref(fpy), sy, ctypes.byref(cp),
                                                    *extra)
    else:
        getattr(_lib, p + "dist_wtd_convolve_2d_hip")(src, src_stride, d, dst_stride, w, h,
                                                     ctypes.byref(fpx), ctypes.byref(fpy), sx,
                                                     sy, ctypes.byref(cp), *extra)
