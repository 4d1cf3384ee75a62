"""Scaled convolution on the MI355X backend:
lavish_convolve_2d_scale_batch replaces av1_convolve_2d_scale_c and
av1_highbd_convolve_2d_scale_c (av1/common/convolve.c:488-574, 992-1078) --
the inter predictor of a reference of another resolution -- for a batch of
blocks; av1_convolve_2d_scale_hip / av1_highbd_convolve_2d_scale_hip are the
per-call RTCD shims (av1_rtcd_defs.pl:580,583)."""
import ctypes

import numpy as np

from . import _lib, _stream_ptr
from .inter import ConvolveParams, InterpFilterParams

_vp, _i32 = ctypes.c_void_p, ctypes.c_int32
_FP = ctypes.POINTER(InterpFilterParams)
_CP = ctypes.POINTER(ConvolveParams)

JOB_DTYPE = np.dtype([("src_off", "<i8"), ("dst_off", "<i8"), ("conv_off", "<i8"),
                      ("subpel_x_qn", "<i4"), ("x_step_qn", "<i4"), ("subpel_y_qn", "<i4"),
                      ("y_step_qn", "<i4")])
assert JOB_DTYPE.itemsize == 40

_lib.lavish_convolve_2d_scale_batch.argtypes = [_vp, _i32, _vp, _i32, _vp, _i32, _i32, _i32, _vp,
                                                _i32, _FP, _FP, _CP, _i32, _i32, _vp]
_lib.lavish_convolve_2d_scale_batch.restype = _i32
_lib.av1_convolve_2d_scale_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _FP, _i32, _i32,
                                           _i32, _i32, _CP]
_lib.av1_convolve_2d_scale_hip.restype = None
_lib.av1_highbd_convolve_2d_scale_hip.argtypes = [_vp, _i32, _vp, _i32, _i32, _i32, _FP, _FP,
                                                  _i32, _i32, _i32, _i32, _CP, _i32]
_lib.av1_highbd_convolve_2d_scale_hip.restype = None


def convolve_2d_scale_batch(src, src_stride, dst, dst_stride, conv, conv_stride, w, h, jobs,
                            njobs, fpx, fpy, cp, bit_depth=8, stream=None):
    """lavish_convolve_2d_scale_batch on device tensors (u8, or int16 views
    of u16 samples; conv an int16 view of the CONV_BUF, None when cp is not
    compound; dst None for a compound first pass)."""
    highbd = src.element_size() == 2
    rc = _lib.lavish_convolve_2d_scale_batch(
        _vp(src.data_ptr()), src_stride, _vp(dst.data_ptr()) if dst is not None else None,
        dst_stride, _vp(conv.data_ptr()) if conv is not None else None, conv_stride, w, h,
        _vp(jobs.data_ptr()), njobs, ctypes.byref(fpx), ctypes.byref(fpy), ctypes.byref(cp),
        bit_depth, int(highbd), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_convolve_2d_scale_batch rejected its arguments (rc=%d)" % rc)


def convolve_2d_scale_shim(src, src_stride, dst, dst_stride, w, h, fpx, fpy, subpel_x_qn,
                           x_step_qn, subpel_y_qn, y_step_qn, cp, bd=8):
    """av1_convolve_2d_scale_hip / av1_highbd_convolve_2d_scale_hip on host
    arrays (src: the flat array positioned at the block via ctypes address)."""
    d = dst.ctypes.data_as(_vp)
    a = (src, src_stride, d, dst_stride, w, h, ctypes.byref(fpx), ctypes.byref(fpy), subpel_x_qn,
         x_step_qn, subpel_y_qn, y_step_qn, ctypes.byref(cp))
    if dst.dtype == np.uint16:
        _lib.av1_highbd_convolve_2d_scale_hip(*a, bd)
    else:
        _lib.av1_convolve_2d_scale_hip(*a)
