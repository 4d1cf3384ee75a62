"""The affine warp predictor on the MI355X backend:
lavish_warp_affine_batch replaces av1_warp_affine_c / av1_highbd_warp_affine_c
(av1/common/warped_motion.c:264-388,538-666) for a batch of prediction
blocks of one (stack of) reference plane(s); lavish_get_shear_params is
av1_get_shear_params (:218-247); av1_warp_affine_hip /
av1_highbd_warp_affine_hip are the per-call RTCD shims."""
import ctypes

import numpy as np

from . import _lib, _stream_ptr
from .inter import ConvolveParams

_vp, _i32 = ctypes.c_void_p, ctypes.c_int32
_CP = ctypes.POINTER(ConvolveParams)

JOB_DTYPE = np.dtype([("mat", "<i4", (6,)), ("alpha", "<i2"), ("beta", "<i2"), ("gamma", "<i2"),
                      ("delta", "<i2"), ("p_col", "<i4"), ("p_row", "<i4"), ("p_width", "<i4"),
                      ("p_height", "<i4"), ("ref_off", "<i8"), ("pred_off", "<i8"),
                      ("dst_off", "<i8")])
assert JOB_DTYPE.itemsize == 72

_lib.lavish_warp_affine_batch.argtypes = [_vp, _i32, _i32, _i32, _vp, _i32, _vp, _i32, _vp, _i32,
                                          _i32, _i32, _i32, _i32, _CP, _vp]
_lib.lavish_warp_affine_batch.restype = _i32
_lib.lavish_get_shear_params.argtypes = [_vp, _vp]
_lib.lavish_get_shear_params.restype = _i32
_lib.av1_warp_affine_hip.argtypes = [_vp, _vp] + [_i32] * 3 + [_vp] + [_i32] * 7 + [_CP] + \
    [ctypes.c_int16] * 4
_lib.av1_warp_affine_hip.restype = None
_lib.av1_highbd_warp_affine_hip.argtypes = [_vp, _vp] + [_i32] * 3 + [_vp] + [_i32] * 8 + \
    [_CP] + [ctypes.c_int16] * 4
_lib.av1_highbd_warp_affine_hip.restype = None


def conv_params(round_0, round_1, is_compound=0, do_average=0, dist_wtd=0, fwd_offset=0,
                bck_offset=0, dst=None, dst_stride=0):
    """A ConvolveParams with the fields the warp reads (dst only for the shims)."""
    d = dst.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)) if dst is not None else None
    return ConvolveParams(do_average, d, dst_stride, round_0, round_1, 0, is_compound, dist_wtd,
                          fwd_offset, bck_offset)


def get_shear_params(mat):
    """-> (valid, (alpha, beta, gamma, delta)) for wmmat[0..5]."""
    m = np.ascontiguousarray(np.asarray(mat, np.int32)[:6])
    out = np.zeros(4, np.int16)
    ok = _lib.lavish_get_shear_params(m.ctypes.data_as(_vp), out.ctypes.data_as(_vp))
    return ok, tuple(int(v) for v in out)


def warp_affine_batch(ref, width, height, stride, pred, p_stride, jobs, njobs, cp, bit_depth=8,
                      conv_dst=None, dst_stride=0, subsampling_x=0, subsampling_y=0,
                      stream=None):
    """lavish_warp_affine_batch on device tensors: ref / pred u8 (or int16 /
    uint16 views of u16 samples), jobs a device byte tensor of JOB_DTYPE
    records, conv_dst an int16 / uint16 tensor (compound), cp a
    ConvolveParams (its dst is ignored)."""
    highbd = ref.element_size() == 2
    rc = _lib.lavish_warp_affine_batch(
        _vp(ref.data_ptr()), width, height, stride, _vp(pred.data_ptr()), p_stride,
        _vp(conv_dst.data_ptr()) if conv_dst is not None else None, dst_stride,
        _vp(jobs.data_ptr()), njobs, subsampling_x, subsampling_y, bit_depth, int(highbd),
        ctypes.byref(cp), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_warp_affine_batch rejected its arguments (rc=%d)" % rc)


def warp_affine_shim(mat, ref, width, height, stride, pred, p_col, p_row, p_width, p_height,
                     p_stride, ss_x, ss_y, cp, params, bd=8):
    """av1_warp_affine_hip / av1_highbd_warp_affine_hip on host numpy arrays
    (in place on pred and on cp's dst)."""
    m = np.ascontiguousarray(np.asarray(mat, np.int32)[:6])
    if ref.dtype == np.uint8:
        _lib.av1_warp_affine_hip(m.ctypes.data_as(_vp), ref.ctypes.data_as(_vp), width, height,
                                 stride, pred.ctypes.data_as(_vp), p_col, p_row, p_width,
                                 p_height, p_stride, ss_x, ss_y, ctypes.byref(cp), *params)
    else:
        _lib.av1_highbd_warp_affine_hip(m.ctypes.data_as(_vp), ref.ctypes.data_as(_vp), width,
                                        height, stride, pred.ctypes.data_as(_vp), p_col, p_row,
                                        p_width, p_height, p_stride, ss_x, ss_y, bd,
                                        ctypes.byref(cp), *params)
