"""Pixel-domain entry points of liblavish_hip.so: SAD, variance, MSE, SSE,
subtract, sum of squares, Hadamard, SATD, block error.

* Per-call mirror: ``sad(w, h, ...)``-style helpers plus every rtcd-named
  shim reachable as ``rtcd(name)`` (e.g. ``rtcd("aom_sad16x16")``) taking
  numpy arrays / views with the reference's argument meaning.  Highbd
  pointers are tagged exactly like CONVERT_TO_BYTEPTR (aom_ports/mem.h:79)
  before the call, so the shims see what the reference's callers pass.
* Batch layer: ``sad_batch``, ``variance_batch`` ... on torch device tensors
  with a LavishPixJob table (include/lavish_dsp.h).
"""
import ctypes

import numpy as np

from . import _lib, _stream_ptr

# @encoder_block_sizes (aom_dsp/aom_dsp_rtcd_defs.pl:42-58)
ENCODER_BLOCK_SIZES = [(128, 128), (128, 64), (64, 128), (64, 64), (64, 32), (32, 64),
                       (32, 32), (32, 16), (16, 32), (16, 16), (16, 8), (8, 16), (8, 8),
                       (8, 4), (4, 8), (4, 4), (4, 16), (16, 4), (8, 32), (32, 8),
                       (16, 64), (64, 16)]

JOB_DTYPE = np.dtype([("src_off", "<i8"), ("ref_off", "<i8", (4,)), ("aux_off", "<i8"),
                      ("xoff", "<i4"), ("yoff", "<i4")], align=True)
assert JOB_DTYPE.itemsize == 56

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_u32 = ctypes.c_uint32
_ssz = ctypes.c_ssize_t


def _addr(a):
    return a.__array_interface__["data"][0]


def _ptr(a, highbd=False):
    """Pointer to the first element of a numpy array/view; tagged for highbd."""
    if a is None:
        return None
    p = _addr(a)
    return _vp(p >> 1) if highbd else _vp(p)


# ------------------------------------------------------------ prototypes --
_PROTOS = {}


def _proto(name, restype, argtypes):
    f = getattr(_lib, name + "_hip")
    f.restype = restype
    f.argtypes = argtypes
    _PROTOS[name] = f


_SAD = [_vp, _i32, _vp, _i32]
_SAD_AVG = _SAD + [_vp]
_X4D = [_vp, _i32, _vp, _i32, _vp]
_X4D_AVG = [_vp, _i32, _vp, _i32, _vp, _vp]
_VAR = [_vp, _i32, _vp, _i32, _vp]
_SUBVAR = [_vp, _i32, _i32, _i32, _vp, _i32, _vp]
for _w, _h in ENCODER_BLOCK_SIZES:
    _s = "%dx%d" % (_w, _h)
    _proto("aom_sad" + _s, ctypes.c_uint, _SAD)
    _proto("aom_sad_skip_" + _s, ctypes.c_uint, _SAD)
    _proto("aom_sad%s_avg" % _s, ctypes.c_uint, _SAD_AVG)
    _proto("aom_sad%sx4d" % _s, None, _X4D)
    _proto("aom_sad%sx3d" % _s, None, _X4D)
    _proto("aom_sad%sx4d_avg" % _s, None, _X4D_AVG)
    _proto("aom_sad_skip_%sx4d" % _s, None, _X4D)
    _proto("aom_highbd_sad" + _s, ctypes.c_uint, _SAD)
    _proto("aom_highbd_sad_skip_" + _s, ctypes.c_uint, _SAD)
    _proto("aom_highbd_sad%s_avg" % _s, ctypes.c_uint, _SAD_AVG)
    _proto("aom_highbd_sad%sx4d" % _s, None, _X4D)
    _proto("aom_highbd_sad%sx3d" % _s, None, _X4D)
    _proto("aom_highbd_sad_skip_%sx4d" % _s, None, _X4D)
    for _pre in ("aom_", "aom_highbd_8_", "aom_highbd_10_", "aom_highbd_12_"):
        _proto(_pre + "variance" + _s, ctypes.c_uint, _VAR)
        _proto(_pre + "sub_pixel_variance" + _s, ctypes.c_uint32, _SUBVAR)
        _proto(_pre + "sub_pixel_avg_variance" + _s, ctypes.c_uint32, _SUBVAR + [_vp])
for _pre in ("aom_", "aom_highbd_8_", "aom_highbd_10_", "aom_highbd_12_"):
    _proto(_pre + "get16x16var", None, [_vp, _i32, _vp, _i32, _vp, _vp])
    _proto(_pre + "get8x8var", None, [_vp, _i32, _vp, _i32, _vp, _vp])
    for _s in ("16x16", "16x8", "8x16", "8x8"):
        _proto(_pre + "mse" + _s, ctypes.c_uint, _VAR)
_proto("aom_subtract_block", None, [_i32, _i32, _vp, _ssz, _vp, _ssz, _vp, _ssz])
_proto("aom_highbd_subtract_block", None, [_i32, _i32, _vp, _ssz, _vp, _ssz, _vp, _ssz])
_proto("aom_sse", ctypes.c_int64, [_vp, _i32, _vp, _i32, _i32, _i32])
_proto("aom_highbd_sse", ctypes.c_int64, [_vp, _i32, _vp, _i32, _i32, _i32])
_proto("aom_sum_squares_2d_i16", ctypes.c_uint64, [_vp, _i32, _i32, _i32])
for _n in ("4x4", "8x8", "16x16", "32x32"):
    _proto("aom_hadamard_" + _n, None, [_vp, _ssz, _vp])
for _n in ("8x8", "16x16", "32x32"):
    _proto("aom_highbd_hadamard_" + _n, None, [_vp, _ssz, _vp])
_proto("aom_satd", ctypes.c_int, [_vp, _i32])
for _n in ("8x8", "16x16", "8x8_dual"):
    _proto("aom_hadamard_lp_" + _n, None, [_vp, _ssz, _vp])
_proto("aom_satd_lp", ctypes.c_int, [_vp, _i32])
_proto("av1_block_error_lp", ctypes.c_int64, [_vp, _vp, _ssz])
_proto("aom_sum_sse_2d_i16", ctypes.c_uint64, [_vp, _i32, _i32, _i32, _vp])
_proto("aom_get_blk_sse_sum", None, [_vp, _i32, _i32, _i32, _vp, _vp])
_proto("av1_fwht4x4", None, [_vp, _vp, _i32])
_proto("av1_highbd_iwht4x4_16_add", None, [_vp, _vp, _i32, _i32])
_proto("av1_highbd_iwht4x4_1_add", None, [_vp, _vp, _i32, _i32])
_proto("av1_block_error", ctypes.c_int64, [_vp, _vp, _ssz, _vp])
_proto("av1_highbd_block_error", ctypes.c_int64, [_vp, _vp, _ssz, _vp, _i32])


def rtcd(name):
    """The ctypes function of shim `name` (reference rtcd name, no suffix)."""
    return _PROTOS[name]


# ------------------------------------------------------ per-call mirror --
def sad(w, h, src, src_stride, ref, ref_stride, highbd=False, skip=False, second_pred=None):
    pre = "aom_highbd_" if highbd else "aom_"
    if second_pred is not None:
        return _PROTOS["%ssad%dx%d_avg" % (pre, w, h)](
            _ptr(src, highbd), src_stride, _ptr(ref, highbd), ref_stride,
            _ptr(second_pred, highbd))
    name = ("%ssad_skip_%dx%d" if skip else "%ssad%dx%d") % (pre, w, h)
    return _PROTOS[name](_ptr(src, highbd), src_stride, _ptr(ref, highbd), ref_stride)


def sad_x4d(w, h, src, src_stride, refs, ref_stride, highbd=False, variant="x4d",
            second_pred=None):
    """variant: x4d, x3d, skip_x4d, x4d_avg (lowbd only).  Returns uint32[4]."""
    pre = "aom_highbd_" if highbd else "aom_"
    out = np.zeros(4, np.uint32)
    arr = (_vp * 4)(*[_ptr(r, highbd).value for r in refs])
    if variant == "skip_x4d":
        name = "%ssad_skip_%dx%dx4d" % (pre, w, h)
    else:
        name = "%ssad%dx%d%s" % (pre, w, h, variant)
    f = _PROTOS[name]
    if variant == "x4d_avg":
        f(_ptr(src, highbd), src_stride, ctypes.cast(arr, _vp), ref_stride,
          _ptr(second_pred, highbd), _ptr(out))
    else:
        f(_ptr(src, highbd), src_stride, ctypes.cast(arr, _vp), ref_stride, _ptr(out))
    return out


def _vpre(bd, highbd):
    return "aom_highbd_%d_" % bd if highbd else "aom_"


def variance(w, h, src, src_stride, ref, ref_stride, bd=8, highbd=False):
    """(var, sse) of aom[_highbd_bd]_variance{w}x{h}."""
    sse = np.zeros(1, np.uint32)
    v = _PROTOS["%svariance%dx%d" % (_vpre(bd, highbd), w, h)](
        _ptr(src, highbd), src_stride, _ptr(ref, highbd), ref_stride, _ptr(sse))
    return v, int(sse[0])


def sub_pixel_variance(w, h, src, src_stride, xoff, yoff, ref, ref_stride, bd=8, highbd=False,
                       second_pred=None):
    sse = np.zeros(1, np.uint32)
    pre = _vpre(bd, highbd)
    if second_pred is None:
        v = _PROTOS["%ssub_pixel_variance%dx%d" % (pre, w, h)](
            _ptr(src, highbd), src_stride, xoff, yoff, _ptr(ref, highbd), ref_stride, _ptr(sse))
    else:
        v = _PROTOS["%ssub_pixel_avg_variance%dx%d" % (pre, w, h)](
            _ptr(src, highbd), src_stride, xoff, yoff, _ptr(ref, highbd), ref_stride, _ptr(sse),
            _ptr(second_pred, highbd))
    return v, int(sse[0])


def mse(w, h, src, src_stride, ref, ref_stride, bd=8, highbd=False):
    sse = np.zeros(1, np.uint32)
    v = _PROTOS["%smse%dx%d" % (_vpre(bd, highbd), w, h)](
        _ptr(src, highbd), src_stride, _ptr(ref, highbd), ref_stride, _ptr(sse))
    return v, int(sse[0])


def get_var(n, src, src_stride, ref, ref_stride, bd=8, highbd=False):
    """(sse, sum) of aom[_highbd_bd]_get{n}x{n}var."""
    sse = np.zeros(1, np.uint32)
    sm = np.zeros(1, np.int32)
    _PROTOS["%sget%dx%dvar" % (_vpre(bd, highbd), n, n)](
        _ptr(src, highbd), src_stride, _ptr(ref, highbd), ref_stride, _ptr(sse), _ptr(sm))
    return int(sse[0]), int(sm[0])


def subtract_block(rows, cols, diff, diff_stride, src, src_stride, pred, pred_stride,
                   highbd=False):
    name = "aom_highbd_subtract_block" if highbd else "aom_subtract_block"
    _PROTOS[name](rows, cols, _ptr(diff), diff_stride, _ptr(src, highbd), src_stride,
                  _ptr(pred, highbd), pred_stride)


def sse(a, a_stride, b, b_stride, w, h, highbd=False):
    name = "aom_highbd_sse" if highbd else "aom_sse"
    return _PROTOS[name](_ptr(a, highbd), a_stride, _ptr(b, highbd), b_stride, w, h)


def sum_squares_2d_i16(src, stride, w, h):
    return _PROTOS["aom_sum_squares_2d_i16"](_ptr(src), stride, w, h)


def hadamard(n, src_diff, stride, highbd=False):
    out = np.zeros(n * n, np.int32)
    name = ("aom_highbd_hadamard_%dx%d" if highbd else "aom_hadamard_%dx%d") % (n, n)
    _PROTOS[name](_ptr(src_diff), stride, _ptr(out))
    return out


def satd(coeff, length):
    return _PROTOS["aom_satd"](_ptr(coeff), length)


def hadamard_lp(n, src_diff, stride, dual=False):
    """aom_hadamard_lp_{8x8,16x16} / _8x8_dual: int16 coefficients."""
    out = np.zeros(n * n * (2 if dual else 1), np.int16)
    name = "aom_hadamard_lp_8x8_dual" if dual else "aom_hadamard_lp_%dx%d" % (n, n)
    _PROTOS[name](_ptr(src_diff), stride, _ptr(out))
    return out


def satd_lp(coeff, length):
    return _PROTOS["aom_satd_lp"](_ptr(np.ascontiguousarray(coeff, np.int16)), length)


def block_error_lp(coeff, dqcoeff, n):
    return _PROTOS["av1_block_error_lp"](_ptr(np.ascontiguousarray(coeff, np.int16)),
                                         _ptr(np.ascontiguousarray(dqcoeff, np.int16)), n)


def sum_sse_2d_i16(src, stride, w, h, sum_in=0):
    """aom_sum_sse_2d_i16: (sse, *sum after the call)."""
    sm = np.array([sum_in], np.int32)
    v = _PROTOS["aom_sum_sse_2d_i16"](_ptr(src), stride, w, h, _ptr(sm))
    return v, int(sm[0])


def get_blk_sse_sum(src, stride, w, h):
    """aom_get_blk_sse_sum: (x_sum, x2_sum)."""
    sm = np.zeros(1, np.int32)
    ss = np.zeros(1, np.int64)
    _PROTOS["aom_get_blk_sse_sum"](_ptr(src), stride, w, h, _ptr(sm), _ptr(ss))
    return int(sm[0]), int(ss[0])


def fwht4x4(src_diff, stride):
    out = np.zeros(16, np.int32)
    _PROTOS["av1_fwht4x4"](_ptr(src_diff), _ptr(out), stride)
    return out


def iwht4x4_add(coeff, dst, stride, bd, full=True):
    """av1_highbd_iwht4x4_16_add (full) / _1_add on a uint16 view (tagged
    pointer, like the reference's callers)."""
    name = "av1_highbd_iwht4x4_16_add" if full else "av1_highbd_iwht4x4_1_add"
    _PROTOS[name](_ptr(np.ascontiguousarray(coeff, np.int32)), _ptr(dst, True), stride, bd)


def block_error(coeff, dqcoeff, n, bd=None):
    """(error, ssz): av1_block_error (bd None) / av1_highbd_block_error."""
    ssz = np.zeros(1, np.int64)
    if bd is None:
        e = _PROTOS["av1_block_error"](_ptr(coeff), _ptr(dqcoeff), n, _ptr(ssz))
    else:
        e = _PROTOS["av1_highbd_block_error"](_ptr(coeff), _ptr(dqcoeff), n, _ptr(ssz), bd)
    return e, int(ssz[0])


# ------------------------------------------------------------ batch layer --
for _n, _a in (
        ("lavish_sad_batch", [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _i32, _i32, _i32, _vp, _i32,
                              _vp, _vp]),
        ("lavish_variance_batch", [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _i32, _i32, _i32, _i32,
                                   _vp, _vp, _vp, _vp, _vp, _vp]),
        ("lavish_subtract_batch", [_i32, _i32, _vp, _i32, _vp, _i32, _vp, _i32, _vp, _i32, _i32,
                                   _vp]),
        ("lavish_sum_squares_batch", [_vp, _i32, _i32, _i32, _vp, _i32, _vp, _vp]),
        ("lavish_hadamard_batch", [_i32, _i32, _vp, _i32, _vp, _i32, _vp, _vp]),
        ("lavish_satd_batch", [_vp, _i32, _i32, _vp, _vp]),
        ("lavish_block_error_batch", [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp]),
        ("lavish_hadamard_lp_batch", [_i32, _vp, _i32, _vp, _i32, _vp, _vp]),
        ("lavish_satd_lp_batch", [_vp, _i32, _i32, _vp, _vp]),
        ("lavish_block_error_lp_batch", [_vp, _vp, _i32, _i32, _vp, _vp]),
        ("lavish_sum_sse_batch", [_vp, _i32, _i32, _i32, _vp, _i32, _vp, _vp, _vp]),
        ("lavish_fwht4x4_batch", [_vp, _i32, _vp, _i32, _vp, _vp]),
        ("lavish_iwht4x4_add_batch", [_vp, _vp, _i32, _vp, _i32, _i32, _i32, _vp])):
    getattr(_lib, _n).argtypes = _a
    getattr(_lib, _n).restype = _i32


def jobs_tensor(jobs, device):
    """Upload a JOB_DTYPE numpy array as a device byte tensor."""
    import torch
    assert jobs.dtype == JOB_DTYPE
    return torch.from_numpy(np.ascontiguousarray(jobs).view(np.uint8).copy()).to(device)


def _d(t):
    if t is None:
        return None
    assert t.dim() == 1 or t.stride(-1) == 1, "rows must be contiguous"
    return _vp(t.data_ptr())


def _check(rc, name):
    if rc != 0:
        raise ValueError("%s rejected its arguments (rc=%d)" % (name, rc))


def sad_batch(src, ref, w, h, jobs, nrefs=1, mode=0, second_pred=None, stream=None):
    """src/ref: 2-D device tensors (uint8, or int16/uint16-as-int16 for highbd).
    jobs: device tensor from jobs_tensor.  Returns uint32 SADs [njobs, nrefs]
    (as int64 tensor)."""
    import torch
    highbd = src.element_size() == 2
    nj = jobs.numel() // JOB_DTYPE.itemsize
    out = torch.empty((nj, nrefs), dtype=torch.int32, device=src.device)
    _check(_lib.lavish_sad_batch(_d(src), src.stride(0), _d(ref), ref.stride(0), w, h, _d(jobs),
                                 nj, nrefs, mode, _d(second_pred), int(highbd), _d(out),
                                 _stream_ptr(stream)), "lavish_sad_batch")
    return out.to(torch.int64) & 0xFFFFFFFF


def variance_batch(a, b, w, h, jobs, kind=0, bit_depth=8, second_pred=None, stream=None):
    """Returns dict var/sse/sum/sse64 tensors (unsigned values widened to int64)."""
    import torch
    highbd = a.element_size() == 2
    nj = jobs.numel() // JOB_DTYPE.itemsize
    dev = a.device
    var = torch.empty(nj, dtype=torch.int32, device=dev)
    sse_ = torch.empty(nj, dtype=torch.int32, device=dev)
    sm = torch.empty(nj, dtype=torch.int32, device=dev)
    s64 = torch.empty(nj, dtype=torch.int64, device=dev)
    _check(_lib.lavish_variance_batch(_d(a), a.stride(0), _d(b), b.stride(0), w, h, _d(jobs), nj,
                                      kind, bit_depth, int(highbd), _d(second_pred), _d(var),
                                      _d(sse_), _d(sm), _d(s64), _stream_ptr(stream)),
           "lavish_variance_batch")
    return {"var": var.to(torch.int64) & 0xFFFFFFFF, "sse": sse_.to(torch.int64) & 0xFFFFFFFF,
            "sum": sm, "sse64": s64}


def subtract_batch(rows, cols, diff, src, pred, jobs, stream=None):
    highbd = src.element_size() == 2
    nj = jobs.numel() // JOB_DTYPE.itemsize
    _check(_lib.lavish_subtract_batch(rows, cols, _d(diff), diff.stride(0), _d(src),
                                      src.stride(0), _d(pred), pred.stride(0), _d(jobs), nj,
                                      int(highbd), _stream_ptr(stream)),
           "lavish_subtract_batch")


def sum_squares_batch(src, w, h, jobs, stream=None):
    import torch
    nj = jobs.numel() // JOB_DTYPE.itemsize
    out = torch.empty(nj, dtype=torch.int64, device=src.device)
    _check(_lib.lavish_sum_squares_batch(_d(src), src.stride(0), w, h, _d(jobs), nj, _d(out),
                                         _stream_ptr(stream)), "lavish_sum_squares_batch")
    return out


def hadamard_batch(n, src_diff, jobs, ncoeff_words, highbd=False, stream=None):
    import torch
    nj = jobs.numel() // JOB_DTYPE.itemsize
    out = torch.zeros(ncoeff_words, dtype=torch.int32, device=src_diff.device)
    _check(_lib.lavish_hadamard_batch(n, int(highbd), _d(src_diff), src_diff.stride(0), _d(jobs),
                                      nj, _d(out), _stream_ptr(stream)), "lavish_hadamard_batch")
    return out


def satd_batch(coeff, stream=None):
    import torch
    nb, length = coeff.shape
    out = torch.empty(nb, dtype=torch.int32, device=coeff.device)
    _check(_lib.lavish_satd_batch(_d(coeff), length, nb, _d(out), _stream_ptr(stream)),
           "lavish_satd_batch")
    return out


def block_error_batch(coeff, dqcoeff, bit_depth=0, stream=None):
    import torch
    nb, n = coeff.shape
    err = torch.empty(nb, dtype=torch.int64, device=coeff.device)
    ssz = torch.empty(nb, dtype=torch.int64, device=coeff.device)
    _check(_lib.lavish_block_error_batch(_d(coeff), _d(dqcoeff), n, nb, bit_depth, _d(err),
                                         _d(ssz), _stream_ptr(stream)),
           "lavish_block_error_batch")
    return err, ssz


def sum_sse_batch(src, w, h, jobs, stream=None):
    """(sum int32, sse int64) tensors of lavish_sum_sse_batch."""
    import torch
    nj = jobs.numel() // JOB_DTYPE.itemsize
    sm = torch.empty(nj, dtype=torch.int32, device=src.device)
    ss = torch.empty(nj, dtype=torch.int64, device=src.device)
    _check(_lib.lavish_sum_sse_batch(_d(src), src.stride(0), w, h, _d(jobs), nj, _d(sm), _d(ss),
                                     _stream_ptr(stream)), "lavish_sum_sse_batch")
    return sm, ss


def hadamard_lp_batch(n, src_diff, jobs, ncoeff_words, stream=None):
    import torch
    nj = jobs.numel() // JOB_DTYPE.itemsize
    out = torch.zeros(ncoeff_words, dtype=torch.int16, device=src_diff.device)
    _check(_lib.lavish_hadamard_lp_batch(n, _d(src_diff), src_diff.stride(0), _d(jobs), nj,
                                         _d(out), _stream_ptr(stream)), "lavish_hadamard_lp_batch")
    return out


def fwht4x4_batch(src_diff, jobs, ncoeff_words, stream=None):
    import torch
    nj = jobs.numel() // JOB_DTYPE.itemsize
    out = torch.zeros(ncoeff_words, dtype=torch.int32, device=src_diff.device)
    _check(_lib.lavish_fwht4x4_batch(_d(src_diff), src_diff.stride(0), _d(jobs), nj, _d(out),
                                     _stream_ptr(stream)), "lavish_fwht4x4_batch")
    return out


def iwht4x4_add_batch(dqcoeff, jobs, dst, bit_depth, stream=None):
    """lavish_iwht4x4_add_batch; jobs: device tensor of lavish_dsp.INV_JOB_DTYPE
    records; dst: uint8 (bd 8) or int16-viewed uint16 plane, updated in place."""
    from . import INV_JOB_DTYPE
    nj = jobs.numel() // INV_JOB_DTYPE.itemsize
    _check(_lib.lavish_iwht4x4_add_batch(_d(dqcoeff), _d(jobs), nj, _d(dst), dst.stride(0),
                                         bit_depth, int(dst.element_size() == 2),
                                         _stream_ptr(stream)), "lavish_iwht4x4_add_batch")
