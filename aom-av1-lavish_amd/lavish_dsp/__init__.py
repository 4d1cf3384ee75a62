"""lavish_dsp -- host-side mirror of the reference's RTCD DSP entry points for
the MI355X backend (liblavish_hip.so).

Two layers, as in include/lavish_dsp.h:

* per-call functions named exactly like the reference's rtcd entries
  (``av1_fwd_txfm2d_4x4``, ``av1_quantize_fp``, ``aom_quantize_b_32x32`` ...)
  taking numpy arrays with the reference's argument meaning -- they call the
  ``*_hip`` C shims, which run the HIP kernels;
* batch functions (``txq_plane``, ``quantize_batch``) on torch device tensors,
  launched asynchronously on the current torch stream.

There is no CPU fallback: if liblavish_hip.so is missing the import fails.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# LAVISH_HIP_LIB: an alternative build of the same library (A/B experiments)
LIB_PATH = os.environ.get("LAVISH_HIP_LIB") or os.path.join(os.path.dirname(_HERE),
                                                            "liblavish_hip.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "liblavish_hip.so not found at %s -- build it with `make -C aom-av1-lavish_amd` "
        "(or __graft_entry__.build()); there is no CPU fallback" % LIB_PATH)

# One HIP runtime per process: torch ships its own libamdhip64.so.7 (same
# soname as /opt/rocm's).  Whichever loads first serves both; device
# tensors come from torch, so load torch's first and let the library bind to
# it (loading ours first left its launches seeing no device on the MI355X box).
try:
    import torch  # noqa: F401
except ImportError:  # a C-only consumer: the library brings /opt/rocm's runtime
    pass

_lib = ctypes.CDLL(LIB_PATH)

TX_SIZES = ["4x4", "8x8", "16x16", "32x32", "64x64", "4x8", "8x4", "8x16", "16x8",
            "16x32", "32x16", "32x64", "64x32", "4x16", "16x4", "8x32", "32x8", "16x64",
            "64x16"]
TX_W = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
TX_H = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]
TX_TYPES = ["DCT_DCT", "ADST_DCT", "DCT_ADST", "ADST_ADST", "FLIPADST_DCT", "DCT_FLIPADST",
            "FLIPADST_FLIPADST", "ADST_FLIPADST", "FLIPADST_ADST", "IDTX", "V_DCT", "H_DCT",
            "V_ADST", "H_ADST", "V_FLIPADST", "H_FLIPADST"]
QUANT_FP, QUANT_B, QUANT_NONE = 0, 1, 2


def max_eob(tx_size):
    """av1_get_max_eob (av1/common/blockd.h:1596-1604)."""
    if tx_size in (17, 18):
        return 512
    if TX_W[tx_size] == 64 or TX_H[tx_size] == 64:
        return 1024
    return TX_W[tx_size] * TX_H[tx_size]


def tx_scale(tx_size):
    """av1_get_tx_scale (av1/common/idct.c:24-28)."""
    p = TX_W[tx_size] * TX_H[tx_size]
    return int(p > 256) + int(p > 1024)


def tx_type_valid(tx_size, tx_type):
    m = max(TX_W[tx_size], TX_H[tx_size])
    if m == 64:
        return tx_type == 0
    if m == 32:
        return tx_type in (0, 9)
    return 0 <= tx_type < 16


def valid_type_mask(tx_size):
    return sum(1 << t for t in range(16) if tx_type_valid(tx_size, t))


class TxfmParam(ctypes.Structure):
    """TxfmParam (aom_dsp/txfm_common.h:89-101)."""
    _fields_ = [("tx_type", ctypes.c_uint8), ("tx_size", ctypes.c_uint8),
                ("lossless", ctypes.c_int), ("bd", ctypes.c_int), ("is_hbd", ctypes.c_int),
                ("tx_set_type", ctypes.c_uint8), ("eob", ctypes.c_int)]


class QuantParams(ctypes.Structure):
    """LavishQuantParams: [0] = DC, [1] = AC."""
    _fields_ = [(n, ctypes.c_int16 * 2) for n in
                ("zbin", "round", "quant", "quant_shift", "dequant")]

    def as_dict(self):
        return {n: np.array(list(getattr(self, n)), np.int16) for n, _ in self._fields_}


_vp, _i32, _i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_lib.lavish_hip_status.restype = _i32
_lib.lavish_hip_status_string.restype = ctypes.c_char_p
_lib.lavish_hip_set_abort_on_error.argtypes = [_i32]
_lib.lavish_hip_init.argtypes = [_i32]
_lib.lavish_hip_version.restype = _i32
_lib.lavish_build_quant_params.argtypes = [_i32, _i32, _i32, _i32, _i32,
                                           ctypes.POINTER(QuantParams)]
_lib.lavish_scan.restype = ctypes.POINTER(ctypes.c_int16)
_lib.lavish_scan.argtypes = [_i32, _i32]
_lib.lavish_iscan.restype = ctypes.POINTER(ctypes.c_int16)
_lib.lavish_iscan.argtypes = [_i32, _i32]
_lib.lavish_txq_plane.argtypes = [_vp, _i32, _i32, _i32, _i32, ctypes.c_uint32, _i32, _i32,
                                  ctypes.POINTER(QuantParams), _vp, _vp, _vp, _vp, _vp]
_lib.lavish_txq_plane.restype = _i32
_lib.lavish_txq_frame.argtypes = [_vp, _i32, _i32, _i32, ctypes.c_uint32, _vp, _i32, _i32,
                                  ctypes.POINTER(QuantParams), _vp, _vp, _vp, _vp]
_lib.lavish_txq_frame.restype = _i32
_lib.lavish_quantize_batch.argtypes = [_vp, _i32, _i32, _vp, _vp, _i32, _i32, _i32,
                                       ctypes.POINTER(QuantParams), _vp, _vp, _vp, _vp]
_lib.lavish_quantize_batch.restype = _i32

_FWD2D = {}
for _s, _name in enumerate(TX_SIZES):
    f = getattr(_lib, "av1_fwd_txfm2d_%s_hip" % _name)
    f.argtypes = [_vp, _vp, _i32, ctypes.c_uint8, _i32]
    f.restype = None
    _FWD2D[_s] = f
_lib.av1_lowbd_fwd_txfm_hip.argtypes = [_vp, _vp, _i32, ctypes.POINTER(TxfmParam)]


class PlaneQuant(ctypes.Structure):
    """LavishPlaneQuant: MACROBLOCK_PLANE's *_QTX tables ([0] DC, [1] AC)."""
    _fields_ = [(n, ctypes.c_int16 * 2) for n in
                ("zbin", "round_fp", "quant_fp", "round", "quant", "quant_shift", "dequant")]


_lib.lavish_build_plane_quant.argtypes = [_i32, _i32, _i32, _i32, ctypes.POINTER(PlaneQuant)]
_lib.lavish_build_plane_quant.restype = _i32
_lib.lavish_av1_quant_batch.argtypes = [_vp, _i32, _i32, _i32, _i32, ctypes.POINTER(PlaneQuant),
                                        _i32, _i32, ctypes.c_uint32, _i32, _vp, _vp, _vp, _vp,
                                        _vp, _vp]
_lib.lavish_av1_quant_batch.restype = _i32
# xform_quant_idx of lavish_av1_quant_batch (AV1_XFORM_QUANT) + the satd gate
AV1_QUANT_FP, AV1_QUANT_B, AV1_QUANT_DC, AV1_QUANT_SKIP, AV1_QUANT_SATD_GATE = range(5)


def build_plane_quant(bit_depth, qindex, quant_sharpness=0, y_dc_delta_q=0):
    q = PlaneQuant()
    if _lib.lavish_build_plane_quant(bit_depth, qindex, quant_sharpness, y_dc_delta_q,
                                     ctypes.byref(q)) != 0:
        raise ValueError("lavish_build_plane_quant(%d, %d) failed" % (bit_depth, qindex))
    return q


def av1_quant_batch(coeff, tx_size, tx_type, bit_depth, pq, mode, skip_trellis=0,
                    threshold=0xFFFFFFFF, qstep=0, dc_only=None, stream=None):
    """lavish_av1_quant_batch over a device int32 [nblocks, n] coefficient
    tensor (n = max_eob(tx_size)); returns (qcoeff, dqcoeff, eob, flags)."""
    import torch
    n = max_eob(tx_size)
    assert coeff.dtype == torch.int32 and coeff.is_contiguous() and coeff.shape[-1] == n
    nb = coeff.numel() // n
    qc, dq = torch.empty_like(coeff), torch.empty_like(coeff)
    eob = torch.empty(nb, dtype=torch.int16, device=coeff.device)
    flags = torch.empty(nb, dtype=torch.uint8, device=coeff.device)
    if dc_only is not None:
        assert dc_only.dtype == torch.uint8 and dc_only.numel() >= nb and dc_only.is_cuda
    rc = _lib.lavish_av1_quant_batch(_p_t(coeff), nb, tx_size, tx_type, bit_depth,
                                     ctypes.byref(pq), mode, skip_trellis, threshold, qstep,
                                     _p_t(dc_only) if dc_only is not None else None, _p_t(qc),
                                     _p_t(dq), _p_t(eob), _p_t(flags), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_av1_quant_batch rejected its arguments (rc=%d)" % rc)
    return qc, dq, eob, flags


def _p_t(t):
    return ctypes.c_void_p(t.data_ptr())


class BitDepthInfo(ctypes.Structure):
    """BitDepthInfo (av1/common/blockd.h:952-960)."""
    _fields_ = [("bit_depth", ctypes.c_int), ("use_highbitdepth_buf", ctypes.c_int)]


_lib.av1_quick_txfm_hip.argtypes = [_i32, ctypes.c_uint8, BitDepthInfo, _vp, _i32, _vp]
_lib.av1_quick_txfm_hip.restype = None

_QARGS = [_vp, ctypes.c_ssize_t, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
_QUANT_NAMES = ["av1_quantize_fp", "av1_quantize_fp_32x32", "av1_quantize_fp_64x64",
                "aom_quantize_b", "aom_quantize_b_32x32", "aom_quantize_b_64x64",
                "aom_highbd_quantize_b", "aom_highbd_quantize_b_32x32",
                "aom_highbd_quantize_b_64x64"]
for _n in _QUANT_NAMES:
    getattr(_lib, _n + "_hip").argtypes = _QARGS
_lib.av1_highbd_quantize_fp_hip.argtypes = _QARGS + [_i32]


def lib():
    return _lib


def status():
    return _lib.lavish_hip_status(), _lib.lavish_hip_status_string().decode()


_lib.lavish_set_fan_width.argtypes = [ctypes.c_int]
_lib.lavish_set_fan_width.restype = ctypes.c_int


def set_fan_width(streams):
    """lavish_set_fan_width: the streams rdo_frame / rdo_reconstruct deal
    their per-size kernels over (3, the default, or 1: all on the caller's
    stream -- isolated per-kernel timings under a profiler)."""
    rc = _lib.lavish_set_fan_width(int(streams))
    if rc != 0:
        raise ValueError("lavish_set_fan_width(%r): %d" % (streams, rc))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- tables --
def build_quant_params(bit_depth, qindex, kind=QUANT_FP, quant_sharpness=0, y_dc_delta_q=0):
    """av1_build_quantizer row for luma at `qindex` (av1/encoder/av1_quantize.c:590)."""
    q = QuantParams()
    rc = _lib.lavish_build_quant_params(bit_depth, qindex, quant_sharpness, y_dc_delta_q,
                                        kind, ctypes.byref(q))
    if rc != 0:
        raise ValueError("lavish_build_quant_params(%d, %d) failed" % (bit_depth, qindex))
    return q


def scan_order(tx_size, tx_type):
    """(scan, iscan) of av1_scan_orders[tx_size][tx_type]."""
    n = min(TX_W[tx_size], 32) * min(TX_H[tx_size], 32)
    s = np.ctypeslib.as_array(_lib.lavish_scan(tx_size, tx_type), shape=(n,)).copy()
    i = np.ctypeslib.as_array(_lib.lavish_iscan(tx_size, tx_type), shape=(n,)).copy()
    return s, i


# ------------------------------------------------- per-call RTCD mirror --
def _fwd2d(tx_size):
    def fn(input, output, stride, tx_type, bd):
        """av1_fwd_txfm2d_%s (av1/common/av1_rtcd_defs.pl:358-399): int16
        residual rows of `stride` -> int32 coefficient buffer (column-major)."""
        assert input.dtype == np.int16 and output.dtype == np.int32
        assert input.size >= (TX_H[tx_size] - 1) * stride + TX_W[tx_size]
        assert output.size >= TX_W[tx_size] * TX_H[tx_size]
        _FWD2D[tx_size](_p(input), _p(output), stride, tx_type, bd)
    fn.__name__ = "av1_fwd_txfm2d_" + TX_SIZES[tx_size]
    return fn


for _s in _FWD2D:
    globals()["av1_fwd_txfm2d_" + TX_SIZES[_s]] = _fwd2d(_s)


def av1_lowbd_fwd_txfm(src_diff, coeff, diff_stride, txfm_param):
    _lib.av1_lowbd_fwd_txfm_hip(_p(src_diff), _p(coeff), diff_stride, ctypes.byref(txfm_param))


def av1_quick_txfm(use_hadamard, tx_size, bd_info, src_diff, src_stride, coeff):
    """av1_quick_txfm (av1/encoder/hybrid_fwd_txfm.c:315-336)."""
    _lib.av1_quick_txfm_hip(int(use_hadamard), tx_size, bd_info, _p(src_diff), src_stride,
                            _p(coeff))


def _quant(name):
    cfn = getattr(_lib, name + "_hip")

    def fn(coeff_ptr, n_coeffs, zbin_ptr, round_ptr, quant_ptr, quant_shift_ptr, qcoeff_ptr,
           dqcoeff_ptr, dequant_ptr, eob_ptr, scan, iscan):
        cfn(_p(coeff_ptr), n_coeffs, _p(zbin_ptr), _p(round_ptr), _p(quant_ptr),
            _p(quant_shift_ptr), _p(qcoeff_ptr), _p(dqcoeff_ptr), _p(dequant_ptr), _p(eob_ptr),
            _p(scan), _p(iscan))
    fn.__name__ = name
    return fn


for _n in _QUANT_NAMES:
    globals()[_n] = _quant(_n)


def av1_highbd_quantize_fp(coeff_ptr, count, zbin_ptr, round_ptr, quant_ptr, quant_shift_ptr,
                           qcoeff_ptr, dqcoeff_ptr, dequant_ptr, eob_ptr, scan, iscan,
                           log_scale):
    _lib.av1_highbd_quantize_fp_hip(_p(coeff_ptr), count, _p(zbin_ptr), _p(round_ptr),
                                    _p(quant_ptr), _p(quant_shift_ptr), _p(qcoeff_ptr),
                                    _p(dqcoeff_ptr), _p(dequant_ptr), _p(eob_ptr), _p(scan),
                                    _p(iscan), log_scale)


# ---------------------------------------------------------- batch layer --
def _stream_ptr(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def txq_plane_out(residual, tx_size, type_mask, with_coeff=False):
    """Allocate the output tensors of txq_plane for a residual plane."""
    import torch
    H, W = residual.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    nt = bin(type_mask).count("1")
    n = max_eob(tx_size)
    dev = residual.device
    out = {
        "qcoeff": torch.empty((nt, nb, n), dtype=torch.int32, device=dev),
        "dqcoeff": torch.empty((nt, nb, n), dtype=torch.int32, device=dev),
        "eob": torch.empty((nt, nb), dtype=torch.int16, device=dev),
    }
    if with_coeff:
        out["coeff"] = torch.empty((nt, nb, n), dtype=torch.int32, device=dev)
    return out


def txq_plane(residual, tx_size, type_mask, qp, bit_depth=8, quant_kind=QUANT_FP, out=None,
              stride=None, width=None, height=None, with_coeff=False, stream=None):
    """Batch fwd transform + quantize of every full `tx_size` block of a device
    int16 residual plane for every type in `type_mask` (see lavish_txq_plane).
    Returns dict of tensors qcoeff/dqcoeff [slot, block, n], eob [slot, block]
    (uint16 values stored in an int16 tensor)."""
    import torch
    assert residual.dtype == torch.int16 and residual.is_cuda
    assert residual.stride(1) == 1, "residual rows must be contiguous"
    if not 0 <= tx_size < len(TX_SIZES):
        raise ValueError("tx_size %d out of range" % tx_size)
    Hh, Ww = residual.shape
    stride = residual.stride(0) if stride is None else stride
    width = Ww if width is None else width
    height = Hh if height is None else height
    if out is None:
        out = txq_plane_out(residual[:height, :width], tx_size, type_mask, with_coeff)
    coeff = out.get("coeff")
    rc = _lib.lavish_txq_plane(
        ctypes.c_void_p(residual.data_ptr()), stride, width, height, tx_size, type_mask,
        bit_depth, quant_kind, ctypes.byref(qp) if qp is not None else None,
        ctypes.c_void_p(out["qcoeff"].data_ptr()), ctypes.c_void_p(out["dqcoeff"].data_ptr()),
        ctypes.c_void_p(out["eob"].data_ptr()),
        ctypes.c_void_p(coeff.data_ptr()) if coeff is not None else None, _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_txq_plane rejected arguments (rc=%d)" % rc)
    return out


class FrameOutputs:
    """Per-size output tensors of txq_frame plus the pointer tables the C ABI
    takes (built once, reused every call)."""

    def __init__(self, residual, sizes, type_masks=None):
        self.sizes = list(sizes)
        self.type_masks = {s: (type_masks or {}).get(s, valid_type_mask(s)) for s in self.sizes}
        self.outs = {s: txq_plane_out(residual, s, self.type_masks[s]) for s in self.sizes}
        self.size_mask = sum(1 << s for s in self.sizes)
        P19 = ctypes.c_void_p * 19
        self.tm = (ctypes.c_uint32 * 19)(*[self.type_masks.get(s, 0) for s in range(19)])
        self.q = P19(*[self.outs[s]["qcoeff"].data_ptr() if s in self.outs else 0 for s in range(19)])
        self.dq = P19(*[self.outs[s]["dqcoeff"].data_ptr() if s in self.outs else 0 for s in range(19)])
        self.eob = P19(*[self.outs[s]["eob"].data_ptr() if s in self.outs else 0 for s in range(19)])


def txq_frame(residual, frame_out, qp, bit_depth=8, quant_kind=QUANT_FP, stream=None,
              size_mask=None):
    """lavish_txq_frame: every size of `frame_out` (or of those, the sizes in
    size_mask) over one residual plane."""
    import torch
    assert residual.dtype == torch.int16 and residual.is_cuda
    assert residual.stride(1) == 1, "residual rows must be contiguous"
    H, W = residual.shape
    mask = frame_out.size_mask if size_mask is None else frame_out.size_mask & size_mask
    rc = _lib.lavish_txq_frame(ctypes.c_void_p(residual.data_ptr()), residual.stride(0), W, H,
                               mask, frame_out.tm, bit_depth, quant_kind,
                               ctypes.byref(qp), frame_out.q, frame_out.dq, frame_out.eob,
                               _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_txq_frame rejected arguments (rc=%d)" % rc)
    return frame_out.outs


def quantize_batch(coeff, scan, log_scale, qp, bit_depth=8, quant_kind=QUANT_FP, stream=None):
    """Quantize coeff[nblocks, n] (device int32) with one scan order."""
    import torch
    nb, n = coeff.shape
    q = torch.empty_like(coeff)
    dq = torch.empty_like(coeff)
    eob = torch.empty((nb,), dtype=torch.int16, device=coeff.device)
    rc = _lib.lavish_quantize_batch(
        ctypes.c_void_p(coeff.data_ptr()), n, nb, ctypes.c_void_p(scan.data_ptr()), None,
        log_scale, bit_depth, quant_kind, ctypes.byref(qp), ctypes.c_void_p(q.data_ptr()),
        ctypes.c_void_p(dq.data_ptr()), ctypes.c_void_p(eob.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_quantize_batch rejected arguments (rc=%d)" % rc)
    return q, dq, eob


# ------------------------------------------------- inverse transforms --
INV_JOB_DTYPE = np.dtype([("dst_off", "<i8"), ("coeff_off", "<i8"), ("tx_type", "<i4"),
                          ("eob", "<i4")], align=True)
assert INV_JOB_DTYPE.itemsize == 24
_lib.lavish_inv_txfm_add_batch.argtypes = [_vp, _i32, _vp, _i32, _vp, _i32, _i32, _i32, _vp]
_lib.lavish_inv_txfm_add_batch.restype = _i32
for _s in range(19):
    _f = getattr(_lib, "av1_inv_txfm2d_add_%s_hip" % TX_SIZES[_s])
    _f.argtypes = [_vp, _vp, _i32, ctypes.c_uint8, _i32]
    _f.restype = None
_lib.av1_inv_txfm_add_hip.argtypes = [_vp, _vp, _i32, ctypes.POINTER(TxfmParam)]
_lib.av1_highbd_inv_txfm_add_hip.argtypes = [_vp, _vp, _i32, ctypes.POINTER(TxfmParam)]


def av1_inv_txfm2d_add(tx_size, input, output, stride, tx_type, bd):
    """av1_inv_txfm2d_add_{WxH} (av1/common/av1_rtcd_defs.pl:222-243): int32
    dqcoeff (reference layout) added into a uint16 destination in place."""
    assert input.dtype == np.int32 and output.dtype == np.uint16
    assert output.strides[-1] == 2
    getattr(_lib, "av1_inv_txfm2d_add_%s_hip" % TX_SIZES[tx_size])(
        _p(input), _p(output), stride, tx_type, bd)


def av1_inv_txfm_add(dqcoeff, dst, stride, txfm_param):
    """av1_inv_txfm_add (u8 destination) / av1_highbd_inv_txfm_add when
    txfm_param.is_hbd (u16 destination, tagged pointer as the reference)."""
    if txfm_param.is_hbd:
        assert dst.dtype == np.uint16
        _lib.av1_highbd_inv_txfm_add_hip(_p(dqcoeff), ctypes.c_void_p(dst.ctypes.data >> 1),
                                         stride, ctypes.byref(txfm_param))
    else:
        assert dst.dtype == np.uint8
        _lib.av1_inv_txfm_add_hip(_p(dqcoeff), _p(dst), stride, ctypes.byref(txfm_param))


def inv_txfm_add_batch(dqcoeff, tx_size, jobs, dst, bit_depth=8, stream=None):
    """lavish_inv_txfm_add_batch on device tensors: dqcoeff int32 (flat),
    jobs a device byte tensor of INV_JOB_DTYPE records, dst a 2-D uint8
    (bit_depth 8) or int16-viewed uint16 plane updated in place."""
    import torch
    assert dst.stride(1) == 1
    highbd = dst.element_size() == 2
    nj = jobs.numel() // INV_JOB_DTYPE.itemsize
    rc = _lib.lavish_inv_txfm_add_batch(ctypes.c_void_p(dqcoeff.data_ptr()), tx_size,
                                        ctypes.c_void_p(jobs.data_ptr()), nj,
                                        ctypes.c_void_p(dst.data_ptr()), dst.stride(0),
                                        bit_depth, int(highbd), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_inv_txfm_add_batch rejected its arguments (rc=%d)" % rc)


# ---------------------------------------------------------------- C4 RDO --
RDO_DTYPE = np.dtype([("best_type", "<i4"), ("eob", "<i4"), ("rate", "<i4"), ("satd", "<i4"),
                      ("dist", "<i8"), ("sse", "<i8"), ("rdcost", "<i8")], align=True)
assert RDO_DTYPE.itemsize == 40
_lib.lavish_rdo_plane.argtypes = [_vp, _vp, _i32, _i32, _i32, _i32, ctypes.c_uint32, _i32,
                                  ctypes.POINTER(QuantParams), _i32, _vp, _vp, _vp, _vp]
_lib.lavish_rdo_plane.restype = _i32
_lib.lavish_rdo_plane_px.argtypes = _lib.lavish_rdo_plane.argtypes
_lib.lavish_rdo_plane_px.restype = _i32


def rdo_out(src, tx_size):
    """Output tensors of rdo_plane for a u16 plane (stored as int16)."""
    import torch
    H, W = src.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    n = max_eob(tx_size)
    dev = src.device
    return {"records": torch.empty(nb * RDO_DTYPE.itemsize, dtype=torch.uint8, device=dev),
            "qcoeff": torch.empty((nb, n), dtype=torch.int32, device=dev),
            "dqcoeff": torch.empty((nb, n), dtype=torch.int32, device=dev)}


def rdo_plane(src, pred, tx_size, type_mask, qp, rdmult, bit_depth=10, out=None, stream=None,
              px=False):
    """lavish_rdo_plane (C4) on device u16 planes held as int16 tensors;
    px=True: lavish_rdo_plane_px (pixel-domain distortion)."""
    import torch
    assert src.dtype == torch.int16 and pred.dtype == torch.int16
    assert src.shape == pred.shape and src.stride(1) == 1 and pred.stride(0) == src.stride(0)
    H, W = src.shape
    if out is None:
        out = rdo_out(src, tx_size)
    fn = _lib.lavish_rdo_plane_px if px else _lib.lavish_rdo_plane
    rc = fn(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(pred.data_ptr()),
                               src.stride(0), W, H, tx_size, type_mask, bit_depth,
                               ctypes.byref(qp), rdmult,
                               ctypes.c_void_p(out["records"].data_ptr()),
                               ctypes.c_void_p(out["qcoeff"].data_ptr()),
                               ctypes.c_void_p(out["dqcoeff"].data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_rdo_plane rejected its arguments (rc=%d)" % rc)
    return out


_lib.lavish_rdo_plane_masked.argtypes = [_vp, _vp, _i32, _i32, _i32, _i32, ctypes.c_uint32, _i32,
                                         ctypes.POINTER(QuantParams), _i32, _vp, _vp, _i32, _vp,
                                         _vp, _vp, _vp]
_lib.lavish_rdo_plane_masked.restype = _i32


def rdo_plane_masked(src, pred, tx_size, type_mask, qp, rdmult, block_mask=None,
                     block_map=None, bit_depth=10, px=False, out=None, stream=None):
    """lavish_rdo_plane_masked: C4 with the per-block allowed_tx_mask (device
    int16 / uint16 tensor [block]) and search order (device uint8 [block, 16])
    that lavish_prune_tx_2d_batch produces."""
    import torch
    assert src.dtype == torch.int16 and pred.dtype == torch.int16
    assert src.is_cuda and pred.is_cuda and src.shape == pred.shape
    assert src.stride(1) == 1 and pred.stride(0) == src.stride(0)
    H, W = src.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    # the kernel reads block_mask[nb] (16-bit) and block_map[nb][16] (u8) on
    # the device: anything else would read out of bounds or host memory
    if block_mask is not None:
        assert block_mask.is_cuda and block_mask.dtype in (torch.int16, torch.uint16)
        assert block_mask.is_contiguous() and tuple(block_mask.shape) == (nb,)
    if block_map is not None:
        assert block_map.is_cuda and block_map.dtype == torch.uint8
        assert block_map.is_contiguous() and tuple(block_map.shape) == (nb, 16)
    if out is None:
        out = rdo_out(src, tx_size)
    rc = _lib.lavish_rdo_plane_masked(
        ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(pred.data_ptr()), src.stride(0), W, H,
        tx_size, type_mask, bit_depth, ctypes.byref(qp), rdmult,
        None if block_mask is None else ctypes.c_void_p(block_mask.data_ptr()),
        None if block_map is None else ctypes.c_void_p(block_map.data_ptr()), int(px),
        ctypes.c_void_p(out["records"].data_ptr()), ctypes.c_void_p(out["qcoeff"].data_ptr()),
        ctypes.c_void_p(out["dqcoeff"].data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_rdo_plane_masked rejected its arguments (rc=%d)" % rc)
    return out


def rdo_records(out):
    return out["records"].cpu().numpy().view(RDO_DTYPE)


_P19 = ctypes.c_void_p * 19
_lib.lavish_rdo_frame.argtypes = [_vp, _vp, _i32, _i32, _i32, ctypes.c_uint32, _vp, _i32,
                                  ctypes.POINTER(QuantParams), _i32, _vp, _vp, _vp, _vp]
_lib.lavish_rdo_frame.restype = _i32
_lib.lavish_rdo_frame_px.argtypes = _lib.lavish_rdo_frame.argtypes
_lib.lavish_rdo_frame_px.restype = _i32
_lib.lavish_rdo_reconstruct.argtypes = [ctypes.c_uint32, _vp, _vp, _i32, _i32, _vp, _vp, _i32,
                                        _i32, _vp, _vp]
_lib.lavish_rdo_reconstruct.restype = _i32

# C4 candidate set: 64x64 DCT, 32x32 DCT + IDTX, 16x16 / 8x8 /
# 4x4 every type
C4_TYPE_MASKS = {4: 0x0001, 3: 0x0201, 2: 0xFFFF, 1: 0xFFFF, 0: 0xFFFF}


class RdoFrame:
    """Per-size outputs of rdo_frame + the reconstruction buffers, allocated
    once for a plane shape and reused every call."""

    def __init__(self, src, type_masks=None, recon=None):
        import torch
        self.type_masks = dict(type_masks or C4_TYPE_MASKS)
        self.sizes = sorted(self.type_masks)
        self.size_mask = sum(1 << s for s in self.sizes)
        self.outs = {s: rdo_out(src, s) for s in self.sizes}
        self.tm = (ctypes.c_uint32 * 19)(*[self.type_masks.get(s, 0) for s in range(19)])
        self.rec = _P19(*[self.outs[s]["records"].data_ptr() if s in self.outs else 0
                          for s in range(19)])
        self.q = _P19(*[self.outs[s]["qcoeff"].data_ptr() if s in self.outs else 0
                        for s in range(19)])
        self.dq = _P19(*[self.outs[s]["dqcoeff"].data_ptr() if s in self.outs else 0
                         for s in range(19)])
        H, W = src.shape
        # the reconstruction keeps the planes' row stride (a view of a wider
        # buffer when src is a column segment of a frame)
        if recon is not None:  # the caller's plane (e.g. a view of a whole frame)
            assert recon.shape == src.shape and recon.stride(0) == src.stride(0) \
                and recon.stride(1) == 1 and recon.dtype == src.dtype
            self.recon = recon
        else:
            self.recon = torch.empty((H, src.stride(0)), dtype=src.dtype,
                                     device=src.device)[:, :W]
        self.sb_tx_size = torch.empty(((W + 63) // 64) * ((H + 63) // 64), dtype=torch.uint8,
                                      device=src.device)


if hasattr(_lib, "lavish_rdo_graph_create"):  # (older A/B builds lack it)
    _lib.lavish_rdo_graph_create.argtypes = [_vp, _vp, _i32, _i32, _i32, ctypes.c_uint32, _vp,
                                             _i32, ctypes.POINTER(QuantParams), _i32, _vp, _vp,
                                             _vp, _vp, _vp, _vp, ctypes.POINTER(ctypes.c_void_p)]
    _lib.lavish_rdo_graph_create.restype = _i32
    _lib.lavish_rdo_graph_launch.argtypes = [_vp, _vp]
    _lib.lavish_rdo_graph_launch.restype = _i32
    _lib.lavish_rdo_graph_destroy.argtypes = [_vp]
    _lib.lavish_rdo_graph_destroy.restype = None


class RdoGraph:
    """lavish_rdo_graph_create: the C4 step (rdo_frame + reconstruct) of one
    RdoFrame on fixed src / pred planes, captured once into a HIP graph;
    launch() replays it with one host call."""

    def __init__(self, src, pred, frame, qp, rdmult, bit_depth=10, stream=None):
        assert src.stride(1) == 1 and src.shape == pred.shape
        H, W = src.shape
        self._keep = (src, pred, frame, qp)
        g = ctypes.c_void_p()
        rc = _lib.lavish_rdo_graph_create(
            ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(pred.data_ptr()), src.stride(0), W,
            H, frame.size_mask, frame.tm, bit_depth, ctypes.byref(qp), rdmult, frame.rec, frame.q,
            frame.dq, ctypes.c_void_p(frame.recon.data_ptr()),
            ctypes.c_void_p(frame.sb_tx_size.data_ptr()), _stream_ptr(stream), ctypes.byref(g))
        if rc != 0:
            raise ValueError("lavish_rdo_graph_create failed (rc=%d)" % rc)
        self._g = g

    def launch(self, stream=None):
        rc = _lib.lavish_rdo_graph_launch(self._g, _stream_ptr(stream))
        if rc != 0:
            raise ValueError("lavish_rdo_graph_launch failed (rc=%d)" % rc)

    def __del__(self):
        g = getattr(self, "_g", None)
        if g:
            _lib.lavish_rdo_graph_destroy(g)
            self._g = None


def rdo_frame(src, pred, frame, qp, rdmult, bit_depth=10, reconstruct=True, stream=None,
              px=False):
    """C4 on one frame: lavish_rdo_frame (px=True: lavish_rdo_frame_px,
    pixel-domain distortion) over the candidate sizes, then (by default)
    lavish_rdo_reconstruct into frame.recon."""
    import torch
    assert src.dtype == torch.int16 and src.stride(1) == 1 and src.shape == pred.shape
    H, W = src.shape
    st = _stream_ptr(stream)
    fn = _lib.lavish_rdo_frame_px if px else _lib.lavish_rdo_frame
    rc = fn(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(pred.data_ptr()),
                               src.stride(0), W, H, frame.size_mask, frame.tm, bit_depth,
                               ctypes.byref(qp), rdmult, frame.rec, frame.q, frame.dq, st)
    if rc != 0:
        raise ValueError("lavish_rdo_frame rejected its arguments (rc=%d)" % rc)
    if reconstruct:
        rc = _lib.lavish_rdo_reconstruct(frame.size_mask, frame.rec, frame.dq, W, H,
                                         ctypes.c_void_p(pred.data_ptr()),
                                         ctypes.c_void_p(frame.recon.data_ptr()), src.stride(0),
                                         bit_depth, ctypes.c_void_p(frame.sb_tx_size.data_ptr()),
                                         st)
        if rc != 0:
            raise ValueError("lavish_rdo_reconstruct rejected its arguments (rc=%d)" % rc)
    return frame


def rdo_reconstruct(sizes, outs, pred, recon, sb_tx_size, bit_depth=10, stream=None):
    """lavish_rdo_reconstruct over per-size rdo_plane outputs `outs[s]`: the
    per-SB TX size into sb_tx_size and recon = pred + the chosen blocks'
    inverse transforms."""
    assert pred.stride(1) == 1 and recon.stride(0) == pred.stride(0)
    H, W = pred.shape
    rec = _P19(*[outs[s]["records"].data_ptr() if s in outs else 0 for s in range(19)])
    dq = _P19(*[outs[s]["dqcoeff"].data_ptr() if s in outs else 0 for s in range(19)])
    rc = _lib.lavish_rdo_reconstruct(sum(1 << s for s in sizes), rec, dq, W, H,
                                     ctypes.c_void_p(pred.data_ptr()),
                                     ctypes.c_void_p(recon.data_ptr()), pred.stride(0), bit_depth,
                                     ctypes.c_void_p(sb_tx_size.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_rdo_reconstruct rejected its arguments (rc=%d)" % rc)


# ----------------------------------------------------- TX-pruning features --
_lib.lavish_horver_correlation_batch.argtypes = [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp]
_lib.lavish_horver_correlation_batch.restype = _i32
_lib.lavish_tx_prune_features_batch.argtypes = [_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp]
_lib.lavish_tx_prune_features_batch.restype = _i32
_lib.av1_get_horver_correlation_full_hip.argtypes = [_vp, _i32, _i32, _i32, _vp, _vp]
_lib.av1_get_horver_correlation_full_hip.restype = None


def horver_correlation_batch(residual, bw, bh, stream=None):
    """lavish_horver_correlation_batch: (hcorr, vcorr) float32 device tensors
    over the full bw x bh blocks of a device int16 residual plane."""
    import torch
    assert residual.dtype == torch.int16 and residual.stride(1) == 1
    H, W = residual.shape
    nb = (W // bw) * (H // bh)
    hc = torch.empty(nb, dtype=torch.float32, device=residual.device)
    vc = torch.empty(nb, dtype=torch.float32, device=residual.device)
    rc = _lib.lavish_horver_correlation_batch(ctypes.c_void_p(residual.data_ptr()),
                                              residual.stride(0), W, H, bw, bh,
                                              ctypes.c_void_p(hc.data_ptr()),
                                              ctypes.c_void_p(vc.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_horver_correlation_batch rejected its arguments (rc=%d)" % rc)
    return hc, vc


def tx_prune_features(residual, tx_size, stream=None):
    """lavish_tx_prune_features_batch: (hfeatures, vfeatures) [block, 16]
    float32 device tensors, prune_tx_2D's neural-net inputs."""
    import torch
    assert residual.dtype == torch.int16 and residual.stride(1) == 1
    H, W = residual.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    hf = torch.empty((nb, 16), dtype=torch.float32, device=residual.device)
    vf = torch.empty((nb, 16), dtype=torch.float32, device=residual.device)
    rc = _lib.lavish_tx_prune_features_batch(ctypes.c_void_p(residual.data_ptr()),
                                             residual.stride(0), W, H, tx_size,
                                             ctypes.c_void_p(hf.data_ptr()),
                                             ctypes.c_void_p(vf.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_tx_prune_features_batch rejected its arguments (rc=%d)" % rc)
    return hf, vf


def av1_get_horver_correlation_full(diff, stride, w, h):
    """Per-call RTCD shim (host int16 buffer): returns (hcorr, vcorr)."""
    hc, vc = ctypes.c_float(), ctypes.c_float()
    _lib.av1_get_horver_correlation_full_hip(_p(diff), stride, w, h, ctypes.byref(hc),
                                             ctypes.byref(vc))
    return hc.value, vc.value
