"""TX-type pruning on the MI355X backend: prune_tx_2D
(av1/encoder/tx_search.c:1487-1641) for whole residual planes
(lavish_prune_tx_2d_batch), av1_nn_predict_c batches (lavish_nn_predict_batch)
and the av1_nn_predict RTCD shim.  Models are NN_CONFIG records
(av1/encoder/ml.h:24-34) -- in an encoder, the reference's own
av1_tx_type_nnconfig_map_hor / _ver entries."""
import ctypes

import numpy as np

from . import _lib, _stream_ptr

EXT_TX_SET_DTT9_IDTX_1DDCT, EXT_TX_SET_ALL16 = 4, 5   # aom_dsp/txfm_common.h:72-86
TX_TYPE_INVALID = 255

_vp, _i32 = ctypes.c_void_p, ctypes.c_int32


class NNConfig(ctypes.Structure):
    """Layout of NN_CONFIG."""
    _fields_ = [("num_inputs", ctypes.c_int), ("num_outputs", ctypes.c_int),
                ("num_hidden_layers", ctypes.c_int), ("num_hidden_nodes", ctypes.c_int * 10),
                ("weights", ctypes.c_void_p * 11), ("bias", ctypes.c_void_p * 11)]


_lib.lavish_prune_tx_2d_batch.argtypes = [_vp, _i32, _i32, _i32, _i32, _i32, _i32,
                                          ctypes.POINTER(NNConfig), ctypes.POINTER(NNConfig),
                                          _vp, ctypes.c_uint16, _vp, _vp, _vp]
_lib.lavish_prune_tx_2d_batch.restype = _i32
_lib.lavish_nn_predict_batch.argtypes = [_vp, ctypes.POINTER(NNConfig), _i32, _vp, _i32, _vp]
_lib.lavish_nn_predict_batch.restype = _i32
_lib.av1_nn_predict_hip.argtypes = [_vp, ctypes.POINTER(NNConfig), _i32, _vp]
_lib.av1_nn_predict_hip.restype = None


def nn_config(num_inputs, num_outputs, hidden, weights, bias):
    """An NNConfig over host float32 arrays (kept alive on the object)."""
    c = NNConfig()
    c.num_inputs, c.num_outputs, c.num_hidden_layers = num_inputs, num_outputs, len(hidden)
    for i, h in enumerate(hidden):
        c.num_hidden_nodes[i] = h
    keep = []
    for i, (w, b) in enumerate(zip(weights, bias)):
        wa = np.ascontiguousarray(w, np.float32)
        ba = np.ascontiguousarray(b, np.float32)
        keep += [wa, ba]
        c.weights[i], c.bias[i] = wa.ctypes.data, ba.ctypes.data
    c._keep = keep
    return c


def prune_tx_2d(residual, tx_size, tx_set_type, prune_mode, nn_hor, nn_ver, allowed_in=None,
                allowed_default=0xFFFF, stream=None):
    """lavish_prune_tx_2d_batch over a device int16 residual plane; returns
    (allowed_out uint16-as-int16 [block], txk_map uint8 [block, 16])."""
    import torch
    from . import TX_W, TX_H
    assert residual.dtype == torch.int16 and residual.stride(1) == 1
    H, W = residual.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    out = torch.empty(nb, dtype=torch.int16, device=residual.device)
    maps = torch.empty((nb, 16), dtype=torch.uint8, device=residual.device)
    rc = _lib.lavish_prune_tx_2d_batch(
        _vp(residual.data_ptr()), residual.stride(0), W, H, tx_size, tx_set_type, prune_mode,
        None if nn_hor is None else ctypes.byref(nn_hor),
        None if nn_ver is None else ctypes.byref(nn_ver),
        None if allowed_in is None else _vp(allowed_in.data_ptr()), allowed_default,
        _vp(out.data_ptr()), _vp(maps.data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_prune_tx_2d_batch rejected its arguments (rc=%d)" % rc)
    return out, maps


def nn_predict_batch(inputs, cfg, reduce_prec=True, stream=None):
    """lavish_nn_predict_batch over a device float32 [n, num_inputs] tensor."""
    import torch
    assert inputs.dtype == torch.float32 and inputs.is_contiguous()
    n = inputs.shape[0]
    out = torch.empty((n, cfg.num_outputs), dtype=torch.float32, device=inputs.device)
    rc = _lib.lavish_nn_predict_batch(_vp(inputs.data_ptr()), ctypes.byref(cfg),
                                      int(reduce_prec), _vp(out.data_ptr()), n,
                                      _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_nn_predict_batch rejected its arguments (rc=%d)" % rc)
    return out


def av1_nn_predict(inputs, cfg, reduce_prec=True):
    """Per-call RTCD shim on a host float32 vector."""
    x = np.ascontiguousarray(inputs, np.float32)
    out = np.zeros(cfg.num_outputs, np.float32)
    _lib.av1_nn_predict_hip(_vp(x.ctypes.data), ctypes.byref(cfg), int(reduce_prec),
                            _vp(out.ctypes.data))
    return out
