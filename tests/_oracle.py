"""ctypes binding of the test-only CPU oracle (oracle/liboracle.so).

Test infrastructure: imported only by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product never imports this module."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def P(a):
    # callers pass explicit row strides: the rows must be contiguous in memory
    assert a.ndim == 0 or a.strides[-1] == a.itemsize, "row-contiguous array expected"
    return a.ctypes.data_as(ctypes.c_void_p)


class OrcQuant(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int16 * 2) for n in
                ("quant", "quant_shift", "zbin", "round", "quant_fp", "round_fp", "dequant")]


def _declare(L):
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    L.orc_fwd_txfm1d.argtypes = [i32, i32, vp, vp, i32]
    L.orc_inv_txfm1d.argtypes = [i32, i32, vp, vp, i32, vp]
    L.orc_fwd_txfm2d.argtypes = [vp, vp, i32, i32, i32, i32]
    L.orc_inv_txfm2d_add.argtypes = [vp, vp, i32, i32, i32, i32]
    L.orc_fwht4x4.argtypes = [vp, vp, i32]
    L.orc_scan.restype = ctypes.POINTER(ctypes.c_int16)
    L.orc_iscan.restype = ctypes.POINTER(ctypes.c_int16)
    L.orc_cospi.restype = ctypes.c_int32
    L.orc_sinpi.restype = ctypes.c_int32
    L.orc_dc_quant.restype = ctypes.c_int16
    L.orc_ac_quant.restype = ctypes.c_int16
    L.orc_build_quant.argtypes = [i32, i32, i32, i32, ctypes.POINTER(OrcQuant)]
    qargs = [vp, ctypes.c_ssize_t, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32]
    for n in ("orc_quantize_fp", "orc_quantize_b", "orc_highbd_quantize_fp",
              "orc_highbd_quantize_b"):
        getattr(L, n).argtypes = qargs
    L.orc_txq_plane.argtypes = [vp, i32, i32, i32, i32, ctypes.c_uint, i32,
                                ctypes.POINTER(OrcQuant), i32, vp, vp, vp, i32]
    L.orc_txq_plane.restype = ctypes.c_long
    L.orc_sad.restype = ctypes.c_uint
    L.orc_sad.argtypes = [vp, i32, vp, i32, i32, i32]
    L.orc_sad_skip.restype = ctypes.c_uint
    L.orc_sad_skip.argtypes = [vp, i32, vp, i32, i32, i32]
    L.orc_sad_avg.restype = ctypes.c_uint
    L.orc_sad_avg.argtypes = [vp, i32, vp, i32, i32, i32, vp]
    L.orc_highbd_sad.restype = ctypes.c_uint
    L.orc_highbd_sad.argtypes = [vp, i32, vp, i32, i32, i32]
    L.orc_variance.restype = ctypes.c_uint
    L.orc_variance.argtypes = [vp, i32, vp, i32, i32, i32, vp]
    L.orc_mse.restype = ctypes.c_uint
    L.orc_mse.argtypes = [vp, i32, vp, i32, i32, i32, vp]
    L.orc_highbd_variance.restype = ctypes.c_uint
    L.orc_highbd_variance.argtypes = [vp, i32, vp, i32, i32, i32, i32, vp]
    L.orc_sub_pixel_variance.restype = ctypes.c_uint
    L.orc_sub_pixel_variance.argtypes = [vp, i32, i32, i32, vp, i32, i32, i32, vp]
    L.orc_sub_pixel_avg_variance.restype = ctypes.c_uint
    L.orc_sub_pixel_avg_variance.argtypes = [vp, i32, i32, i32, vp, i32, i32, i32, vp, vp]
    L.orc_highbd_sub_pixel_variance.restype = ctypes.c_uint
    L.orc_highbd_sub_pixel_variance.argtypes = [vp, i32, i32, i32, vp, i32, i32, i32, i32,
                                                vp, vp]
    L.orc_highbd_sad_avg.restype = ctypes.c_uint
    L.orc_highbd_sad_avg.argtypes = [vp, i32, vp, i32, i32, i32, vp]
    L.orc_highbd_hadamard.argtypes = [i32, vp, ctypes.c_ssize_t, vp]
    L.orc_sse.restype = i64
    L.orc_sse.argtypes = [vp, i32, vp, i32, i32, i32]
    L.orc_highbd_sse.restype = i64
    L.orc_highbd_sse.argtypes = [vp, i32, vp, i32, i32, i32]
    L.orc_subtract_block.argtypes = [i32, i32, vp, ctypes.c_ssize_t, vp,
                                     ctypes.c_ssize_t, vp, ctypes.c_ssize_t]
    L.orc_highbd_subtract_block.argtypes = L.orc_subtract_block.argtypes
    L.orc_sum_squares_2d_i16.restype = ctypes.c_uint64
    L.orc_sum_squares_2d_i16.argtypes = [vp, i32, i32, i32]
    L.orc_hadamard.argtypes = [i32, vp, ctypes.c_ssize_t, vp]
    L.orc_satd.argtypes = [vp, i32]
    L.orc_hadamard_lp.argtypes = [i32, vp, ctypes.c_ssize_t, vp]
    L.orc_satd_lp.argtypes = [vp, i32]
    L.orc_block_error_lp.argtypes = [vp, vp, ctypes.c_ssize_t]
    L.orc_block_error_lp.restype = i64
    L.orc_sum_sse.argtypes = [vp, i32, i32, i32, vp, vp]
    L.orc_iwht4x4_add.argtypes = [vp, vp, i32, i32, i32]
    L.orc_block_error.restype = i64
    L.orc_block_error.argtypes = [vp, vp, ctypes.c_ssize_t, vp]
    L.orc_highbd_block_error.restype = i64
    L.orc_highbd_block_error.argtypes = [vp, vp, ctypes.c_ssize_t, vp, i32]


TX_W = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
TX_H = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]
TX_NAMES = ["4x4", "8x8", "16x16", "32x32", "64x64", "4x8", "8x4", "8x16",
            "16x8", "16x32", "32x16", "32x64", "64x32", "4x16", "16x4",
            "8x32", "32x8", "16x64", "64x16"]


def max_eob(s):
    if s in (17, 18):
        return 512
    if TX_W[s] == 64 or TX_H[s] == 64:
        return 1024
    return TX_W[s] * TX_H[s]


def tx_scale(s):
    p = TX_W[s] * TX_H[s]
    return int(p > 256) + int(p > 1024)


def type_valid(s, t):
    m = max(TX_W[s], TX_H[s])
    if m == 64:
        return t == 0
    if m == 32:
        return t in (0, 9)
    return 0 <= t < 16


def fwd_txfm1d(kind, x, cos_bit):
    x = np.ascontiguousarray(x, dtype=np.int32)
    y = np.zeros_like(x)
    lib().orc_fwd_txfm1d(kind, len(x), P(x), P(y), cos_bit)
    return y


def inv_txfm1d(kind, x, cos_bit, stage_range):
    x = np.ascontiguousarray(x, dtype=np.int32)
    y = np.zeros_like(x)
    sr = np.ascontiguousarray(stage_range, dtype=np.int8)
    lib().orc_inv_txfm1d(kind, len(x), P(x), P(y), cos_bit, P(sr))
    return y


def fwd_txfm2d(block, tx_type, tx_size, bd=8):
    """block: int16 [H, stride>=W] array; returns int32 coefficient buffer of
    W*H words (the reference's output buffer, column-major)."""
    block = np.ascontiguousarray(block, dtype=np.int16)
    out = np.zeros(TX_W[tx_size] * TX_H[tx_size], dtype=np.int32)
    lib().orc_fwd_txfm2d(P(block), P(out), block.shape[1], tx_type, tx_size, bd)
    return out


def inv_txfm2d_add(coeff, dst, tx_type, tx_size, bd):
    coeff = np.ascontiguousarray(coeff, dtype=np.int32)
    dst = np.ascontiguousarray(dst, dtype=np.uint16).copy()
    lib().orc_inv_txfm2d_add(P(coeff), P(dst), dst.shape[1], tx_type, tx_size, bd)
    return dst


def scan(tx_size, tx_type):
    W, H = min(TX_W[tx_size], 32), min(TX_H[tx_size], 32)
    p = lib().orc_scan(tx_size, tx_type)
    return np.ctypeslib.as_array(p, shape=(W * H,)).copy()


def iscan(tx_size, tx_type):
    W, H = min(TX_W[tx_size], 32), min(TX_H[tx_size], 32)
    p = lib().orc_iscan(tx_size, tx_type)
    return np.ctypeslib.as_array(p, shape=(W * H,)).copy()


def build_quant(bd, qindex, sharpness=0, y_dc_delta_q=0):
    q = OrcQuant()
    lib().orc_build_quant(bd, qindex, sharpness, y_dc_delta_q, ctypes.byref(q))
    return q


def quant_arrays(q):
    return {n: np.array(list(getattr(q, n)), dtype=np.int16) for n, _ in OrcQuant._fields_}


def quantize(kind, coeff, n, q, scan_, iscan_, log_scale, highbd=False):
    """kind 'fp' or 'b' with the reference's argument wiring
    (av1_quantize_fp_facade / av1_quantize_b_facade)."""
    qa = quant_arrays(q)
    coeff = np.ascontiguousarray(coeff, dtype=np.int32)
    qc = np.zeros(n, np.int32)
    dq = np.zeros(n, np.int32)
    eob = np.zeros(1, np.uint16)
    if kind == "fp":
        rnd, qt = qa["round_fp"], qa["quant_fp"]
        fn = lib().orc_highbd_quantize_fp if highbd else lib().orc_quantize_fp
    else:
        rnd, qt = qa["round"], qa["quant"]
        fn = lib().orc_highbd_quantize_b if highbd else lib().orc_quantize_b
    sc = np.ascontiguousarray(scan_, np.int16)
    isc = np.ascontiguousarray(iscan_, np.int16)
    fn(P(coeff), n, P(qa["zbin"]), P(rnd), P(qt), P(qa["quant_shift"]), P(qc),
       P(dq), P(qa["dequant"]), P(eob), P(sc), P(isc), log_scale)
    return qc, dq, int(eob[0])


def txq_plane(residual, tx_size, type_mask, q, bd=8, quant_b=False, threads=1):
    residual = np.ascontiguousarray(residual, dtype=np.int16)
    H, W = residual.shape
    bw, bh = W // TX_W[tx_size], H // TX_H[tx_size]
    nt = bin(type_mask).count("1")
    n = max_eob(tx_size)
    qc = np.zeros((bh * bw, nt, n), np.int32)
    dq = np.zeros((bh * bw, nt, n), np.int32)
    eob = np.zeros((bh * bw, nt), np.uint16)
    lib().orc_txq_plane(P(residual), W, W, H, tx_size, type_mask, bd,
                        ctypes.byref(q), int(quant_b), P(qc), P(dq), P(eob), threads)
    return qc, dq, eob


class ACMRandom:
    """test/acm_random.h over gtest's LCG (gtest.cc:378-381)."""

    def __init__(self, seed=0xBABA):
        self.state = seed

    def _gen(self, rng):
        self.state = (1103515245 * self.state + 12345) % (1 << 31)
        return self.state % rng

    def rand31(self):
        return self._gen(1 << 31)

    def rand16(self):
        return (self._gen(1 << 31) >> 15) & 0xFFFF

    def rand8(self):
        return (self._gen(1 << 31) >> 23) & 0xFF

    def rand12(self):
        return (self._gen(1 << 31) >> 19) & 0xFFF

    def pseudo_uniform(self, r):
        return self._gen(r)

    def rand9signed(self):
        return self._gen(512) - 256

    def rand15signed(self):
        return ((self._gen(1 << 31) >> 16) & 0x7FFF) - (1 << 14)

    def rand8extremes(self):
        r = self.rand8()
        return (r << 4) & 0xFF if r < 128 else r >> 4


# ---------------------------------------------------------- pixel kernels --
def sad(a, a_stride, b, b_stride, w, h, highbd=False, skip=False, second_pred=None):
    L = lib()
    if second_pred is not None:
        f = L.orc_highbd_sad_avg if highbd else L.orc_sad_avg
        return f(P(a), a_stride, P(b), b_stride, w, h, P(second_pred))
    if highbd:
        if skip:
            return 2 * L.orc_highbd_sad(P(a), 2 * a_stride, P(b), 2 * b_stride, w, h // 2)
        return L.orc_highbd_sad(P(a), a_stride, P(b), b_stride, w, h)
    f = L.orc_sad_skip if skip else L.orc_sad
    return f(P(a), a_stride, P(b), b_stride, w, h)


def variance(a, a_stride, b, b_stride, w, h, bd=8, highbd=False):
    L = lib()
    sse = ctypes.c_uint(0)
    if highbd:
        v = L.orc_highbd_variance(P(a), a_stride, P(b), b_stride, w, h, bd, ctypes.byref(sse))
    else:
        v = L.orc_variance(P(a), a_stride, P(b), b_stride, w, h, ctypes.byref(sse))
    return v, sse.value


def mse(a, a_stride, b, b_stride, w, h, bd=8, highbd=False):
    if highbd:
        v, s = variance(a, a_stride, b, b_stride, w, h, bd, True)
        return s, s
    sse = ctypes.c_uint(0)
    v = lib().orc_mse(P(a), a_stride, P(b), b_stride, w, h, ctypes.byref(sse))
    return v, sse.value


def get_var(a, a_stride, b, b_stride, w, h, bd=8, highbd=False):
    """(sse, sum) as aom[_highbd_bd]_get{n}x{n}var (variance.c:187-238)."""
    if highbd:
        # sum = the rounded sum of highbd_{bd}_variance: recover it from var/sse
        a64 = a[:h, :w].astype(np.int64)
        b64 = b[:h, :w].astype(np.int64)
        d = a64 - b64
        tsum = int(d.sum())
        _, sse = variance(a, a_stride, b, b_stride, w, h, bd, True)
        if bd == 8:
            return sse, tsum
        sh = 2 if bd == 10 else 4
        return sse, (tsum + ((1 << sh) >> 1)) >> sh
    _, sse = variance(a, a_stride, b, b_stride, w, h)
    d = a[:h, :w].astype(np.int64) - b[:h, :w].astype(np.int64)
    return sse, int(d.sum())


def sub_pixel_variance(a, a_stride, xo, yo, b, b_stride, w, h, bd=8, highbd=False,
                       second_pred=None):
    L = lib()
    sse = ctypes.c_uint(0)
    if highbd:
        v = L.orc_highbd_sub_pixel_variance(P(a), a_stride, xo, yo, P(b), b_stride, w, h, bd,
                                            ctypes.byref(sse),
                                            P(second_pred) if second_pred is not None else None)
    elif second_pred is not None:
        v = L.orc_sub_pixel_avg_variance(P(a), a_stride, xo, yo, P(b), b_stride, w, h,
                                         ctypes.byref(sse), P(second_pred))
    else:
        v = L.orc_sub_pixel_variance(P(a), a_stride, xo, yo, P(b), b_stride, w, h,
                                     ctypes.byref(sse))
    return v, sse.value


def sse(a, a_stride, b, b_stride, w, h, highbd=False):
    f = lib().orc_highbd_sse if highbd else lib().orc_sse
    return f(P(a), a_stride, P(b), b_stride, w, h)


def subtract_block(rows, cols, diff, ds, src, ss, pred, ps, highbd=False):
    f = lib().orc_highbd_subtract_block if highbd else lib().orc_subtract_block
    f(rows, cols, P(diff), ds, P(src), ss, P(pred), ps)


def sum_squares_2d_i16(src, stride, w, h):
    return lib().orc_sum_squares_2d_i16(P(src), stride, w, h)


def hadamard(n, src, stride, highbd=False):
    out = np.zeros(n * n, np.int32)
    f = lib().orc_highbd_hadamard if highbd else lib().orc_hadamard
    f(n, P(src), stride, P(out))
    return out


def satd(coeff, length):
    return lib().orc_satd(P(coeff), length)


def hadamard_lp(n, src, stride):
    out = np.zeros(n * n, np.int16)
    lib().orc_hadamard_lp(n, P(np.ascontiguousarray(src, np.int16)), stride, P(out))
    return out


def satd_lp(coeff, length):
    return lib().orc_satd_lp(P(np.ascontiguousarray(coeff, np.int16)), length)


def block_error_lp(coeff, dqcoeff, n):
    return lib().orc_block_error_lp(P(np.ascontiguousarray(coeff, np.int16)),
                                    P(np.ascontiguousarray(dqcoeff, np.int16)), n)


def sum_sse(src, stride, w, h):
    """(sum, sse) of an int16 block (aom_sum_sse_2d_i16 / aom_get_blk_sse_sum)."""
    sm, ss = ctypes.c_int(0), ctypes.c_int64(0)
    lib().orc_sum_sse(P(np.ascontiguousarray(src, np.int16)), stride, w, h, ctypes.byref(sm),
                      ctypes.byref(ss))
    return sm.value, ss.value


def fwht4x4(block, stride):
    out = np.zeros(16, np.int32)
    lib().orc_fwht4x4(P(np.ascontiguousarray(block, np.int16)), P(out), stride)
    return out


def iwht4x4_add(coeff, dst, eob, bd):
    dst = np.ascontiguousarray(dst, np.uint16).copy()
    lib().orc_iwht4x4_add(P(np.ascontiguousarray(coeff, np.int32)), P(dst), dst.shape[1], eob, bd)
    return dst


def block_error(coeff, dqcoeff, n, bd=None):
    ssz = ctypes.c_int64(0)
    if bd is None:
        e = lib().orc_block_error(P(coeff), P(dqcoeff), n, ctypes.byref(ssz))
    else:
        e = lib().orc_highbd_block_error(P(coeff), P(dqcoeff), n, ctypes.byref(ssz), bd)
    return e, ssz.value


# ------------------------------------------------------ C3 diamond search --
def diamond_batch(src, ref, stride, w, h, jobs, step_param=0, mv_cost_type=3, skip=False,
                  threads=1, method="diamond"):
    """orc_diamond_batch (method "bigdia": orc_bigdia_batch, FAST_BIGDIA) over
    JOB_DTYPE records (lavish_dsp.motion); src and ref are the flat padded
    planes (ref holds all reference planes)."""
    L = lib()
    fn = L.orc_bigdia_batch if method == "bigdia" else L.orc_diamond_batch
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_int]
    jobs = np.ascontiguousarray(jobs)
    out = np.zeros(len(jobs), np.dtype([("best_row", "<i2"), ("best_col", "<i2"),
                                        ("bestsme", "<i4"), ("steps", "<i4"),
                                        ("searches", "<i4")], align=True))
    fn(P(src), stride, P(ref), stride, w, h, P(jobs), len(jobs), step_param, mv_cost_type,
       int(skip), P(out), threads)
    return out


class OrcMvCost(ctypes.Structure):
    _fields_ = [("mv_cost_type", ctypes.c_int), ("sad_per_bit", ctypes.c_int),
                ("error_per_bit", ctypes.c_int), ("mvjcost", ctypes.c_void_p),
                ("mvcost", ctypes.c_void_p * 2)]


FP_METHODS = {"diamond": 0, "nstep": 1, "nstep_8pt": 2, "hex": 4, "bigdia": 5, "square": 6,
              "fast_hex": 7, "fast_diamond": 8, "fast_bigdia": 9, "vfast_diamond": 10}


class OrcMeshParams(ctypes.Structure):
    """The mesh fields of FULLPEL_MOTION_SEARCH_PARAMS (mcomp.h:114-123) with
    the pattern set mesh_patterns[is_intra_mode]; the field order of
    MESH_FIELDS in tests/golden/gen_fixtures.py is (6 scalars, then range /
    interval pairs)."""
    _fields_ = [("run_mesh_search", ctypes.c_int), ("force_mesh_thresh", ctypes.c_int),
                ("prune_mesh_search", ctypes.c_int),
                ("mesh_search_mv_diff_threshold", ctypes.c_int),
                ("fine_search_interval", ctypes.c_int), ("is_intra_mode", ctypes.c_int),
                ("range", ctypes.c_int * 4), ("interval", ctypes.c_int * 4)]

    @classmethod
    def from_row(cls, row):
        """From a fix_mcomp3 "mesh" row (MESH_FIELDS order)."""
        r = [int(v) for v in row]
        m = cls(*r[:6])
        for i in range(4):
            m.range[i], m.interval[i] = r[6 + 2 * i], r[7 + 2 * i]
        return m


def full_pixel_search_batch(src, ref, stride, w, h, jobs, method="diamond", step_param=0,
                            mv_cost_type=3, sad_per_bit=0, error_per_bit=0, mvjcost=None,
                            mvcost=None, skip=False, cost_list=False, threads=1, mesh=None):
    """orc_full_pixel_search_batch_ex: av1_full_pixel_search with any method
    and any mv cost, and the mesh refinement when `mesh` (OrcMeshParams) is
    given.  mvjcost int32[4], mvcost int32[2][MV_VALS] (centred at MV_MAX) for
    MV_COST_ENTROPY.  Returns (results, cost_lists int32[n][5] or None)."""
    L = lib()
    fn = L.orc_full_pixel_search_batch_ex
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(OrcMvCost), ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_int, ctypes.POINTER(OrcMeshParams)]
    jobs = np.ascontiguousarray(jobs)
    keep = []
    c = OrcMvCost(mv_cost_type, sad_per_bit, error_per_bit)
    if mvjcost is not None:
        mj = np.ascontiguousarray(mvjcost, np.int32)
        mc = np.ascontiguousarray(mvcost, np.int32)
        keep += [mj, mc]
        mid = (mc.shape[1] - 1) // 2
        c.mvjcost = mj.ctypes.data
        c.mvcost[0] = mc.ctypes.data + 4 * mid
        c.mvcost[1] = mc.ctypes.data + 4 * (mc.shape[1] + mid)
    out = np.zeros(len(jobs), np.dtype([("best_row", "<i2"), ("best_col", "<i2"),
                                        ("bestsme", "<i4"), ("steps", "<i4"),
                                        ("searches", "<i4")], align=True))
    cls = np.full((len(jobs), 5), 0x7FFFFFFF, np.int32) if cost_list else None
    fn(P(src), stride, P(ref), stride, w, h, P(jobs), len(jobs), FP_METHODS[method], step_param,
       ctypes.byref(c), int(skip), P(cls) if cost_list else None, P(out), threads,
       ctypes.byref(mesh) if mesh is not None else None)
    return out, cls


def tpl_motion_search(src, ref, stride, jobs, cols, rows, nrefs, method="fast_bigdia",
                      step_param=6, skip=False, prune_starting_mv=3, skip_alike_starting_mv=2,
                      sad_per_bit=0, error_per_bit=0, mvjcost=None, mvcost=None, mv_cost_type=0,
                      third=None, cost_list=True):
    """orc_tpl_motion_search: mode_estimation's per-reference motion search with
    the neighbour start mvs (16x16, FULL_PEL).  Returns (mvs int32 int_mv,
    results, cost lists or None, centers int32 int_mv)."""
    L = lib()
    fn = L.orc_tpl_motion_search
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(OrcMvCost),
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_void_p]
    jobs = np.ascontiguousarray(jobs)
    assert len(jobs) == nrefs * rows * cols
    keep = []
    c = OrcMvCost(mv_cost_type, sad_per_bit, error_per_bit)
    if mvjcost is not None:
        mj = np.ascontiguousarray(mvjcost, np.int32)
        mc = np.ascontiguousarray(mvcost, np.int32)
        keep += [mj, mc]
        mid = (mc.shape[1] - 1) // 2
        c.mvjcost = mj.ctypes.data
        c.mvcost[0] = mc.ctypes.data + 4 * mid
        c.mvcost[1] = mc.ctypes.data + 4 * (mc.shape[1] + mid)
    n = len(jobs)
    out = np.zeros(n, np.dtype([("best_row", "<i2"), ("best_col", "<i2"), ("bestsme", "<i4"),
                                ("steps", "<i4"), ("searches", "<i4")], align=True))
    cls = np.full((n, 5), 0x7FFFFFFF, np.int32) if cost_list else None
    mvs = np.zeros(n, np.int32)
    centers = np.zeros(n, np.int32)
    if third is not None:
        third = np.ascontiguousarray(third, np.int32)
    fn(P(src), stride, P(ref), stride, P(jobs), cols, rows, nrefs, FP_METHODS[method], step_param,
       int(skip), prune_starting_mv, skip_alike_starting_mv, ctypes.byref(c),
       P(third) if third is not None else None, P(mvs), P(out), P(cls) if cost_list else None,
       P(centers))
    return mvs, out, cls, centers


def subpel_search_batch(src, ref, stride, w, h, jobs, method=2, forced_stop=0, allow_hp=False,
                        iters=1, mv_cost_type=3, error_per_bit=0, mvjcost=None, mvcost=None,
                        cost_lists=None, threads=1, search_type=0):
    """orc_subpel_search_batch_ex: SUBPEL_TREE (method 0; bilinear error with
    search_type 0 USE_2_TAPS_ORIG, else the upsampled prediction of
    USE_2_TAPS / USE_4_TAPS / USE_8_TAPS), SUBPEL_TREE_PRUNED (1) /
    _PRUNED_MORE (2) with any mv cost and optional full-pel cost lists."""
    L = lib()
    fn = L.orc_subpel_search_batch_ex
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(OrcMvCost),
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    jobs = np.ascontiguousarray(jobs)
    c = OrcMvCost(mv_cost_type, 0, error_per_bit)
    keep = []
    if mvjcost is not None:
        mj = np.ascontiguousarray(mvjcost, np.int32)
        mc = np.ascontiguousarray(mvcost, np.int32)
        keep += [mj, mc]
        mid = (mc.shape[1] - 1) // 2
        c.mvjcost = mj.ctypes.data
        c.mvcost[0] = mc.ctypes.data + 4 * mid
        c.mvcost[1] = mc.ctypes.data + 4 * (mc.shape[1] + mid)
    out = np.zeros(len(jobs), SUBPEL_RESULT)
    cl = None if cost_lists is None else np.ascontiguousarray(cost_lists, np.int32)
    fn(P(src), stride, P(ref), stride, w, h, P(jobs), len(jobs), method, search_type,
       forced_stop, int(allow_hp), iters, ctypes.byref(c), None if cl is None else P(cl), P(out),
       threads)
    return out


SUBPEL_RESULT = np.dtype([("best_row", "<i2"), ("best_col", "<i2"), ("besterr", "<u4"),
                          ("distortion", "<i4"), ("sse", "<u4")], align=True)


def subpel_batch(src, ref, stride, w, h, jobs, forced_stop=0, allow_hp=False, iters=1,
                 mv_cost_type=3, threads=1):
    """orc_subpel_batch over SUBPEL_JOB_DTYPE records (lavish_dsp.motion)."""
    L = lib()
    L.orc_subpel_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_int]
    jobs = np.ascontiguousarray(jobs)
    out = np.zeros(len(jobs), SUBPEL_RESULT)
    L.orc_subpel_batch(P(src), stride, P(ref), stride, w, h, P(jobs), len(jobs), forced_stop,
                       int(allow_hp), iters, mv_cost_type, P(out), threads)
    return out


# ------------------------------------------------------------- C4 RDO --
RDO_DTYPE = np.dtype([("best_type", "<i4"), ("eob", "<i4"), ("rate", "<i4"), ("satd", "<i4"),
                      ("dist", "<i8"), ("sse", "<i8"), ("rdcost", "<i8")], align=True)


def rdo_plane(src, pred, tx_size, type_mask, bd, q, rdmult, threads=1, px=False):
    """orc_rdo_plane (px: orc_rdo_plane_px, pixel-domain distortion) over u16
    planes of equal shape; returns (records, qcoeff[block, n], dqcoeff[block, n])."""
    L = lib()
    fn = L.orc_rdo_plane_px if px else L.orc_rdo_plane
    fn.restype = ctypes.c_long
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(OrcQuant),
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    src = np.ascontiguousarray(src, dtype=np.uint16)
    pred = np.ascontiguousarray(pred, dtype=np.uint16)
    H, W = src.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    n = max_eob(tx_size)
    out = np.zeros(nb, RDO_DTYPE)
    qc = np.zeros((nb, n), np.int32)
    dq = np.zeros((nb, n), np.int32)
    if nb == 0:  # the plane is narrower / lower than one block of this size
        return out, qc, dq
    fn(P(src), P(pred), W, W, H, tx_size, type_mask, bd, ctypes.byref(q), rdmult, P(out), P(qc),
       P(dq), threads)
    return out, qc, dq


def rdo_plane_masked(src, pred, tx_size, type_mask, bd, q, rdmult, block_mask=None,
                     block_map=None, px=False, threads=1):
    """orc_rdo_plane_masked: search_tx_type's txk_map / allowed_tx_mask loop."""
    L = lib()
    fn = L.orc_rdo_plane_masked
    fn.restype = ctypes.c_long
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(OrcQuant),
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    src = np.ascontiguousarray(src, dtype=np.uint16)
    pred = np.ascontiguousarray(pred, dtype=np.uint16)
    H, W = src.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    n = max_eob(tx_size)
    out = np.zeros(nb, RDO_DTYPE)
    qc = np.zeros((nb, n), np.int32)
    dq = np.zeros((nb, n), np.int32)
    bm = None if block_mask is None else np.ascontiguousarray(block_mask, np.uint16)
    mp = None if block_map is None else np.ascontiguousarray(block_map, np.uint8)
    fn(P(src), P(pred), W, W, H, tx_size, type_mask, bd, ctypes.byref(q), rdmult,
       None if bm is None else P(bm), None if mp is None else P(mp), int(px), P(out), P(qc),
       P(dq), threads)
    return out, qc, dq


def rdo_reconstruct(sizes, recs, dqs, pred, bd):
    """orc_rdo_reconstruct: per-SB TX size (lowest saturating sum of block
    costs, ties to the larger size) and recon = pred + the chosen blocks'
    inverse transforms.  recs / dqs are per entry of `sizes`.  Returns
    (recon, sb_tx_size)."""
    L = lib()
    vp = ctypes.c_void_p
    L.orc_rdo_reconstruct.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp,
                                      vp, ctypes.c_int, ctypes.c_int, vp]
    order = sorted(range(len(sizes)), key=lambda i: -TX_W[sizes[i]] * TX_H[sizes[i]])
    sz = np.array([sizes[i] for i in order], np.int32)
    recs = [np.ascontiguousarray(recs[i]) for i in order]
    dqs = [np.ascontiguousarray(dqs[i], np.int32) for i in order]
    rp = (vp * len(sz))(*[r.ctypes.data for r in recs])
    dp = (vp * len(sz))(*[d.ctypes.data for d in dqs])
    pred = np.ascontiguousarray(pred, dtype=np.uint16)
    H, W = pred.shape
    recon = np.empty_like(pred)
    choice = np.zeros(((W + 63) // 64) * ((H + 63) // 64), np.uint8)
    L.orc_rdo_reconstruct(len(sz), P(sz), ctypes.cast(rp, vp), ctypes.cast(dp, vp), W, H, P(pred),
                          P(recon), W, bd, P(choice))
    return recon, choice


# ---------------------------------------------------- TX-pruning features --
def horver_full(diff, stride, w, h):
    """orc_horver_correlation_full on a host int16 buffer: (hcorr, vcorr)."""
    L = lib()
    L.orc_horver_correlation_full.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    hc, vc = ctypes.c_float(), ctypes.c_float()
    diff = np.ascontiguousarray(diff, dtype=np.int16)
    L.orc_horver_correlation_full(P(diff), stride, w, h, ctypes.byref(hc), ctypes.byref(vc))
    return np.float32(hc.value), np.float32(vc.value)


def tx_prune_features(res, bw, bh):
    """orc_tx_prune_features over an int16 plane: (hfeatures, vfeatures) [block, 16]."""
    L = lib()
    L.orc_tx_prune_features.restype = ctypes.c_long
    L.orc_tx_prune_features.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p]
    res = np.ascontiguousarray(res, dtype=np.int16)
    H, W = res.shape
    nb = (W // bw) * (H // bh)
    hf = np.zeros((nb, 16), np.float32)
    vf = np.zeros((nb, 16), np.float32)
    L.orc_tx_prune_features(P(res), W, W, H, bw, bh, P(hf), P(vf))
    return hf, vf


# ------------------------------------------------- inter prediction --
INTER_JOB = np.dtype([("ref_off", "<i8"), ("dst_off", "<i8"), ("pix_row", "<i4"),
                      ("pix_col", "<i4"), ("mv_row", "<i2"), ("mv_col", "<i2"),
                      ("filter_x", "u1"), ("filter_y", "u1"), ("pad", "u1", (2,))], align=True)


def interp_kernel(interp_filter, size, subpel):
    """orc_interp_kernel: the kernel row the oracle uses (taps, int16 array)."""
    L = lib()
    L.orc_interp_kernel.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    out = np.zeros(12, np.int16)
    taps = L.orc_interp_kernel(interp_filter, size, subpel, P(out))
    return out[:taps]


def conv_rounds(bd):
    L = lib()
    r0, r1 = ctypes.c_int(), ctypes.c_int()
    L.orc_conv_rounds(bd, ctypes.byref(r0), ctypes.byref(r1))
    return r0.value, r1.value


def convolve_block(src, src_off, ss, w, h, path, fx, fy, round_0, round_1, bd):
    """orc_convolve_block on a numpy plane (uint8 / uint16); src_off = element
    offset of the block's integer position.  Returns the (h, w) block."""
    L = lib()
    L.orc_convolve_block.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_void_p,
                                     ctypes.c_ssize_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int]
    hb = src.dtype == np.uint16
    out = np.zeros((h, w), src.dtype)
    fx = np.ascontiguousarray(fx if fx is not None else np.zeros(8), np.int16)
    fy = np.ascontiguousarray(fy if fy is not None else np.zeros(8), np.int16)
    L.orc_convolve_block(ctypes.c_void_p(src.ctypes.data + src_off * src.itemsize), ss, P(out),
                         w, w, h, path, P(fx), len(fx), P(fy), len(fy), round_0, round_1, bd,
                         int(hb))
    return out


def build_inter_pred(ref, ref_origin, ref_width, ref_height, ss_x, ss_y, w, h, jobs, dst_shape,
                     bd=8, mvs=None, dst_stride=None):
    """orc_build_inter_pred_batch over INTER_JOB records; ref is a bordered
    numpy plane whose frame origin is element offset ref_origin."""
    L = lib()
    L.orc_build_inter_pred_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.orc_build_inter_pred_batch.restype = ctypes.c_long
    hb = ref.dtype == np.uint16
    jobs = np.ascontiguousarray(jobs)
    out = np.zeros(dst_shape, ref.dtype)
    ds = out.shape[-1] if dst_stride is None else dst_stride
    m = None if mvs is None else np.ascontiguousarray(mvs)
    L.orc_build_inter_pred_batch(ctypes.c_void_p(ref.ctypes.data + ref_origin * ref.itemsize),
                                 ref.strides[0] // ref.itemsize, ref_width, ref_height, ss_x,
                                 ss_y, w, h, P(jobs), len(jobs),
                                 None if m is None else P(m), P(out), ds, bd, int(hb))
    return out


# ------------------------------------------------------ TX-type pruning --
class OrcNNConfig(ctypes.Structure):
    _fields_ = [("num_inputs", ctypes.c_int), ("num_outputs", ctypes.c_int),
                ("num_hidden_layers", ctypes.c_int), ("num_hidden_nodes", ctypes.c_int * 10),
                ("weights", ctypes.c_void_p * 11), ("bias", ctypes.c_void_p * 11)]


def nn_config(cfg):
    """An OrcNNConfig over a json model dict {num_inputs, num_outputs, hidden,
    weights, bias} (arrays kept alive on the returned object)."""
    c = OrcNNConfig()
    c.num_inputs, c.num_outputs = cfg["num_inputs"], cfg["num_outputs"]
    c.num_hidden_layers = len(cfg["hidden"])
    for i, h in enumerate(cfg["hidden"]):
        c.num_hidden_nodes[i] = h
    keep = []
    for i, (w, b) in enumerate(zip(cfg["weights"], cfg["bias"])):
        wa, ba = np.asarray(w, np.float32), np.asarray(b, np.float32)
        keep += [wa, ba]
        c.weights[i] = wa.ctypes.data
        c.bias[i] = ba.ctypes.data
    c._keep = keep
    return c


def nn_predict(inp, cfg, reduce_prec=True):
    L = lib()
    L.orc_nn_predict.argtypes = [ctypes.c_void_p, ctypes.POINTER(OrcNNConfig), ctypes.c_int,
                                 ctypes.c_void_p]
    c = cfg if isinstance(cfg, OrcNNConfig) else nn_config(cfg)
    x = np.ascontiguousarray(inp, np.float32)
    out = np.zeros(c.num_outputs, np.float32)
    L.orc_nn_predict(P(x), ctypes.byref(c), int(reduce_prec), P(out))
    return out


def sort_fi32(k, v, n):
    L = lib()
    L.orc_sort_fi32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    k = np.ascontiguousarray(k, np.float32).copy()
    v = np.ascontiguousarray(v, np.int32).copy()
    L.orc_sort_fi32(P(k), P(v), n)
    return k, v


def prune_tx_2d(res, bw, bh, tx_set_type, prune_mode, thresholds, hor, ver, allowed_in=None,
                allowed_default=0xFFFF):
    """orc_prune_tx_2d over an int16 residual plane: (allowed_out[nblk],
    txk_map[nblk, 16])."""
    L = lib()
    L.orc_prune_tx_2d.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_uint16, ctypes.c_void_p,
                                  ctypes.c_void_p]
    L.orc_prune_tx_2d.restype = ctypes.c_long
    H, W = res.shape
    n = (W // bw) * (H // bh)
    out = np.zeros(n, np.uint16)
    maps = np.zeros((n, 16), np.uint8)
    th = None if thresholds is None else np.ascontiguousarray(thresholds, np.float32)
    hc = None if hor is None else (hor if isinstance(hor, OrcNNConfig) else nn_config(hor))
    vc = None if ver is None else (ver if isinstance(ver, OrcNNConfig) else nn_config(ver))
    ai = None if allowed_in is None else np.ascontiguousarray(allowed_in, np.uint16)
    L.orc_prune_tx_2d(P(res), res.strides[0] // 2, W, H, bw, bh, tx_set_type, prune_mode,
                      None if th is None else P(th),
                      None if hc is None else ctypes.addressof(hc),
                      None if vc is None else ctypes.addressof(vc),
                      None if ai is None else P(ai), allowed_default, P(out), P(maps))
    return out, maps


# ------------------------------------------------------------ TPL block leg --
TPL_BLOCK = np.dtype([("best_ref", "<i4"), ("inter_cost", "<i4"), ("rate_cost", "<i4"),
                      ("eob", "<i4"), ("recon_error", "<i8"), ("sse", "<i8")])


def tpl_block_batch(src, preds, bsize, bd, qindex, threads=1):
    """orc_tpl_block_batch: src [H, W] (uint8 at bd 8, uint16 above), preds
    [nrefs, H, W] of the same type.  Returns (records, recon, ref_costs)."""
    L = lib()
    fn = L.orc_tpl_block_batch
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_int,
                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(OrcQuant), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_int]
    src = np.ascontiguousarray(src)
    preds = np.ascontiguousarray(preds)
    H, W = src.shape
    nrefs = preds.shape[0]
    nb = (W // bsize) * (H // bsize)
    out = np.zeros(nb, TPL_BLOCK)
    recon = np.zeros_like(src)
    costs = np.zeros((nb, nrefs), np.int32)
    q = build_quant(bd, qindex)
    fn(P(src), W, P(preds), preds[0].size, W, nrefs, W, H, bsize, bd, ctypes.byref(q), P(out),
       P(recon), W, P(costs), threads)
    return out, recon, costs


def av1_quant_block(coeff, tx_size, tx_type, bd, qindex, mode, skip_trellis=0,
                    threshold=0xFFFFFFFF, qstep=0, dc_only=0):
    """orc_av1_quant_block -> (flags, qcoeff, dqcoeff, eob)."""
    L = lib()
    fn = L.orc_av1_quant_block
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(OrcQuant), ctypes.c_int, ctypes.c_int, ctypes.c_uint,
                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    c = np.ascontiguousarray(coeff, np.int32)
    qc, dq = np.zeros(len(c), np.int32), np.zeros(len(c), np.int32)
    eob = np.zeros(1, np.uint16)
    q = build_quant(bd, qindex)
    flags = fn(P(c), tx_size, tx_type, bd, ctypes.byref(q), mode, skip_trellis, threshold, qstep,
               dc_only, P(qc), P(dq), P(eob))
    return flags, qc, dq, int(eob[0])


CC_COEFF_COST = 944   # int32 cells of one LV_MAP_COEFF_COST
CC_EOB_COST = 22      # int32 cells of one LV_MAP_EOB_COST


def coeff_costs_blob(coeff_costs, eob_costs):
    """CoeffCosts (av1/encoder/block.h:806-811) as one flat int32 array:
    coeff_costs[5][2] (LV_MAP_COEFF_COST) then eob_costs[7][2]."""
    a = np.ascontiguousarray(coeff_costs, np.int32).reshape(-1)
    b = np.ascontiguousarray(eob_costs, np.int32).reshape(-1)
    assert a.size == 10 * CC_COEFF_COST and b.size == 14 * CC_EOB_COST
    return np.concatenate([a, b])


def cost_coeffs_txb(blob, qcoeff, eob, plane, tx_size, tx_type, txb_skip_ctx=0, dc_sign_ctx=0,
                    tx_type_cost=0, laplacian=False):
    """orc_cost_coeffs_txb: av1_cost_coeffs_txb / _laplacian(adjust_eob 0)."""
    fn = lib().orc_cost_coeffs_txb
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 8
    fn.restype = ctypes.c_int
    q = np.ascontiguousarray(qcoeff, np.int32)
    return fn(P(blob), P(q), eob, plane, tx_size, tx_type, txb_skip_ctx, dc_sign_ctx,
              tx_type_cost, int(laplacian))


def cost_coeffs_txb_batch(blob, qcoeff, eob, plane, tx_size, tx_type, txb_ctx=None,
                          tx_type_cost=0, laplacian=False):
    """orc_cost_coeffs_txb_batch over qcoeff [nblocks, n] -> int32 rates."""
    fn = lib().orc_cost_coeffs_txb_batch
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    q = np.ascontiguousarray(qcoeff, np.int32)
    e = np.ascontiguousarray(eob, np.uint16)
    ctx = None if txb_ctx is None else np.ascontiguousarray(txb_ctx, np.int32)
    out = np.zeros(q.shape[0], np.int32)
    fn(P(blob), P(q), q.shape[1], P(e), q.shape[0], plane, tx_size, tx_type,
       P(ctx) if ctx is not None else None, tx_type_cost, int(laplacian), P(out))
    return out


def rdo_plane_rate(src, pred, tx_size, type_mask, bd, q, rdmult, blob, txb_ctx=None,
                   tx_type_costs=None, block_mask=None, block_map=None, threads=1):
    """orc_rdo_plane_rate: the TX-domain C4 decision with rate =
    orc_cost_coeffs_txb (search_tx_type's cost_coeffs)."""
    fn = lib().orc_rdo_plane_rate
    fn.restype = ctypes.c_long
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(OrcQuant),
                   ctypes.c_int] + [ctypes.c_void_p] * 8 + [ctypes.c_int]
    src = np.ascontiguousarray(src, dtype=np.uint16)
    pred = np.ascontiguousarray(pred, dtype=np.uint16)
    H, W = src.shape
    nb = (W // TX_W[tx_size]) * (H // TX_H[tx_size])
    n = max_eob(tx_size)
    out = np.zeros(nb, RDO_DTYPE)
    qc = np.zeros((nb, n), np.int32)
    dq = np.zeros((nb, n), np.int32)
    arr = lambda a, t: None if a is None else np.ascontiguousarray(a, t)
    ctx, ttc = arr(txb_ctx, np.int32), arr(tx_type_costs, np.int32)
    bm, mp = arr(block_mask, np.uint16), arr(block_map, np.uint8)
    pp = lambda a: None if a is None else P(a)
    fn(P(src), P(pred), W, W, H, tx_size, type_mask, bd, ctypes.byref(q), rdmult, P(blob),
       pp(ctx), pp(ttc), pp(bm), pp(mp), P(out), P(qc), P(dq), threads)
    return out, qc, dq


def optimize_b(blob, tcoeff, qcoeff, dqcoeff, eob, plane, tx_size, tx_type, bd, is_inter,
               x_rdmult, sharpness, dequant, txb_skip_ctx=0, dc_sign_ctx=0, tx_type_cost=0):
    """orc_optimize_b -> (eob, rate, entropy_ctx, qcoeff, dqcoeff) (copies)."""
    fn = lib().orc_optimize_b
    fn.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 8 + [ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    t = np.ascontiguousarray(tcoeff, np.int32)
    q = np.array(qcoeff, np.int32)
    d = np.array(dqcoeff, np.int32)
    dqv = np.ascontiguousarray(dequant, np.int16)
    rate = np.zeros(1, np.int32)
    ec = np.zeros(1, np.uint8)
    e = fn(P(blob), P(t), P(q), P(d), eob, plane, tx_size, tx_type, bd, is_inter, x_rdmult,
           sharpness, P(dqv), txb_skip_ctx, dc_sign_ctx, tx_type_cost, P(rate), P(ec))
    return e, int(rate[0]), int(ec[0]), q, d


def pixel_batch(src, ss, ref, rs, w, h, jobs, threads=1):
    """orc_pixel_batch: (sad [n, 4], var [n], sse [n]) of 8-bit jobs (JOB_DTYPE)."""
    fn = lib().orc_pixel_batch
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 3 + \
        [ctypes.c_void_p, ctypes.c_long] + [ctypes.c_void_p] * 3 + [ctypes.c_int]
    fn.restype = None
    n = len(jobs)
    sad = np.zeros((n, 4), np.uint32)
    var = np.zeros(n, np.uint32)
    sse = np.zeros(n, np.uint32)
    jobs = np.ascontiguousarray(jobs)
    fn(P(src), ss, P(ref), rs, w, h, P(jobs), n, P(sad), P(var), P(sse), threads)
    return sad, var, sse


class OrcConvParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("do_average", "round_0", "round_1", "is_compound",
                                             "use_dist_wtd_comp_avg", "fwd_offset", "bck_offset")]


def get_shear_params(mat):
    """orc_get_shear_params -> (valid, (alpha, beta, gamma, delta))."""
    fn = lib().orc_get_shear_params
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    m = np.ascontiguousarray(mat[:6], np.int32)
    out = np.zeros(4, np.int16)
    ok = fn(P(m), P(out))
    return ok, tuple(int(v) for v in out)


def warp_affine(mat, ref, width, height, stride, pred, p_col, p_row, p_width, p_height,
                p_stride, ss_x, ss_y, bd, hbd, cp, conv_dst, dst_stride, params):
    """orc_warp_affine in place on pred (u8 / u16) and conv_dst (u16 or None);
    cp: dict of OrcConvParams fields; params: (alpha, beta, gamma, delta)."""
    fn = lib().orc_warp_affine
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_void_p] + \
        [ctypes.c_int] * 9 + [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 5
    fn.restype = None
    m = np.ascontiguousarray(mat[:6], np.int32)
    c = OrcConvParams(**cp)
    fn(P(m), P(ref), width, height, stride, P(pred), p_col, p_row, p_width, p_height, p_stride,
       ss_x, ss_y, bd, hbd, ctypes.byref(c), P(conv_dst) if conv_dst is not None else None,
       dst_stride, *params)


def warp_batch(ref, width, height, stride, pred, p_stride, jobs, cp, bd=8, dst=None,
               dst_stride=0, ss_x=0, ss_y=0, threads=1):
    """orc_warp_batch in place on pred / dst (jobs: lavish_dsp.warp.JOB_DTYPE)."""
    fn = lib().orc_warp_batch
    fn.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int,
                                                            ctypes.c_void_p, ctypes.c_int,
                                                            ctypes.c_void_p, ctypes.c_long] + \
        [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int]
    fn.restype = None
    c = OrcConvParams(**cp)
    jobs = np.ascontiguousarray(jobs)
    fn(P(ref), width, height, stride, P(pred), p_stride, P(dst) if dst is not None else None,
       dst_stride, P(jobs), len(jobs), ss_x, ss_y, bd, int(ref.dtype == np.uint16),
       ctypes.byref(c), threads)


def dist_wtd_convolve(path, src, src_stride, dst, dst_stride, w, h, fx, fy, cp, conv,
                      conv_stride, bd, hbd, src_off=0):
    """orc_dist_wtd_convolve in place on dst / conv; src_off: element offset
    of the block's integer position in the flat src array."""
    fn = lib().orc_dist_wtd_convolve
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 3
    fn.restype = None
    fxa = np.ascontiguousarray(fx, np.int16)
    fya = np.ascontiguousarray(fy, np.int16)
    c = OrcConvParams(**cp)
    base = src.ctypes.data + src_off * src.itemsize
    fn(path, ctypes.c_void_p(base), src_stride, P(dst), dst_stride, w, h, P(fxa), len(fxa),
       P(fya), len(fya), ctypes.byref(c), P(conv), conv_stride, bd, hbd)


def interp_table(interp_filter, size):
    """The 16 kernel rows (int16 [16, taps]) of av1_get_interp_filter_params_
    with_block_size(interp_filter, size) as the oracle holds them."""
    return np.stack([interp_kernel(interp_filter, size, p) for p in range(16)])


def convolve_2d_scale(src, src_stride, dst, dst_stride, w, h, fx_table, fy_table, subpel_x_qn,
                      x_step_qn, subpel_y_qn, y_step_qn, cp, conv, conv_stride, bd, hbd,
                      src_off=0):
    """orc_convolve_2d_scale in place on dst / conv (cp: OrcConvParams fields
    incl. is_compound); src_off: element offset of the block's position."""
    fn = lib().orc_convolve_2d_scale
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int] + \
        [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int]
    fn.restype = None
    fx = np.ascontiguousarray(fx_table, np.int16)
    fy = np.ascontiguousarray(fy_table, np.int16)
    c = OrcConvParams(**cp)
    base = src.ctypes.data + src_off * src.itemsize
    fn(ctypes.c_void_p(base), src_stride, P(dst), dst_stride, w, h, P(fx), fx.shape[1], P(fy),
       fy.shape[1], subpel_x_qn, x_step_qn, subpel_y_qn, y_step_qn, ctypes.byref(c), P(conv),
       conv_stride, bd, hbd)


def dist_wtd_batch(src, src_stride, dst, dst_stride, conv, conv_stride, w, h, jobs, fx_table,
                   fy_table, cp, bd=8, threads=1):
    """orc_dist_wtd_batch in place on dst / conv (jobs: lavish_dsp.compound.JOB_DTYPE,
    fx_table / fy_table: int16 [16, taps])."""
    fn = lib().orc_dist_wtd_batch
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 3
    fn.restype = None
    fx = np.ascontiguousarray(fx_table, np.int16)
    fy = np.ascontiguousarray(fy_table, np.int16)
    c = OrcConvParams(**cp)
    jobs = np.ascontiguousarray(jobs)
    fn(P(src), src_stride, P(dst), dst_stride, P(conv), conv_stride, w, h, P(jobs), len(jobs),
       P(fx), fx.shape[1], P(fy), fy.shape[1], ctypes.byref(c), bd, int(src.dtype == np.uint16),
       threads)


def convolve_2d_scale_batch(src, src_stride, dst, dst_stride, conv, conv_stride, w, h, jobs,
                            fx_table, fy_table, cp, bd=8, threads=1):
    """orc_convolve_2d_scale_batch in place on dst / conv (jobs:
    lavish_dsp.scale.JOB_DTYPE; fx_table / fy_table: int16 [16, taps];
    conv None outside the compound forms)."""
    fn = lib().orc_convolve_2d_scale_batch
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 3
    fn.restype = None
    fx = np.ascontiguousarray(fx_table, np.int16)
    fy = np.ascontiguousarray(fy_table, np.int16)
    c = OrcConvParams(**cp)
    jobs = np.ascontiguousarray(jobs)
    fn(P(src), src_stride, P(dst) if dst is not None else None, dst_stride,
       P(conv) if conv is not None else None, conv_stride, w, h, P(jobs), len(jobs), P(fx),
       fx.shape[1], P(fy), fy.shape[1], ctypes.byref(c), bd, int(src.dtype == np.uint16), threads)


def rd_select(rdmult, rates, dists):
    """orc_rd_select: RDCOST of each (rate, dist) and the index of the first
    strictly lowest (search_tx_type's update)."""
    L = lib()
    rates = np.ascontiguousarray(rates, np.int32)
    dists = np.ascontiguousarray(dists, np.int64)
    rds = np.zeros(len(rates), np.int64)
    L.orc_rd_select.restype = ctypes.c_int
    best = L.orc_rd_select(ctypes.c_int(int(rdmult)), P(rates), P(dists),
                           ctypes.c_int(len(rates)), P(rds))
    return best, rds
