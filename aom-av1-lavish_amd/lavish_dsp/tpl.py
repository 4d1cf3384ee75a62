"""The TPL model's per-block inter leg on the MI355X backend (SURVEY.md 8(f)
rank 1): lavish_tpl_block_batch, and tpl_frame, which chains the whole leg on
the device for every 16x16 block x reference of a frame:

  av1_full_pixel_search (motion_estimation, av1/encoder/tpl_model.c:249-300:
    tpl_sf.search_method, step_param = reduce_first_step_size, the frame's
    mv costs, a cost list)            -> lavish_full_pixel_search_batch
  find_fractional_mv_step (MV_COST_NONE, tpl_sf.subpel_force_stop, 2-tap)
                                      -> lavish_find_best_sub_pixel_tree_batch
  the inter predictor (EIGHTTAP_REGULAR, av1_enc_build_one_inter_predictor)
                                      -> lavish_build_inter_pred_after_subpel
  tpl_get_satd_cost per reference, the cheapest one, txfm_quant_rdcost
                                      -> lavish_tpl_block_batch

The full-pel step runs with the reference's per-block start-mv selection
(tpl_motion_search: neighbouring tpl mvs, is_alike_mv, prune_starting_mv;
a device wavefront, since each block needs its finished neighbours) or,
with neighbour_starts=False, from the jobs' start mvs.  Intra candidates
stay with the caller."""
import ctypes

import numpy as np

from . import QuantParams, _lib, _stream_ptr
from . import inter as I
from . import motion as M

TPL_BLOCK_DTYPE = np.dtype([("best_ref", "<i4"), ("inter_cost", "<i4"), ("rate_cost", "<i4"),
                            ("eob", "<i4"), ("recon_error", "<i8"), ("sse", "<i8")])
assert TPL_BLOCK_DTYPE.itemsize == 32

_vp, _i32, _i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
_lib.lavish_tpl_block_batch.argtypes = [_vp, _i32, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _i32,
                                        ctypes.POINTER(QuantParams), _vp, _vp, _i32, _vp, _vp]
_lib.lavish_tpl_block_batch.restype = _i32

TPL_BSIZE = 16  # set_tpl_stats_block_size (tpl_model.c:137-145)
# tpl_data->border_in_pixels = ALIGN_POWER_OF_TWO(16 + 2 * AOM_INTERP_EXTEND, 5)
# (tpl_model.c:155-156): the mv limits of the TPL motion search
TPL_BORDER = 32


def tpl_block_batch(src, preds, bsize, bit_depth, qp, width=None, height=None, out=None,
                    recon=None, ref_costs=None, stream=None):
    """lavish_tpl_block_batch.  src: 2-D device tensor whose [0, 0] is the
    frame origin (a view into a padded plane is fine: its row stride is
    used); preds: [nrefs, H, W] device tensor (or a 2-D one for a single
    reference); qp: QuantParams for LAVISH_QUANT_FP; ref_costs: None, True
    (allocate) or an int32 [nblocks, nrefs] device tensor.  Returns (records
    byte tensor, recon tensor, costs or None)."""
    import torch
    assert src.dtype in (torch.uint8, torch.uint16, torch.int16) and preds.dtype == src.dtype
    assert (src.dtype == torch.uint8) == (bit_depth == 8), "8-bit planes are uint8, else u16"
    assert src.stride(1) == 1 and preds.stride(-1) == 1
    if preds.dim() == 2:
        preds = preds.unsqueeze(0)
    nrefs = preds.shape[0]
    H = src.shape[0] if height is None else height
    W = src.shape[1] if width is None else width
    nb = (W // bsize) * (H // bsize)
    if out is None:
        out = torch.empty(nb * TPL_BLOCK_DTYPE.itemsize, dtype=torch.uint8, device=src.device)
    if recon is None:
        recon = torch.empty((H, W), dtype=src.dtype, device=src.device)
    costs = ref_costs
    if ref_costs is True:
        costs = torch.empty((nb, nrefs), dtype=torch.int32, device=src.device)
    if costs is not None:
        assert costs.dtype == torch.int32 and costs.numel() >= nb * nrefs
    pp = preds.stride(0) if nrefs > 1 else 0
    rc = _lib.lavish_tpl_block_batch(
        _vp(src.data_ptr()), src.stride(0), _vp(preds.data_ptr()), pp, preds.stride(1), nrefs,
        W, H, bsize, bit_depth, ctypes.byref(qp), _vp(out.data_ptr()), _vp(recon.data_ptr()),
        recon.stride(0), _vp(costs.data_ptr()) if costs is not None else None,
        _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_tpl_block_batch rejected its arguments (rc=%d)" % rc)
    return out, recon, costs


def records_numpy(out):
    return out.cpu().numpy().view(TPL_BLOCK_DTYPE)


class TplMvParams(ctypes.Structure):
    """LavishTplMvParams: the tpl_sf / mv_sf fields motion_estimation reads."""
    _fields_ = [("search_method", _i32), ("step_param", _i32), ("use_downsampled_sad", _i32),
                ("prune_starting_mv", _i32), ("skip_alike_starting_mv", _i32),
                ("subpel_force_stop", _i32)]


_lib.lavish_tpl_motion_sync_ints.argtypes = [_i32, _i32]
_lib.lavish_tpl_motion_sync_ints.restype = _i64
_lib.lavish_tpl_motion_search.argtypes = [_vp, _i32, _vp, _i32, _vp, _i32, _i32, _i32,
                                          ctypes.POINTER(TplMvParams),
                                          ctypes.POINTER(M.MvCostParams), _vp, _vp, _vp, _vp,
                                          _vp, _vp, _vp]
_lib.lavish_tpl_motion_search.restype = _i32
INVALID_MV = -0x7FFF8000  # 0x80008000 as int32


def pack_mv(row, col):
    """int_mv.as_int of (row, col) (1/8 pel, row in the low half)."""
    r = np.asarray(row, np.int64) & 0xFFFF
    c = np.asarray(col, np.int64) & 0xFFFF
    return ((c << 16) | r).astype(np.uint32).view(np.int32)


def unpack_mv(m):
    m = np.asarray(m).astype(np.int32).view(np.uint32)
    return ((m & 0xFFFF).astype(np.uint16).view(np.int16).astype(np.int32),
            (m >> 16).astype(np.uint16).view(np.int16).astype(np.int32))


def tpl_motion_search(src, ref, jobs, cols, rows, nrefs, cost, search_method="fast_bigdia",
                      step_param=6, use_downsampled_sad=False, prune_starting_mv=3,
                      skip_alike_starting_mv=2, third_pass_mvs=None, cost_list=True,
                      out=None, stream=None):
    """lavish_tpl_motion_search: mode_estimation's per-reference motion search
    with neighbour start mvs, as a device wavefront.  src / ref / jobs as
    motion.full_pixel_search_batch (jobs [nrefs][rows * cols] raster, limits
    = x->mv_limits); third_pass_mvs: None or an int32 device tensor of int_mv.
    out: None or a dict of preallocated tensors (mvs, fp, cl, centers, sync).
    Returns that dict: mvs int32 [nrefs * rows * cols] (int_mv), fp (RESULT
    records), cl (int32 [n, 5] or None), centers (int_mv), sync."""
    import torch
    assert src.dtype == torch.uint8 and ref.dtype == torch.uint8
    assert src.is_contiguous() and ref.is_contiguous(), "planes must be C-contiguous"
    n = nrefs * rows * cols
    assert jobs.numel() == n * M.JOB_DTYPE.itemsize
    dev = src.device
    if out is None:
        out = {"mvs": torch.empty(n, dtype=torch.int32, device=dev),
               "fp": torch.empty(n * M.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev),
               "cl": torch.empty((n, 5), dtype=torch.int32, device=dev) if cost_list else None,
               "centers": torch.empty(n, dtype=torch.int32, device=dev),
               "sync": torch.empty(int(_lib.lavish_tpl_motion_sync_ints(nrefs, rows)),
                                   dtype=torch.int32, device=dev)}
    p = TplMvParams(M.SEARCH_METHODS[search_method], step_param, int(use_downsampled_sad),
                    prune_starting_mv, skip_alike_starting_mv, M.FULL_PEL)
    if third_pass_mvs is not None:
        assert third_pass_mvs.dtype == torch.int32 and third_pass_mvs.numel() == n
    cl = out["cl"]
    rc = _lib.lavish_tpl_motion_search(
        _vp(src.data_ptr()), src.stride(0), _vp(ref.data_ptr()), src.stride(0),
        _vp(jobs.data_ptr()), cols, rows, nrefs, ctypes.byref(p), ctypes.byref(cost),
        _vp(third_pass_mvs.data_ptr()) if third_pass_mvs is not None else None,
        _vp(out["mvs"].data_ptr()), _vp(out["fp"].data_ptr()),
        _vp(cl.data_ptr()) if cl is not None else None, _vp(out["centers"].data_ptr()),
        _vp(out["sync"].data_ptr()), _stream_ptr(stream))
    if rc != 0:
        raise ValueError("lavish_tpl_motion_search rejected its arguments (rc=%d)" % rc)
    return out


def tpl_motion_failures(out):
    """Waits that timed out in the last tpl_motion_search (0 = valid)."""
    return int(out["sync"][-1].item())


class TplFrame:
    """Device state of one TPL frame leg (8-bit): padded source / reference
    planes (border >= AOM_BORDER_IN_PIXELS for the predictor), the motion jobs
    of every (block, reference), and the intermediate buffers, so that step()
    launches only kernels."""

    def __init__(self, src_np, refs_np, width, height, border, qindex, rdmult,
                 search_method="fast_bigdia", step_param=6, forced_stop=M.FULL_PEL,
                 subpel_method="pruned_more", start_mvs=None, device="cuda",
                 neighbour_starts=True, prune_starting_mv=3, skip_alike_starting_mv=2,
                 use_downsampled_sad=False, mv_border=TPL_BORDER):
        import torch
        from . import build_quant_params, QUANT_FP
        assert border >= I.AOM_BORDER_IN_PIXELS
        self.W, self.H, self.border = width, height, border
        self.nrefs = refs_np.shape[0]
        self.stride = src_np.shape[1]
        bs = TPL_BSIZE
        self.src = torch.from_numpy(src_np).to(device)
        self.refs = torch.from_numpy(refs_np).to(device)
        org = border * self.stride + border
        self.org = org
        jobs = M.frame_jobs(width, height, self.stride, border, src_np.size, bs, bs, self.nrefs,
                            mv_border=mv_border)
        # the reference's start mvs (mode_estimation, tpl_model.c:640-735):
        # neighbour-seeded centres, a device wavefront; needs FULL_PEL
        self.neighbour_starts = neighbour_starts and start_mvs is None
        assert not self.neighbour_starts or forced_stop == M.FULL_PEL, \
            "neighbour start mvs need tpl_sf.subpel_force_stop FULL_PEL"
        self.prune, self.alike = prune_starting_mv, skip_alike_starting_mv
        self.skip_sad = use_downsampled_sad
        self.cols, self.rows = width // bs, height // bs
        if start_mvs is not None:
            jobs["start_row"], jobs["start_col"] = start_mvs[:, 0], start_mvs[:, 1]
        self.jobs_np = jobs
        self.jobs = M.to_device(jobs)
        sj = M.subpel_jobs(width, height, mv_border, bs, bs, jobs,
                           np.zeros(len(jobs), M.RESULT_DTYPE))
        self.sub_jobs = M.to_device(sj)
        # inter prediction jobs: job j = (ref k, block) -> pred plane k, same position
        nb = (width // bs) * (height // bs)
        ij = []
        for k in range(self.nrefs):
            pj = I.plane_jobs(width, height, bs, bs, (0, 0), ref_off=k * src_np.size,
                              dst_stride=width)
            pj["dst_off"] += k * width * height
            ij.append(pj)
        self.inter_jobs = M.to_device(np.concatenate(ij))
        self.nb = nb
        allow_hp = qindex < 128
        self.allow_hp = allow_hp
        self.mv_costs = M.MvCosts(*M.default_mv_cost_tables(allow_hp), device=device)
        self.cost = self.mv_costs.cost_params(M.sad_per_bit(qindex), M.error_per_bit(rdmult),
                                              M.MV_COST_ENTROPY)
        self.cost_none = M.l1_cost_params(M.MV_COST_NONE)
        self.search_method, self.step_param = search_method, step_param
        self.forced_stop, self.subpel_method = forced_stop, subpel_method
        self.qp = build_quant_params(8, qindex, QUANT_FP)
        n = len(jobs)
        self.fp = torch.empty(n * M.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=device)
        self.cl = torch.empty((n, 5), dtype=torch.int32, device=device)
        self.sub = torch.empty(n * M.SUBPEL_RESULT_DTYPE.itemsize, dtype=torch.uint8,
                               device=device)
        self.preds = torch.empty((self.nrefs, height, width), dtype=torch.uint8, device=device)
        self.out = torch.empty(nb * TPL_BLOCK_DTYPE.itemsize, dtype=torch.uint8, device=device)
        self.recon = torch.empty((height, width), dtype=torch.uint8, device=device)
        self.costs = torch.empty((nb, self.nrefs), dtype=torch.int32, device=device)
        self.src_view = self.src[border:border + height, border:border + width]
        self.mv_out = None
        if self.neighbour_starts:
            self.mv_out = {"mvs": torch.empty(n, dtype=torch.int32, device=device), "fp": self.fp,
                           "cl": self.cl,
                           "centers": torch.empty(n, dtype=torch.int32, device=device),
                           "sync": torch.empty(int(_lib.lavish_tpl_motion_sync_ints(
                               self.nrefs, self.rows)), dtype=torch.int32, device=device)}

    def step(self, stream=None, ref_costs=True, check=True):
        """One TPL frame leg.  check (default): wait for the frame and raise
        if a wavefront wait timed out -- such a frame's start mvs are not the
        reference's (the kernel skips the unpublished neighbour and counts
        it); check=False leaves the frame asynchronous, and the caller must
        call check() before using the results."""
        bs = TPL_BSIZE
        self._stream = stream
        if self.neighbour_starts:
            tpl_motion_search(self.src, self.refs, self.jobs, self.cols, self.rows, self.nrefs,
                              self.cost, self.search_method, self.step_param, self.skip_sad,
                              self.prune, self.alike, out=self.mv_out, stream=stream)
        else:
            M.full_pixel_search_batch(self.src, self.refs, bs, bs, self.jobs, self.cost,
                                      self.search_method, self.step_param, self.skip_sad, True,
                                      out=self.fp, cost_lists=self.cl, stream=stream)
        M.find_best_sub_pixel_tree_batch(self.src, self.refs, bs, bs, self.sub_jobs,
                                         self.cost_none, self.subpel_method, self.forced_stop,
                                         self.allow_hp, 1, fullpel=self.fp, cost_lists=self.cl,
                                         out=self.sub, stream=stream)
        I.build_inter_pred_batch(self.refs.view(-1, self.stride), self.org, self.W, self.H, bs, bs,
                                 self.inter_jobs, dst=self.preds.view(-1, self.W),
                                 dst_stride=self.W, bit_depth=8, mvs=self.sub, stream=stream)
        tpl_block_batch(self.src_view, self.preds, bs, 8, self.qp, out=self.out,
                        recon=self.recon, ref_costs=self.costs if ref_costs else None,
                        stream=stream)
        if check:
            self.check()
        return self.out

    def check(self):
        """Raise if the last wavefront's waits timed out.  Synchronises the
        stream step() ran on first: the failure count is written there, and a
        read ordered on another stream could see it before the kernel ends."""
        import torch
        st = getattr(self, "_stream", None)
        if st is not None:
            st.synchronize()
        else:
            torch.cuda.current_stream().synchronize()
        if self.neighbour_starts and tpl_motion_failures(self.mv_out):
            raise RuntimeError("tpl motion wavefront: %d wait(s) timed out; the frame's start "
                               "mvs are invalid" % tpl_motion_failures(self.mv_out))
