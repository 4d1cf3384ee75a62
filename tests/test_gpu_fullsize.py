"""GPU parity at the BASELINE.json configurations' full sizes (SURVEY.md
8(d)), every job / block / superblock against the oracle:

* C2: lavish_txq_frame -- the call bench.py times -- on the bench's 1920x1080
  residual: every block of all 14 TX sizes <= 32x32 x every valid TX type,
  qcoeff / dqcoeff / eob bit-exact;

* C3: DIAMOND full-pel search of every 16x16 block of a 1920x1080 frame
  against 7 references (56 280 jobs) with the 1080p speed features bench.py
  times (downsampled SAD, entropy mv cost, cost lists) and the sub-pel
  refinement chained after it;
* C4: the 3840x2160 10-bit RDO step (all candidate sizes / types, per-SB TX
  size, reconstruction) -- records, sb_tx_size and the reconstruction;
* C5 at world 1: the SB-row band processor of lavish_dsp/shard.py over 3
  bands on 3 streams equals the whole-frame step.
"""
import gc
import os

import numpy as np
import pytest

import _oracle as O
from _c4ref import oracle_frame_c

pytestmark = pytest.mark.gpu

THREADS = max(1, min(32, os.cpu_count() or 1))


@pytest.fixture(scope="module")
def L():
    import torch
    assert torch.cuda.is_available()
    import lavish_dsp
    return lavish_dsp


def _bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_c2_txq_frame_1080p_all_blocks(L):
    """The bench's C2 leg exactly as timed (lavish_txq_frame, one launch per
    size class) against the oracle's txq_plane of every size."""
    import torch
    import lavish_dsp.synth as synth
    res = synth.residual_plane(1920, 1080, 8, seed=1234)
    dres = torch.from_numpy(res).cuda()
    sizes = [s for s in range(19) if L.TX_W[s] <= 32 and L.TX_H[s] <= 32]
    qp = L.build_quant_params(8, 128, L.QUANT_FP)
    frame = L.FrameOutputs(dres, sizes)
    outs = L.txq_frame(dres, frame, qp)
    torch.cuda.synchronize()
    oq = O.build_quant(8, 128)
    for s in sizes:
        qc, dq, eob = O.txq_plane(res, s, L.valid_type_mask(s), oq, threads=THREADS)
        np.testing.assert_array_equal(outs[s]["qcoeff"].cpu().numpy(), qc.transpose(1, 0, 2),
                                      err_msg="size %d qcoeff" % s)
        np.testing.assert_array_equal(outs[s]["dqcoeff"].cpu().numpy(), dq.transpose(1, 0, 2),
                                      err_msg="size %d dqcoeff" % s)
        np.testing.assert_array_equal(outs[s]["eob"].cpu().numpy().view(np.uint16), eob.T,
                                      err_msg="size %d eob" % s)
        del qc, dq, eob


def test_c3_1080p_7refs_all_jobs(L):
    """The bench's C3 leg (DIAMOND, downsampled SAD, MV_COST_ENTROPY over the
    default nmv tables, cost lists) and its c3sub continuation (pruned_more
    from the device results and cost lists) on all 56 280 jobs."""
    import torch
    import lavish_dsp.motion as M
    import lavish_dsp.synth as synth
    b = _bench()
    W, H, R, border, qindex, rdmult = 1920, 1080, 7, 160, 128, 2000
    src, refs = synth.motion_planes(W, H, R, border, seed=1234)
    st = src.shape[1]
    jobs = M.frame_jobs(W, H, st, border, src.size, b.C3_BLOCK, b.C3_BLOCK, R)
    assert len(jobs) == 56280
    allow_hp = qindex < 128
    mvj, mvc = M.default_mv_cost_tables(allow_hp)
    spb, epb = M.sad_per_bit(qindex), M.error_per_bit(rdmult)
    cp = M.MvCosts(mvj, mvc).cost_params(spb, epb, b.C3_COST)
    tsrc, trefs = torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda()
    fp, cl = M.full_pixel_search_batch(tsrc, trefs, b.C3_BLOCK, b.C3_BLOCK, M.to_device(jobs), cp,
                                       "diamond", 0, b.C3_SKIP, b.C3_CL)
    sj = M.subpel_jobs(W, H, border, b.C3_BLOCK, b.C3_BLOCK, jobs,
                       np.zeros(len(jobs), M.RESULT_DTYPE))
    sub = M.find_best_sub_pixel_tree_batch(tsrc, trefs, b.C3_BLOCK, b.C3_BLOCK, M.to_device(sj),
                                           cp, "pruned_more", b.SUB_FORCED_STOP, allow_hp,
                                           b.SUB_ITERS, fullpel=fp, cost_lists=cl)
    # the bench's form: candidate rows from the tiled copy (LavishRefTiles)
    tiles = M.RefTiles(trefs, st).build()
    fpt, clt = M.full_pixel_search_batch(tsrc, trefs, b.C3_BLOCK, b.C3_BLOCK, M.to_device(jobs),
                                         cp, "diamond", 0, b.C3_SKIP, b.C3_CL, tiles=tiles)
    torch.cuda.synchronize()
    got, got_cl = M.results_numpy(fp), cl.cpu().numpy()
    np.testing.assert_array_equal(M.results_numpy(fpt), got)
    np.testing.assert_array_equal(clt.cpu().numpy(), got_cl)
    exp, exp_cl = O.full_pixel_search_batch(src.reshape(-1), refs.reshape(-1), st, b.C3_BLOCK,
                                            b.C3_BLOCK, jobs, "diamond", 0, b.C3_COST, spb, epb,
                                            mvj, mvc, skip=b.C3_SKIP, cost_list=b.C3_CL,
                                            threads=THREADS)
    for f in ("best_row", "best_col", "bestsme", "steps"):  # the oracle has no search count
        np.testing.assert_array_equal(got[f], exp[f], err_msg=f)
    np.testing.assert_array_equal(got_cl, exp_cl)
    assert (np.abs(got["best_row"]) + np.abs(got["best_col"]) > 0).mean() > 0.5
    sj_exp = M.subpel_jobs(W, H, border, b.C3_BLOCK, b.C3_BLOCK, jobs, exp)
    sexp = O.subpel_search_batch(src.reshape(-1), refs.reshape(-1), st, b.C3_BLOCK, b.C3_BLOCK,
                                 sj_exp, 2, b.SUB_FORCED_STOP, allow_hp, b.SUB_ITERS, b.C3_COST,
                                 epb, mvj, mvc, exp_cl, threads=THREADS)
    sgot = M.subpel_results_numpy(sub)
    for f in ("best_row", "best_col", "besterr", "distortion", "sse"):
        np.testing.assert_array_equal(sgot[f], sexp[f], err_msg="subpel " + f)


def _c4_planes(W, H):
    import lavish_dsp.synth as synth
    src = synth.frame(W, H, 10, 1234).astype(np.uint16)
    pred = synth.shifted(synth.frame(W, H, 10, 1235), 3, -2).astype(np.uint16)
    return src, pred


def test_c4_4k_10bit_frame(L):
    """bench.py --workload c4's frame and parameters."""
    import torch
    W, H, rdmult = 3840, 2160, 2000
    src, pred = _c4_planes(W, H)
    masks = dict(L.C4_TYPE_MASKS)
    per, choice, recon = oracle_frame_c(src, pred, 10, masks, rdmult, threads=THREADS)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    fr = L.RdoFrame(ts)
    L.rdo_frame(ts, tp, fr, L.build_quant_params(10, 128, L.QUANT_FP), rdmult, 10)
    for s in masks:
        got = L.rdo_records(fr.outs[s])
        for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
            np.testing.assert_array_equal(got[f], per[s][0][f], err_msg="%d %s" % (s, f))
        np.testing.assert_array_equal(fr.outs[s]["qcoeff"].cpu().numpy(), per[s][1])
        np.testing.assert_array_equal(fr.outs[s]["dqcoeff"].cpu().numpy(), per[s][2])
    np.testing.assert_array_equal(fr.sb_tx_size.cpu().numpy(), choice)
    np.testing.assert_array_equal(fr.recon.cpu().numpy().view(np.uint16), recon)
    assert len(np.unique(choice)) > 1
    # every size's kernels on the caller's stream (lavish_set_fan_width(1), the
    # profiling arrangement): the same frame
    fr1 = L.RdoFrame(ts)
    L.set_fan_width(1)
    try:
        L.rdo_frame(ts, tp, fr1, L.build_quant_params(10, 128, L.QUANT_FP), rdmult, 10)
        torch.cuda.synchronize()
    finally:
        L.set_fan_width(3)
    np.testing.assert_array_equal(fr1.sb_tx_size.cpu().numpy(), choice)
    np.testing.assert_array_equal(fr1.recon.cpu().numpy().view(np.uint16), recon)
    for s in masks:
        np.testing.assert_array_equal(L.rdo_records(fr1.outs[s])["rdcost"], per[s][0]["rdcost"])


def test_c5_bands_world1_three_streams(L):
    """shard.c4_band_processor on the 3 bands bands(H, 3) gives, each on its
    own stream, the whole-frame step's reconstruction (SB rows are
    independent for C4); the bands run concurrently, so the library's reused
    device scratch must be ordered across streams."""
    import torch
    import lavish_dsp.shard as shard
    W, H, rdmult = 1280, 720, 1700
    src, pred = _c4_planes(W, H)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    qp = L.build_quant_params(10, 128, L.QUANT_FP)
    whole = L.RdoFrame(ts)
    L.rdo_frame(ts, tp, whole, qp, rdmult, 10)
    torch.cuda.synchronize()
    frames = {}
    proc = shard.c4_band_processor(ts, tp, qp, rdmult, 10, frames)
    streams = [torch.cuda.Stream() for _ in range(3)]
    parts = []
    for it in range(2):  # twice: the second pass reuses every cached buffer
        parts = []
        for (y0, y1), st in zip(shard.bands(H, 3), streams):
            with torch.cuda.stream(st):
                parts.append(proc(y0, y1).clone())
        torch.cuda.synchronize()
    full = torch.cat(parts, 0)
    np.testing.assert_array_equal(full.cpu().numpy(), whole.recon.cpu().numpy())
    # and through sharded_frame (world 1: one band, the whole frame)
    rect = shard.c4_rect_processor(ts, tp, qp, rdmult, 10, frames)
    one = shard.sharded_frame(H, W, 0, 1, rect)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(one.cpu().numpy(), whole.recon.cpu().numpy())


def test_c5_partition_rects_on_gpu(L):
    """Every rank's band and tail rectangle of shard.partition for worlds
    2..8 (tails are column segments: views with the frame's stride), each
    computed by the HIP C4 step on its own, assemble to the whole-frame
    reconstruction; so does the row-wavefront form at world 1 (3 column
    chunks per SB row), once with copies and once writing every chunk
    straight into the frame.  C5's configuration: 3840x2160 10-bit."""
    import torch
    import lavish_dsp.shard as shard
    W, H, rdmult = 3840, 2160, 1700   # 34 SB rows: tails for every world but 2
    src, pred = _c4_planes(W, H)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    qp = L.build_quant_params(10, 128, L.QUANT_FP)
    whole = L.RdoFrame(ts)
    L.rdo_frame(ts, tp, whole, qp, rdmult, 10)
    ref = whole.recon.cpu().numpy()
    frames = {}
    rect = shard.c4_rect_processor(ts, tp, qp, rdmult, 10, frames)
    for world in range(2, 9):
        full = torch.empty_like(ts)
        for band, tail in shard.partition(H, W, world):
            for r in (band, tail):
                if r is not None:
                    y0, y1, x0, x1 = r
                    full[y0:y1, x0:x1] = rect(*r)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(full.cpu().numpy(), ref, err_msg="world %d" % world)
    wf = shard.wavefront_frame(H, W, 0, 1, rect, chunks=3, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(wf.cpu().numpy(), ref)
    # direct launches / each chunk a replayed HIP graph / graphs over 4
    # streams with the chunk dependencies as events / one chunk per row (the
    # bench's form: the rows in order on one of the streams, no events)
    for graphs, nst, chunks in ((False, 0, 4), (True, 0, 4), (True, 4, 4), (False, 4, 1),
                                (True, 4, 1)):
        out = torch.full_like(ts, -1)
        direct = shard.c4_rect_processor(ts, tp, qp, rdmult, 10, {}, out=out, graphs=graphs)
        streams = [torch.cuda.Stream() for _ in range(nst)] or None
        if graphs and streams:
            # every chunk's graph captured first, on one stream (as bench.py
            # does); the captures run after the uncaptured whole-frame step
            # above on this thread -- the order that crashed the host inside
            # hipGraphLaunch before captures got their own fork / join set
            shard.wavefront_frame(H, W, 0, 1, direct, chunks=chunks, out=out)
            torch.cuda.synchronize()
        for _ in range(2):  # the second pass replays every cached chunk
            out.fill_(-1)
            wf = shard.wavefront_frame(H, W, 0, 1, direct, chunks=chunks, out=out,
                                       streams=streams)
            torch.cuda.synchronize()
            assert wf.data_ptr() == out.data_ptr()
            np.testing.assert_array_equal(out.cpu().numpy(), ref,
                                          err_msg="graphs %s chunks %d" % (graphs, chunks))
        # this case's graphs freed here, not by a later collection in the
        # middle of the next case's replays
        del direct, wf
        gc.collect()
        torch.cuda.synchronize()


def _rect_records(whole, s, rect, W, H, L):
    """The whole-frame records of size s restricted to a rectangle (raster
    order over the rectangle's blocks, as a rectangle's own step writes them)."""
    w, h = L.TX_W[s], L.TX_H[s]
    y0, y1, x0, x1 = rect
    rec = L.rdo_records(whole.outs[s]).reshape(H // h, W // w)
    return rec[y0 // h:y1 // h, x0 // w:x1 // w].reshape(-1)


def test_c5_tile_form_on_gpu_as_timed(L):
    """The C5 tile form exactly as bench.py's c5_leg (and --c5-emulate) runs
    it: grid_partition(2160, 3840, G) for G = 2..8, each rank's tile through
    c4_rect_processor(..., out=frame, graphs=True) -- one captured HIP graph
    per tile writing its reconstruction straight into its view of the frame --
    replayed twice (capture, then replay), and once more through the direct
    (uncaptured) step.  The assembled frame, every tile's per-SB TX sizes and
    every candidate size's records and coefficients equal the whole-frame
    step's, which test_c4_4k_10bit_frame holds to the oracle.  Tiles are
    multi-row, column-cut rectangles (17 x 15 SBs at G = 8): strided views,
    the small-rectangle rdo_small_kernel selection, a fan set per graph.
    Reference dependency: ethread.c:113-160 (SBs of one frame are
    independent for C4 as defined)."""
    import torch
    import lavish_dsp.shard as shard
    W, H, rdmult, qindex = 3840, 2160, 2000, 128
    src, pred = _c4_planes(W, H)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    qp = L.build_quant_params(10, qindex, L.QUANT_FP)
    whole = L.RdoFrame(ts)
    L.rdo_frame(ts, tp, whole, qp, rdmult, 10)
    torch.cuda.synchronize()
    ref = whole.recon.cpu().numpy()
    ref_sb = whole.sb_tx_size.cpu().numpy().reshape(34, 60)
    for G in range(2, 9):
        rects = shard.grid_partition(H, W, G)
        assert len(rects) == G
        for graphs in (True, False):
            frame = torch.full_like(ts, -1)
            frames = {}
            proc = shard.c4_rect_processor(ts, tp, qp, rdmult, 10, frames, out=frame,
                                           graphs=graphs)
            for it in range(2 if graphs else 1):
                frame.fill_(-1)
                for r in rects:
                    got = proc(*r)
                    y0, y1, x0, x1 = r
                    assert got.data_ptr() == frame[y0:y1, x0:x1].data_ptr()
                torch.cuda.synchronize()
                np.testing.assert_array_equal(frame.cpu().numpy(), ref,
                                              err_msg="G %d graphs %s pass %d" % (G, graphs, it))
            for r in rects:
                fr = frames[r]
                y0, y1, x0, x1 = r
                np.testing.assert_array_equal(
                    fr.sb_tx_size.cpu().numpy().reshape((y1 - y0 + 63) // 64, (x1 - x0 + 63) // 64),
                    ref_sb[y0 // 64:(y1 + 63) // 64, x0 // 64:(x1 + 63) // 64],
                    err_msg="G %d rect %s sb_tx_size" % (G, r))
                for s in fr.sizes:
                    w, h = L.TX_W[s], L.TX_H[s]
                    exp = _rect_records(whole, s, r, W, H, L)
                    got = L.rdo_records(fr.outs[s])
                    for f in ("best_type", "eob", "rate", "satd", "dist", "sse", "rdcost"):
                        np.testing.assert_array_equal(got[f], exp[f],
                                                      err_msg="G %d %s size %d %s" % (G, r, s, f))
                    if G in (2, 8):   # coefficients too (the largest and smallest tiles)
                        nb = (W // w) * (H // h)
                        q = whole.outs[s]["qcoeff"].view(H // h, W // w, -1)
                        qe = q[y0 // h:y1 // h, x0 // w:x1 // w].reshape(-1, q.shape[-1])
                        assert torch.equal(fr.outs[s]["qcoeff"], qe), (G, r, s, nb)
            del proc, frames
            gc.collect()
            torch.cuda.synchronize()


def test_rdo_graph_replays_new_inputs(L):
    """lavish_rdo_graph_create captures the C4 step for fixed buffers; a replay
    after the planes' contents change gives the direct step's result on the
    new contents (records, coefficients, reconstruction, per-SB sizes)."""
    import torch
    W, H, rdmult = 640, 448, 1700
    src, pred = _c4_planes(W, H)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    qp = L.build_quant_params(10, 128, L.QUANT_FP)
    gfr = L.RdoFrame(ts)
    # creation runs the step once after the caller's queued work on the
    # outputs: the fill below must not land after the warm-up
    gfr.recon.fill_(-1)
    g = L.RdoGraph(ts, tp, gfr, qp, rdmult, 10)
    torch.cuda.synchronize()
    dfr0 = L.RdoFrame(ts)
    L.rdo_frame(ts, tp, dfr0, qp, rdmult, 10)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gfr.recon.cpu().numpy(), dfr0.recon.cpu().numpy())
    for it in range(3):
        if it:
            tp.copy_(torch.roll(tp, shifts=(it, 2 * it), dims=(0, 1)))
        g.launch()
        dfr = L.RdoFrame(ts)
        L.rdo_frame(ts, tp, dfr, qp, rdmult, 10)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(gfr.recon.cpu().numpy(), dfr.recon.cpu().numpy())
        np.testing.assert_array_equal(gfr.sb_tx_size.cpu().numpy(), dfr.sb_tx_size.cpu().numpy())
        for s in gfr.sizes:
            for k in ("records", "qcoeff"):
                np.testing.assert_array_equal(gfr.outs[s][k].cpu().numpy(),
                                              dfr.outs[s][k].cpu().numpy(), err_msg=str((it, s)))


def test_pixel_1080p_7refs_all_jobs(L):
    """bench.py --workload pixel: aom_sad16x16x4d + aom_variance16x16 of every
    16x16 block x 7 refs at the seeded candidates, against orc_pixel_batch."""
    import torch
    import lavish_dsp.pixel as P
    b = _bench()
    src, refs, st, jobs = b.pixel_setup(1920, 1080, 7, 160, 1234)
    tsrc = torch.from_numpy(src).cuda()
    trefs = torch.from_numpy(refs.reshape(-1, st)).cuda()
    tj = P.jobs_tensor(jobs, "cuda")
    sad = P.sad_batch(tsrc, trefs, 16, 16, tj, nrefs=4).cpu().numpy()
    vb = P.variance_batch(tsrc, trefs, 16, 16, tj, kind=0)
    esad, evar, esse = O.pixel_batch(src.reshape(-1), st, refs.reshape(-1), st, 16, 16, jobs,
                                     threads=THREADS)
    np.testing.assert_array_equal(sad, esad)
    np.testing.assert_array_equal(vb["var"].cpu().numpy(), evar)
    np.testing.assert_array_equal(vb["sse"].cpu().numpy(), esse)


def test_warp_1080p_7refs_all_blocks(L):
    """bench.py --workload warp: av1_warp_affine of every 16x16 block x 7 refs
    with its own local model, against orc_warp_batch."""
    import torch
    import lavish_dsp.warp as Wp
    b = _bench()
    W, H = 1920, 1080
    refs, jobs = b.warp_setup(W, H, 7, 1234)
    tref = torch.from_numpy(refs.reshape(-1, W)).cuda()
    pred = torch.zeros_like(tref)
    Wp.warp_affine_batch(tref, W, H, W, pred, W, torch.from_numpy(jobs.view(np.uint8)).cuda(),
                         len(jobs), Wp.conv_params(3, 11), 8)
    exp = np.zeros_like(refs)
    O.warp_batch(refs.reshape(-1, W), W, H, W, exp.reshape(-1, W), W, jobs,
                 dict(do_average=0, round_0=3, round_1=11, is_compound=0,
                      use_dist_wtd_comp_avg=0, fwd_offset=0, bck_offset=0), threads=THREADS)
    np.testing.assert_array_equal(pred.cpu().numpy(), exp.reshape(-1, W))
