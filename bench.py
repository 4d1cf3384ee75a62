#!/usr/bin/env python3
"""bench.py -- MI355X throughput of the per-block RDO hot path.

One step = one pass of the RDO inner loop over a synthetic, seeded 1080p
frame; a 1080p frame is 30 x 17 = 510 64x64
superblocks and value = superblocks processed per second by the whole job.
The default workload ("rdo") is the metric's "fwd_txfm+quant+SAD" loop:

  C2  the 1920x1080 luma residual through the batched forward transform +
      quantize_fp of every TX size <= 32x32 and every valid TX type (9 sizes
      x 16 types + 5 sizes x 2 types): search_tx_type's per-type loop
      (av1/encoder/tx_search.c:2148-2312) for the frame (lavish_txq_frame);
  C3  DIAMOND full-pixel motion search of every 16x16 block against 7
      reference frames (av1_full_pixel_search, av1/encoder/mcomp.c:1755),
      as the RDO path runs it at 1080p speed 6: use_downsampled_sad,
      MV_COST_ENTROPY over the default-context nmv cost tables with
      sadperbit / errorperbit of the qindex / rdmult, and the cost list the
      sub-pel search consumes (lavish_full_pixel_search_batch),

by default side by side: the legs are independent (the residual is given),
so C3 runs on a second stream beside C2 -- C3 is bound by the vector-memory
address path, C2 by HBM writes -- which shortens the step ~10 % (measured
0.967 -> 0.872 ms).  The per-kernel roofline and legs_ms come from a serial
pass after the timed region (isolated legs); legs_overlapped_ms keeps the
stretched spans of the timed region.  --serial times the legs back to back
on one stream; --workload c2 / c3 times one leg alone.

Multi-GPU: one process per GPU (torchrun), each rank processes its own frame
(independent units, no data-path collective): weak scaling.  Timing: barrier +
device sync on both sides of exactly `--steps` steps, max over ranks.

Extra fields: `roofline` for the dominant kernel (algorithmic bytes / average
launch duration, from HIP events on the launch stream) and `cpu_baseline`
(the oracle's C restatement on the host cores, rank 0 at N=1, bounded sample).
"""
import argparse
import ctypes
import json

import numpy as np
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))

METRIC = "superblocks/s (fwd_txfm+quant+SAD RDO inner loop), 1080p cpu-used=6, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# int32 VALU peak: 256 CUs x 2 wave64 instructions / cycle (a wave issues a
# VALU op over 2 cycles, 4 SIMDs) x 64 lanes x 2.4 GHz (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 256 * 2 * 64 * 2.4e9 / 1e12
C4_VALU_JSON = os.path.join(ROOT, "profiles", "c4_valu.json")


def metric_name(args):
    """BASELINE.json's metric for the default (headline) workload; the other
    workloads name themselves so their lines are never read as the headline."""
    if args.workload == "rdo":
        return METRIC
    return "superblocks/s, workload %s (component bench; not the headline metric)" % args.workload


def _hw_queues(v):
    """--hw-queues: 0 (the runtime's default) or 1..32 -- the HIP runtime
    refuses GPU_MAX_HW_QUEUES above 32 only once the run has started."""
    n = int(v)
    if n != 0 and not 1 <= n <= 32:
        raise argparse.ArgumentTypeError("--hw-queues must be 0 or within 1..32, got %d" % n)
    return n


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks; without a launcher (no WORLD_SIZE) bench.py starts them itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="with --gpus N > 1 and no launcher: print the ranks' plan, start nothing")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("rdo", "c2", "c3", "c3sub", "c4", "c4px", "c5", "inter",
                                           "tpl", "rate", "pixel", "warp", "compound", "scale", "mesh"),
                    default="rdo")
    ap.add_argument("--rdmult", type=int, default=2000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--qindex", type=int, default=128)
    ap.add_argument("--refs", type=int, default=7)
    ap.add_argument("--border", type=int, default=160)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--c5-no-graphs", action="store_true",
                    help="c5: launch each rectangle's step directly instead of replaying its "
                         "captured HIP graph")
    ap.add_argument("--c5-chunks", type=int, default=1,
                    help="c5 wavefront: column chunks per SB row (1: each row one step, "
                         "the rows a chain on one stream; 4 chunks measured 24-25 ms per 4K "
                         "frame in round 4 against 6.3-6.8 for 1)")
    ap.add_argument("--c5-form", choices=("tiles", "band", "wavefront"), default="tiles",
                    help="C5 sharding: balanced band + tail segments with overlapped "
                         "all-gathers, or the row-wavefront with p2p edges (lavish_dsp/shard.py)")
    ap.add_argument("--c5-emulate", default="",
                    help="c5 at world 1: also time every rank's partition() rectangles for "
                         "these world sizes (comma list, e.g. 2,4,8) one rank at a time on this "
                         "GPU -- the compute-only per-rank time at G ranks")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the c4 sub-object (4K 10-bit RDO step) of the default line")
    ap.add_argument("--c3-wg-cap", type=int, default=C3_WG_CAP,
                    help="workgroups of the C3 search when it runs beside C2 (0: no cap)")
    ap.add_argument("--c3-static", action="store_true",
                    help="the capped C3 search strides statically over virtual workgroups "
                         "instead of pulling its wave units from per-XCD queues (A/B)")
    ap.add_argument("--c3-mode", choices=("fused", "streams", "split32"), default=C3_MODE,
                    help="how C3 runs beside C2: one launch with the search's job groups "
                         "interleaved among C2's workgroups (lavish_txq_frame_search), C3 on a "
                         "second stream in at most --c3-wg-cap workgroups (streams), or that "
                         "with C2's 32-point sizes after C3 on the second stream (split32)")
    ap.add_argument("--c3-every", type=int, default=C3_EVERY,
                    help="fused: a search unit (8 workgroups) every this many units of the "
                         "dispatch order")
    ap.add_argument("--c2-priority", type=int, default=0,
                    help="1: the C2 leg on a high-priority stream beside C3")
    ap.add_argument("--serial", action="store_true",
                    help="run the C3 and C2 legs back to back on one stream (default: C3 on a "
                         "second stream beside C2)")
    ap.add_argument("--overlap", action="store_true", help=argparse.SUPPRESS)  # the default
    ap.add_argument("--hw-queues", type=_hw_queues, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts; "
                         "0: the runtime's default)")
    ap.add_argument("--fan-width", type=int, default=0,
                    help="1: C4's per-size kernels all on the caller's stream (isolated "
                         "per-kernel timings under a profiler; lavish_set_fan_width)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def host_cores():
    """CPUs this process may actually run on: the affinity set, capped by a
    cgroup v2 CPU quota when one is set (a GPU box grants each job a share
    of the host; os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def sb64_count(w, h):
    return ((w + 63) // 64) * ((h + 63) // 64)


def algorithmic_bytes(L, s, width, height):
    """C2 bytes one launch must move: the residual once, then
    per (block, type) qcoeff + dqcoeff (8 B/coefficient) + a 2-byte eob."""
    W, H = L.TX_W[s], L.TX_H[s]
    nb = (width // W) * (height // H)
    nt = bin(L.valid_type_mask(s)).count("1")
    n = L.max_eob(s)
    return nb * (2 * W * H + nt * (8 * n + 2))


def c3_algorithmic_bytes(res, njobs, bw, bh, skip, cost_list=False):
    """C3 bytes: per (block, ref) the source block once,
    8 candidate blocks per executed diamond step (the x4d contract; skip rows
    halve it), the source + reference block for every var cost, 16 B out;
    with a cost list the 5 SADs of calc_int_sad_list and 20 B more out."""
    rows = bh // 2 if skip and bh >= 16 else bh
    steps = int(res["steps"].astype("int64").sum())
    searches = int(res["searches"].astype("int64").sum())
    cl = njobs * (5 * rows * bw + 20) if cost_list else 0
    return njobs * (bw * bh + 16) + steps * 8 * rows * bw + searches * 2 * bw * bh + cl


C3_BLOCK = 16
C3_COST = 0     # MV_COST_ENTROPY (the RDO path's x->mv_cost_type)
C3_SKIP = True  # use_downsampled_sad (>= 720p, speed_features.c:205-209)
C3_CL = True    # cost list: subpel_search_method != SUBPEL_TREE (cond_cost_list)
C3_WG_CAP = 384  # C3's workgroups beside C2 (1.5 per CU; the queue-fed search: profiles/r06_c3_cap_sweep.txt)
# C3 on a second stream beside C2, C2's 32-point class after C3 on that
# stream (0.717-0.720 vs 0.727-0.729 ms with the whole of C2 on the caller's
# stream, profiles/r05_split32_ab.txt; fused: measured slower, DESIGN.md
# section 5)
C3_MODE = "split32"
C3_EVERY = 10      # fused: a search unit every 10 units of the dispatch order
# sub-pixel refinement after the full-pel search (c3sub): SUBPEL_TREE_PRUNED_MORE
# (speed >= 4), subpel_force_stop EIGHTH_PEL, iters_per_step 1 (speed >= 2),
# allow_high_precision_mv = qindex < HIGH_PRECISION_MV_QTHRESH (128)
SUB_FORCED_STOP = 0
SUB_ITERS = 1


def cpu_baseline(args):
    """The oracle's C restatement (oracle/liboracle.so, -O3, pthreads) on a
    bounded sample: a 4-superblock-row strip (1920x256) of the same synthetic
    content through the same step, repeated until ~cpu_seconds of wall time;
    reported as SB64/s."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    import lavish_dsp as L
    import lavish_dsp.motion as M
    import lavish_dsp.synth as synth
    threads = host_cores()
    W, Hs = args.width, 256
    do_c2 = args.workload in ("rdo", "c2")
    do_c3 = args.workload in ("rdo", "c3", "c3sub")
    do_sub = args.workload == "c3sub"
    res = synth.residual_plane(W, Hs, 8)
    q = O.build_quant(8, args.qindex)
    sizes = [s for s in range(19) if L.TX_W[s] <= 32 and L.TX_H[s] <= 32]
    src, refs = synth.motion_planes(W, Hs, args.refs, args.border)
    st = src.shape[1]
    jobs = M.frame_jobs(W, Hs, st, args.border, src.size, C3_BLOCK, C3_BLOCK, args.refs)
    allow_hp = args.qindex < 128
    mvj, mvc = M.default_mv_cost_tables(allow_hp)
    spb, epb = M.sad_per_bit(args.qindex), M.error_per_bit(args.rdmult)
    sb = sb64_count(W, Hs)
    passes = 0
    t0 = time.perf_counter()
    while True:
        if do_c2:
            for s in sizes:
                O.txq_plane(res, s, L.valid_type_mask(s), q, threads=threads)
        if do_c3:
            fp, cl = O.full_pixel_search_batch(
                src.reshape(-1), refs.reshape(-1), st, C3_BLOCK, C3_BLOCK, jobs, "diamond", 0,
                C3_COST, spb, epb, mvj, mvc, skip=C3_SKIP, cost_list=C3_CL, threads=threads)
        if do_sub:
            sj = M.subpel_jobs(W, Hs, args.border, C3_BLOCK, C3_BLOCK, jobs, fp)
            O.subpel_search_batch(src.reshape(-1), refs.reshape(-1), st, C3_BLOCK, C3_BLOCK, sj,
                                  2, SUB_FORCED_STOP, allow_hp, SUB_ITERS, C3_COST, epb, mvj,
                                  mvc, cl, threads=threads)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(passes * sb / dt, 2), "unit": "SB64/s", "cores": threads,
            "kind": "port",
            "sample": "%d passes of a %dx%d strip (%d SB64) through the %s step, oracle C "
                      "restatement (-O3, %d pthreads), %.1f s"
                      % (passes, W, Hs, sb, args.workload, threads, dt)}


def c4_algorithmic_bytes(L, W, H, coded=None):
    """C4 bytes per frame (decision mode): per candidate size
    src + pred read once (2 x 2 B / pixel), the winner's qcoeff + dqcoeff
    (8 B / coefficient) and a 40 B decision record per block, the decision's
    read of each record's 8 B cost; then the reconstruction reads pred and
    writes recon (4 B / pixel) and reads the dqcoeff of the chosen coded
    blocks (`coded`: per size, per type counts, c4_coded_blocks; without it
    every chosen block, <= 4 B / pixel)."""
    tot = 0
    for s in L.C4_TYPE_MASKS:
        nb = (W // L.TX_W[s]) * (H // L.TX_H[s])
        tot += 4 * W * H + nb * (8 * L.max_eob(s) + 40 + 8)
        if coded is not None:
            tot += 4 * L.max_eob(s) * int(np.sum(coded.get(s, 0)))
    return tot + (4 if coded is not None else 8) * W * H


def cpu_baseline_c4(args):
    """Oracle C4 (oracle/oracle_rdo.c + the per-SB choice + oracle inverse
    transforms, tests/_c4ref.py) on a 3840x128 strip (2 SB rows) of the same
    content, repeated for ~cpu_seconds."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _c4ref
    import lavish_dsp as L
    threads = host_cores()
    W = args.width if args.width != 1920 else 3840
    src, pred = _c4ref.planes(10, 1234, Wp=W, Hp=128)
    sb = sb64_count(W, 128)
    passes = 0
    t0 = time.perf_counter()
    px = args.workload == "c4px"
    while True:
        _c4ref.oracle_frame_c(src, pred, 10, dict(L.C4_TYPE_MASKS), args.rdmult, threads=threads,
                              px=px)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(passes * sb / dt, 2), "unit": "SB64/s", "cores": threads,
            "kind": "port",
            "sample": "%d passes of a %dx128 10-bit strip (%d SB64) through the %s step (RDO of "
                      "all candidate sizes/types, per-SB TX size, reconstruction), oracle C "
                      "restatement (-O3, %d pthreads), %.1f s"
                      % (passes, W, sb, args.workload, threads, dt)}


C4_OPS_JSON = os.path.join(ROOT, "profiles", "c4_ops.json")


def c4_coded_blocks(L, fr):
    """Per (size, type): the blocks the per-SB decision chose with eob > 0 --
    the ones the reconstruction inverse-transforms (idct.c:308: eob 0 adds
    nothing).  Read back after the timed region."""
    sb = fr.sb_tx_size.cpu().numpy()
    H, W = fr.recon.shape
    sbw = (W + 63) // 64
    out = {}
    for s in fr.sizes:
        w, h = L.TX_W[s], L.TX_H[s]
        rec = fr.outs[s]["records"].cpu().numpy().view(L.RDO_DTYPE)
        bw, bh = W // w, H // h
        if bw * bh == 0:
            continue
        by, bx = np.divmod(np.arange(bw * bh), bw)
        chosen = sb[(by * h // 64) * sbw + bx * w // 64] == s
        coded = chosen & (rec["eob"] != 0)
        out[s] = np.bincount(rec["best_type"][coded], minlength=16)
    return out


def c4_algorithmic_ops(W, H, masks, coded):
    """Algorithmic int32 ops of the C4 step ("C4
    algorithmic ops"), from profiles/c4_ops.json (tools/c4_ops.py: the
    reference's 1-D bodies executed with a counting integer).  Per candidate
    size s (w x h, n stored coefficients) and block:
      subtract w h + sum over the mask's vertical kinds of fwd_col[v]
      + sum over the mask's types t of (fwd_row[h(t)] + 41 n + 17) + 3
    (41 per coefficient: quantize_fp 21, satd 2, block error 9,
    rate_estimator 9; 17 per (block, type): distortion shift, RDCOST, select;
    3: the per-SB sum), then per chosen coded block of type t:
      inv_row[h(t)] + inv_col[v(t)]."""
    c = json.load(open(C4_OPS_JSON))
    vtx, htx = c["vtx"], c["htx"]
    pc = sum(c["per_coefficient"].values())
    pbt = c["per_block_type"]["dist_shift_rdcost_select"]
    total = 0
    for s, mask in masks.items():
        z = c["sizes"][str(s)]
        nb = (W // z["W"]) * (H // z["H"])
        types = [t for t in range(16) if (mask >> t) & 1]
        per = z["W"] * z["H"] + c["per_block_decide"]
        per += sum(z["fwd_col"][str(v)] for v in sorted({vtx[t] for t in types}))
        per += sum(z["fwd_row"][str(htx[t])] + pc * z["n"] + pbt for t in types)
        total += nb * per
        for t, k in enumerate(coded.get(s, [])):
            if k:
                total += int(k) * (z["inv_row"][str(htx[t])] + z["inv_col"][str(vtx[t])])
    return total


def c4_roofline(ms, W, H, masks, coded, nbytes):
    """C4 is VALU-bound (decision mode writes little), so its roofline is
    int32 VALU lane-operations: `frac` = the algorithmic op count
    (c4_algorithmic_ops) over the live event-timed step against the VALU
    peak; `issue_frac` = the issued SQ_INSTS_VALU x 64 lanes of a rocprofv3
    --pmc pass (profiles/c4_valu.json, tools/valu_summary.py) over the same
    time; `traffic_over_algorithmic` = that pass's HBM bytes (FETCH_SIZE x2 +
    WRITE_SIZE) over the algorithmic bytes."""
    if not os.path.exists(C4_OPS_JSON):
        return None
    ops = c4_algorithmic_ops(W, H, masks, coded)
    achieved = ops / (ms * 1e-3) / 1e12
    roof = {"bound": "valu", "kernel": "all kernels of the C4 step (rdo_kernel x5 sizes + "
            "sb_decide + reconstruction)", "achieved": round(achieved, 2),
            "peak": round(VALU_PEAK_TOPS, 1), "unit": "Tops (int32 lane-ops)",
            "frac": round(achieved / VALU_PEAK_TOPS, 4), "traffic": None,
            "avg_launch_ms": round(ms, 4), "algorithmic_ops_per_launch": ops,
            "ops": "algorithmic (DESIGN.md section 5; profiles/c4_ops.json)"}
    if (W, H) == (3840, 2160) and os.path.exists(C4_VALU_JSON):
        try:
            v = json.load(open(C4_VALU_JSON))
        except (ValueError, OSError):
            v = None
        stale = c4_counts_stale(v) if v is not None else "unreadable"
        if stale:
            # the counts describe other code: report the
            # algorithmic fraction only, and say why the counted ones are gone
            roof["counts_stale"] = stale
            v = None
        if v is not None:
            issued = float(v["valu_instr_per_step"]) * 64
            roof["issue_frac"] = round(issued / (ms * 1e-3) / 1e12 / VALU_PEAK_TOPS, 4)
            roof["issued_ops_per_launch"] = round(issued)
            roof["traffic"] = v.get("hbm_bytes_per_step")
            if roof["traffic"]:
                roof["traffic_over_algorithmic"] = round(roof["traffic"] / nbytes, 3)
            roof["counts"] = "profiles/c4_valu.json (round %s: %s)" % (v.get("round"),
                                                                      v.get("source", ""))
    return roof


def c4_counts_stale(v):
    """Why profiles/c4_valu.json no longer describes the library's C4 kernels
    (None when it does): every counted kernel must still exist with the
    resource signature (VGPR / SGPR / spills / LDS / scratch from the
    code-object metadata, tools/kernel_resources.py) it had when counted."""
    sig = v.get("kernels") or {}
    if "round" not in v or not sig or any("signature" not in k for k in sig.values()):
        return "no per-kernel signatures (written before round 6)"
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import kernel_resources as KR
        res = KR.kernel_resources(os.path.join(ROOT, "aom-av1-lavish_amd", "liblavish_hip.so"))
        names = sorted(res)
        now = {}
        for n, d in zip(names, KR.demangled(names)):
            k = (d or n).replace("void ", "").replace("lavish::(anonymous namespace)::", "")
            now[k.split("(")[0]] = res[n]
    except Exception as e:  # no llvm tools: cannot vouch for the counts
        return "signature check unavailable (%s)" % type(e).__name__
    for k, rec in sig.items():
        if now.get(k) != rec["signature"]:
            return "kernel %s changed since the counts (round %s)" % (k, v.get("round"))
    return None


def c4_leg(L, steps, warmup, rdmult, qindex, W=3840, H=2160):
    """The C4 step (4K 10-bit RDO of every candidate size / type + per-SB TX
    size + reconstruction, bench.py --workload c4) timed with HIP events on
    the current stream; returned as the default line's `c4` sub-object."""
    import torch
    import lavish_dsp.synth as synth
    src_np = synth.frame(W, H, 10, 1234).astype(np.uint16)
    pred_np = synth.shifted(synth.frame(W, H, 10, 1235), 3, -2).astype(np.uint16)
    src = torch.from_numpy(src_np.view(np.int16)).cuda()
    pred = torch.from_numpy(pred_np.view(np.int16)).cuda()
    qp = L.build_quant_params(10, qindex, L.QUANT_FP)
    fr = L.RdoFrame(src)
    stream = torch.cuda.current_stream()
    for _ in range(warmup):
        L.rdo_frame(src, pred, fr, qp, rdmult, 10)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for k in range(steps):
        ev[k][0].record(stream)
        L.rdo_frame(src, pred, fr, qp, rdmult, 10)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    coded = c4_coded_blocks(L, fr)
    nbytes = c4_algorithmic_bytes(L, W, H, coded)
    sb = sb64_count(W, H)
    roof = c4_roofline(ms, W, H, fr.type_masks, coded, nbytes)
    return roof, {"workload": "c4: %dx%d 10-bit frame; fused TX-type RDO (subtract, fwd txfm, highbd "
                        "quantize_fp, satd, TX-domain block error, rate_estimator, RDCOST) of "
                        "64x64 DCT, 32x32 DCT+IDTX, 16x16/8x8/4x4 all types; per-SB TX size; "
                        "reconstruction; rdmult %d, qindex %d" % (W, H, rdmult, qindex),
            "ms_per_frame": round(ms, 4), "SB64_per_s": round(sb / (ms * 1e-3), 1),
            "steps": steps, "algorithmic_bytes": nbytes,
            "achieved_GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
            "hbm_frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def c5_leg(L, steps, warmup, rdmult, qindex, world, rank, W=3840, H=2160, graphs=True,
           c4_ms=None, form="tiles"):
    """C5 (BASELINE configs[4]) inside the default line at N > 1: the C4 step
    of ONE 4K 10-bit frame sharded over the ranks (lavish_dsp/shard.py) --
    tiles: one grid tile of R C / G SBs per rank, one all-gather of the
    tiles over RCCL; band: floor(R / G) SB rows per rank + a column segment
    of the leftover rows, each part all-gathered as soon as it is computed
    -- timed barrier to barrier, max over ranks; plus each rank's compute
    alone (its rectangles, no exchange) and the all-gathers alone (the same
    tensors, no compute), so the line shows where the time goes."""
    import torch
    import torch.distributed as dist
    import lavish_dsp.shard as shard
    import lavish_dsp.synth as synth
    src_np = synth.frame(W, H, 10, 1234).astype(np.uint16)
    pred_np = synth.shifted(synth.frame(W, H, 10, 1235), 3, -2).astype(np.uint16)
    src = torch.from_numpy(src_np.view(np.int16)).cuda()
    pred = torch.from_numpy(pred_np.view(np.int16)).cuda()
    qp = L.build_quant_params(10, qindex, L.QUANT_FP)
    frames = {}
    frame_out = torch.empty_like(src)
    proc = shard.c4_rect_processor(src, pred, qp, rdmult, 10, frames, out=frame_out,
                                   graphs=graphs)
    if form == "tiles":
        parts = [(r,) for r in shard.grid_partition(H, W, world)]
    else:
        parts = shard.partition(H, W, world)
    mine = [r for r in parts[rank] if r is not None]

    def timed(fn, n):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        mx = torch.tensor([el], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        return el / n * 1e3, float(mx.item()) / n * 1e3

    streams = [torch.cuda.Stream(), torch.cuda.Stream()] if graphs else None

    def frame_step():
        if form == "tiles":
            shard.tiled_frame(H, W, rank, world, proc)
        else:
            shard.sharded_frame(H, W, rank, world, proc, streams=streams)

    caller = torch.cuda.current_stream()

    def compute_only():  # the rank's band and tail side by side, as in frame_step
        if streams is None or len(mine) == 1:
            for r in mine:
                proc(*r)
            return
        ev = torch.cuda.Event()
        ev.record(caller)
        for st, r in zip(streams, mine):
            st.wait_event(ev)
            with torch.cuda.stream(st):
                proc(*r)
        for st in streams:
            caller.wait_stream(st)

    # the exchange alone: each phase's all-gather of equal zero-padded parts
    gathers = []
    for phase in range(len(parts[0])):
        rects = [p[phase] for p in parts]
        if all(r is None for r in rects):
            continue
        hmax = max(r[1] - r[0] for r in rects if r is not None)
        wmax = max(r[3] - r[2] for r in rects if r is not None)
        snd = torch.zeros((hmax, wmax), dtype=torch.int16, device="cuda")
        rcv = torch.empty((world * hmax, wmax), dtype=torch.int16, device="cuda")
        gathers.append((snd, rcv))
    gather_bytes = sum(r.numel() * 2 for _, r in gathers)

    def gather_only():
        for snd, rcv in gathers:
            if world > 1:
                dist.all_gather_into_tensor(rcv.view(torch.uint8), snd.view(torch.uint8))
            else:
                rcv.copy_(snd.repeat(world, 1))

    for _ in range(warmup):
        frame_step()
        compute_only()
        gather_only()
    mine_ms, step_ms = timed(frame_step, steps)
    comp_ms, comp_max = timed(compute_only, steps)
    gath_ms, gath_max = timed(gather_only, steps)
    per_rank = [None] * world
    if world > 1:
        t = torch.zeros(world, dtype=torch.float64, device="cuda")
        t[rank] = comp_ms
        dist.all_reduce(t)
        per_rank = [round(float(x), 4) for x in t.cpu()]
    else:
        per_rank = [round(comp_ms, 4)]
    sb = sb64_count(W, H)
    how = ("tile form: one grid tile of whole SBs per rank, the tiles' reconstruction "
           "all-gathered over RCCL" if form == "tiles" else
           "band form: floor(R/G) SB rows + a column segment of the leftover rows per rank; "
           "each part's reconstruction all-gathered over RCCL")
    out = {"workload": "c5: one %dx%d 10-bit frame per step, the C4 step sharded over %d ranks "
                       "(%s)" % (W, H, world, how), "form": form,
           "n_ranks": world, "ms_per_frame": round(step_ms, 4),
           "SB64_per_s": round(sb / (step_ms * 1e-3), 1),
           "rank_rects": [list(p) for p in parts],
           "compute_ms_per_rank": per_rank, "compute_ms_max": round(comp_max, 4),
           "allgather_bytes": gather_bytes, "allgather_ms": round(gath_max, 4),
           "allgather_GBps": round(gather_bytes / (gath_max * 1e-3) / 1e9, 1) if gath_max else None,
           "graphs": graphs, "steps": steps}
    if c4_ms:
        # whole-frame C4 on one GPU (the c4 leg of the same line) over N x this
        out["strong_scaling_efficiency_vs_c4_leg"] = round(c4_ms / (world * step_ms), 4)
    return out


def c5_emulate(H, W, proc, worlds, steps, warmup, frame_ms, form="tiles"):
    """On one GPU, rank g's share of the C5 form for each world size G --
    tiles: its one grid_partition() tile; band: its partition() rectangles
    (band and tail segment side by side on two streams, as sharded_frame
    runs them) -- replayed as captured graphs with nothing else on the
    device, timed with HIP events: the compute-only time of that rank at G
    GPUs (no exchange, no contention from other ranks: each rank owns its
    GPU).  Reports every rank's time, the slowest, and the compute-only
    speed-up frame_ms / slowest."""
    import torch
    import lavish_dsp.shard as shard
    stream = torch.cuda.current_stream()
    side = [torch.cuda.Stream(), torch.cuda.Stream()]
    out = {}

    def rank_step(rects):  # band and tail side by side (shard.sharded_frame's streams)
        if len(rects) == 1:
            proc(*rects[0])
            return
        ev = torch.cuda.Event()
        ev.record(stream)
        for st, r in zip(side, rects):
            st.wait_event(ev)
            with torch.cuda.stream(st):
                proc(*r)
        for st in side:
            stream.wait_stream(st)

    for G in worlds:
        if form == "tiles":
            parts = [(r,) for r in shard.grid_partition(H, W, G)]
        else:
            parts = shard.partition(H, W, G)
        per, enq = [], []
        for g in range(G):
            rects = [r for r in parts[g] if r is not None]
            for _ in range(warmup):
                rank_step(rects)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(steps)]
            t0 = time.perf_counter()
            for a, b in ev:
                a.record(stream)
                rank_step(rects)
                b.record(stream)
            enq.append((time.perf_counter() - t0) / steps * 1e3)
            torch.cuda.synchronize()
            per.append(sum(a.elapsed_time(b) for a, b in ev) / steps)
        slow = max(per)
        out[str(G)] = {"form": form, "rank_ms": [round(x, 4) for x in per],
                       "max_rank_ms": round(slow, 4),
                       "host_enqueue_ms": round(max(enq), 4),
                       "projected_speedup_compute_only": round(frame_ms / slow, 3),
                       "rects": [list(p) for p in parts]}
    return out


def main_c4(args):
    """C4 (1 GPU) / C5 (SB rows sharded over the ranks, reconstructed rows
    all-gathered over RCCL) on a 4K 10-bit frame."""
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.shard as shard
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    W = args.width if args.width != 1920 else 3840
    H = args.height if args.height != 1080 else 2160
    import lavish_dsp.synth as synth
    src_np = synth.frame(W, H, 10, 1234).astype(np.uint16)
    pred_np = synth.shifted(synth.frame(W, H, 10, 1235), 3, -2).astype(np.uint16)
    src = torch.from_numpy(src_np.view(np.int16)).cuda()
    pred = torch.from_numpy(pred_np.view(np.int16)).cuda()
    qp = L.build_quant_params(10, args.qindex, L.QUANT_FP)
    stream = torch.cuda.current_stream()
    frames = {}
    if args.workload == "c5":
        # every rectangle reconstructs straight into its view of one frame plane
        frame_out = torch.empty_like(src)
        proc = shard.c4_rect_processor(src, pred, qp, args.rdmult, 10, frames, out=frame_out,
                                       graphs=not args.c5_no_graphs)
        if args.c5_form == "wavefront":
            # edges and row gathers on separate communicators (shard.py)
            p2p = dist.new_group(list(range(world))) if world > 1 else None

            # one GPU: the rows over 4 streams with event dependencies
            wstreams = [torch.cuda.Stream() for _ in range(4)] \
                if world == 1 and not args.c5_no_graphs else None

            def step():
                return shard.wavefront_frame(H, W, rank, world, proc, chunks=args.c5_chunks,
                                             p2p_group=p2p, out=frame_out, streams=wstreams)
            if wstreams is not None:
                # the chunks' graphs captured first, on one stream (no capture
                # interleaved with replays on the row streams)
                shard.wavefront_frame(H, W, rank, world, proc, chunks=args.c5_chunks,
                                      p2p_group=p2p, out=frame_out)
                torch.cuda.synchronize()
        elif args.c5_form == "tiles":
            def step():
                return shard.tiled_frame(H, W, rank, world, proc)
        else:
            bstreams = None if args.c5_no_graphs else [torch.cuda.Stream(), torch.cuda.Stream()]

            def step():
                return shard.sharded_frame(H, W, rank, world, proc, streams=bstreams)
    else:
        fr = L.RdoFrame(src)

        px = args.workload == "c4px"

        def step():
            L.rdo_frame(src, pred, fr, qp, args.rdmult, 10, px=px)
            return fr.recon
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    t_enq = time.perf_counter() - t0  # host time to enqueue the steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    step_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    sb = sb64_count(W, H)
    value = sb * args.steps / elapsed  # one frame per step for the whole job
    coded = c4_coded_blocks(L, fr) if args.workload != "c5" else None
    c4_bytes = c4_algorithmic_bytes(L, W, H, coded)
    band, tail = shard.partition(H, W, world)[rank]
    tile = shard.grid_partition(H, W, world)[rank]
    line = {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(value, 2),
        "unit": "SB64/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.workload == "c5" else "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded 4K 10-bit content, lavish_dsp/synth.py)",
        "config": {
            "workload": "%s: %dx%d 10-bit frame per step; fused TX-type RDO (subtract, fwd "
                        "txfm, highbd quantize_fp, satd, %s, rate_estimator, RDCOST) of "
                        "64x64 DCT, 32x32 DCT+IDTX, 16x16/8x8/4x4 all types; per-SB TX size; "
                        "reconstruction%s; %d SB64/frame"
                        % (args.workload, W, H,
                           "pixel-domain distortion (inverse txfm + recon + sse per type)"
                           if args.workload == "c4px" else "TX-domain block error",
                           ("; SB rows sharded over ranks (%s form) + RCCL all-gather of "
                            "the reconstruction" % args.c5_form) if args.workload == "c5" else "",
                           sb),
            "parallelism": (("sb grid tiles x%d (rank %d: tile %s)" % (world, rank, tile))
                            if args.c5_form == "tiles" else
                            "sb-row %s x%d (rank %d: band %s, tail %s)"
                            % ("band+tail segments" if args.c5_form == "band"
                               else "round-robin rows, p2p edge wavefront", world, rank, band,
                               tail))
            if args.workload == "c5" else "frame-per-rank x%d" % world,
        },
        "roofline": {"bound": "hbm", "kernel": "rdo_kernel<W,H,%d> x5 sizes + reconstruction "
                     "(lavish_rdo_frame%s + lavish_rdo_reconstruct)"
                     % ((2, "_px") if args.workload == "c4px" else (1, "")),
                     "achieved": round(c4_bytes / (step_ms * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": None,
                     "avg_launch_ms": round(step_ms, 4),
                     "algorithmic_bytes_per_launch": c4_bytes},
    }
    line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBS, 4)
    if coded is not None:  # chosen blocks with eob > 0 per TX size (what the inverse runs on)
        line["coded_blocks"] = {"%dx%d" % (L.TX_W[s], L.TX_H[s]): int(v.sum())
                                for s, v in coded.items()}
        line["sb_tx_size"] = {"%dx%d" % (L.TX_W[s], L.TX_H[s]): int(n) for s, n in zip(
            *np.unique(fr.sb_tx_size.cpu().numpy(), return_counts=True)) if s < 19}
    if args.workload == "c5" and world == 1 and args.c5_emulate:
        line["c5_emulation"] = c5_emulate(H, W, proc, [int(g) for g in args.c5_emulate.replace(":", ",").split(",")],
                                          args.steps, args.warmup, step_ms,
                                          form="band" if args.c5_form == "band" else "tiles")
    if args.workload == "c4" and world == 1:
        # the bound that applies: int32 VALU
        rv = c4_roofline(step_ms, W, H, fr.type_masks, coded, c4_bytes)
        if rv is not None:
            line["hbm_roofline"] = line["roofline"]
            line["roofline"] = rv
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_c4(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


INTER_BORDER = 288  # AOM_BORDER_IN_PIXELS: the clamp window of init_subpel_params


def inter_setup(W, H, nrefs, seed):
    """Inter-prediction workload: nrefs bordered 8-bit references and one job
    per 16x16 block x reference with a seeded sub-pel mv (+-32 px) and a
    seeded dual-filter pair from {REGULAR, SMOOTH, SHARP}."""
    import lavish_dsp.inter as I
    import lavish_dsp.synth as synth
    _, refs = synth.motion_planes(W, H, nrefs, INTER_BORDER, seed=seed)
    plane = refs[0].size
    org = INTER_BORDER * refs.shape[2] + INTER_BORDER
    rng = np.random.default_rng(seed)
    jobs = []
    for k in range(nrefs):
        n = (W // C3_BLOCK) * (H // C3_BLOCK)
        j = I.plane_jobs(W, H, C3_BLOCK, C3_BLOCK, rng.integers(-256, 257, size=(n, 2)),
                         rng.integers(0, 3, size=(n, 2)), ref_off=k * plane)
        j["dst_off"] += k * W * H
        jobs.append(j)
    return refs, org, np.concatenate(jobs)


def inter_bytes(W, H, nrefs, njobs):
    """Algorithmic bytes of one step: every reference pixel read once and every
    prediction pixel written once (u8), plus the 32 B job records; the
    per-block source windows ((16 + 7)^2 per block) overlap and are L2 hits."""
    return nrefs * 2 * W * H + 32 * njobs


def cpu_baseline_inter(args):
    """orc_build_inter_pred_batch (one thread) on a 1920x256 strip of the same
    workload, repeated for ~cpu_seconds; SB64/s."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    W, Hs = args.width, 256
    refs, org, jobs = inter_setup(W, Hs, args.refs, 1234)
    flat = refs.reshape(refs.shape[0] * refs.shape[1], refs.shape[2])
    sb = sb64_count(W, Hs)
    passes = 0
    t0 = time.perf_counter()
    while True:
        O.build_inter_pred(flat, org, W, Hs, 0, 0, C3_BLOCK, C3_BLOCK, jobs,
                           (args.refs * Hs, W))
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(passes * sb / dt, 2), "unit": "SB64/s", "cores": 1, "kind": "port",
            "sample": "%d passes of a %dx%d strip (%d SB64, %d predictions) through the inter "
                      "step, oracle C restatement (-O3, 1 thread), %.1f s"
                      % (passes, W, Hs, sb, len(jobs), dt)}


def main_inter(args):
    """Single-reference inter prediction of every 16x16 block against every
    reference (lavish_build_inter_pred_batch), one 1080p frame per step."""
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.inter as I
    import lavish_dsp.motion as M
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    W, H = args.width, args.height
    refs, org, jobs_np = inter_setup(W, H, args.refs, 1234 + rank)
    tref = torch.from_numpy(refs.reshape(-1, refs.shape[2])).cuda()
    tjobs = M.to_device(jobs_np)
    dst = torch.empty((args.refs * H, W), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        I.build_inter_pred_batch(tref, org, W, H, C3_BLOCK, C3_BLOCK, tjobs, dst=dst,
                                 stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    t_enq = time.perf_counter() - t0  # host time to enqueue the steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    k_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    nbytes = inter_bytes(W, H, args.refs, len(jobs_np))
    traffic = None
    if os.path.exists(args.pmc_json) and (W, H, args.refs) == (1920, 1080, 7):
        try:
            traffic = json.load(open(args.pmc_json)).get("inter", {}).get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None
    sb = sb64_count(W, H)
    line = {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(world * sb * args.steps / elapsed, 2),
        "unit": "SB64/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded 1080p content, lavish_dsp/synth.py; seeded mvs / filters)",
        "config": {
            "workload": "inter: %dx%d 8-bit; single-reference inter prediction "
                        "(av1_enc_build_one_inter_predictor: border clamp, dual-filter 8-tap "
                        "REGULAR/SMOOTH/SHARP, x/y/2d sub-pel convolution) of every %dx%d block "
                        "x %d refs, %d predictions; %d SB64/frame"
                        % (W, H, C3_BLOCK, C3_BLOCK, args.refs, len(jobs_np), sb),
            "parallelism": "frame-per-rank x%d" % world,
        },
        "roofline": {"bound": "hbm", "kernel": "inter_kernel<u8,4,16,FAST> "
                     "(lavish_build_inter_pred_batch)",
                     "achieved": round(nbytes / (k_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "traffic": traffic, "avg_launch_ms": round(k_ms, 4),
                     "algorithmic_bytes_per_launch": nbytes},
    }
    line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBS, 4)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_inter(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


PIX_RADIUS = 16  # candidate offsets of the pixel workload: within +-16 px


def pixel_setup(W, H, nrefs, border, seed):
    """Pixel workload: the motion planes and one LavishPixJob per 16x16 block
    x reference: src = the block, ref_off[0..3] = four seeded candidate
    positions within +-PIX_RADIUS px in that reference (an x4d call)."""
    import lavish_dsp.pixel as P
    import lavish_dsp.synth as synth
    src, refs = synth.motion_planes(W, H, nrefs, border, seed=seed)
    st = src.shape[1]
    nbx, nby = W // C3_BLOCK, H // C3_BLOCK
    ys = np.repeat(np.arange(nby) * C3_BLOCK, nbx)
    xs = np.tile(np.arange(nbx) * C3_BLOCK, nby)
    org = (ys + border) * st + xs + border
    rng = np.random.default_rng(seed)
    jobs = np.zeros(nrefs * len(org), P.JOB_DTYPE)
    jobs["src_off"] = np.tile(org, nrefs)
    d = rng.integers(-PIX_RADIUS, PIX_RADIUS + 1, size=(len(jobs), 4, 2))
    plane = np.repeat(np.arange(nrefs) * refs[0].size, len(org))
    jobs["ref_off"] = (plane + np.tile(org, nrefs))[:, None] + d[..., 0] * st + d[..., 1]
    return src, refs, st, jobs


def pixel_bytes(njobs, bw=16, bh=16):
    """Algorithmic bytes of one step: per job the x4d SAD reads the source
    block and 4 candidate blocks (5 * w * h) and writes 16 B; the variance
    reads 2 * w * h and writes 8 B; 56 B job record read by each call."""
    return njobs * (5 * bw * bh + 16 + 2 * bw * bh + 8 + 2 * 56)


def cpu_baseline_pixel(args):
    """orc_pixel_batch (the oracle's orc_sad x 4 + orc_variance per job) on a
    1920x256 strip of the same workload on all host cores, ~cpu_seconds."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    W, Hs = args.width, 256
    src, refs, st, jobs = pixel_setup(W, Hs, args.refs, args.border, 1234)
    threads = host_cores()
    sb = sb64_count(W, Hs)
    passes = 0
    t0 = time.perf_counter()
    while True:
        O.pixel_batch(src.reshape(-1), st, refs.reshape(-1), st, C3_BLOCK, C3_BLOCK, jobs,
                      threads=threads)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(passes * sb / dt, 2), "unit": "SB64/s", "cores": threads,
            "kind": "port",
            "sample": "%d passes of a %dx%d strip (%d SB64, %d jobs) through the pixel step, "
                      "oracle C restatement (-O3, %d pthreads), %.1f s"
                      % (passes, W, Hs, sb, len(jobs), threads, dt)}


def main_pixel(args):
    """The pixel batch kernels on a 1080p frame: aom_sad16x16x4d of every
    16x16 block x reference at 4 seeded candidates (lavish_sad_batch, nrefs
    4) then aom_variance16x16 at candidate 0 (lavish_variance_batch)."""
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.pixel as P
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    W, H = args.width, args.height
    src, refs, st, jobs_np = pixel_setup(W, H, args.refs, args.border, 1234 + rank)
    tsrc = torch.from_numpy(src).cuda()
    trefs = torch.from_numpy(refs.reshape(-1, st)).cuda()  # the refs stacked, one stride
    tjobs = P.jobs_tensor(jobs_np, "cuda")
    nj = len(jobs_np)
    sad = torch.empty((nj, 4), dtype=torch.int32, device="cuda")
    var = torch.empty(nj, dtype=torch.int32, device="cuda")
    sse = torch.empty(nj, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    sp = ctypes.c_void_p(stream.cuda_stream)

    def step():  # the C ABI directly: no wrapper-side conversions in the timed region
        rc = P._lib.lavish_sad_batch(vp(tsrc), st, vp(trefs), st, C3_BLOCK, C3_BLOCK, vp(tjobs),
                                     nj, 4, 0, None, 0, vp(sad), sp)
        rc |= P._lib.lavish_variance_batch(vp(tsrc), st, vp(trefs), st, C3_BLOCK, C3_BLOCK,
                                           vp(tjobs), nj, 0, 8, 0, None, vp(var), vp(sse), None,
                                           None, sp)
        assert rc == 0

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    t_enq = time.perf_counter() - t0  # host time to enqueue the steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    k_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    nbytes = pixel_bytes(len(jobs_np))
    sb = sb64_count(W, H)
    line = {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(world * sb * args.steps / elapsed, 2),
        "unit": "SB64/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded 1080p content, lavish_dsp/synth.py; seeded candidates)",
        "config": {
            "workload": "pixel: %dx%d 8-bit; aom_sad16x16x4d (4 candidates within +-%d px) + "
                        "aom_variance16x16 of every 16x16 block x %d refs, %d jobs; %d SB64/frame"
                        % (W, H, PIX_RADIUS, args.refs, len(jobs_np), sb),
            "parallelism": "frame-per-rank x%d" % world,
        },
        "roofline": {"bound": "hbm", "kernel": "sad_u8_kernel + var_u8_kernel "
                     "(lavish_sad_batch + lavish_variance_batch)",
                     "achieved": round(nbytes / (k_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "traffic": None, "avg_launch_ms": round(k_ms, 4),
                     "algorithmic_bytes_per_launch": nbytes,
                     "note": "overlapping candidate blocks are L2 hits: algorithmic bytes "
                             "exceed the HBM bytes"},
    }
    line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBS, 4)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_pixel(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()



def warp_setup(W, H, nrefs, seed):
    """Warp workload: nrefs 8-bit references (the seeded motion planes without
    their border: the warp clamps to the plane) and one LavishWarpJob per
    16x16 block x reference: a seeded valid affine model (AFFINE or ROTZOOM,
    the reference test's parameter ranges) whose projection of the block
    centre lands within +-16 px of the block, and its av1_get_shear_params."""
    import lavish_dsp.synth as synth
    import lavish_dsp.warp as Wp
    border = 160
    _, refs = synth.motion_planes(W, H, nrefs, border, seed=seed)
    refs = np.ascontiguousarray(refs[:, border:border + H, border:border + W])
    rng = np.random.default_rng(seed)
    nbx, nby = W // C3_BLOCK, H // C3_BLOCK
    jobs = np.zeros(nrefs * nbx * nby, Wp.JOB_DTYPE)
    n = 0
    for k in range(nrefs):
        for by in range(nby):
            for bx in range(nbx):
                while True:
                    m = [0, 0, (1 << 16) + int(rng.integers(-3000, 3001)),
                         int(rng.integers(-3000, 3001)), 0, 0]
                    if rng.integers(0, 3) == 0:
                        m[4], m[5] = -m[3], m[2]
                    else:
                        m[4] = int(rng.integers(-3000, 3001))
                        m[5] = (1 << 16) + int(rng.integers(-3000, 3001))
                    cx, cy = bx * C3_BLOCK + 8, by * C3_BLOCK + 8
                    dx, dy = rng.integers(-16, 17, 2)
                    m[0] = int(((cx + dx) << 16) - (m[2] * cx + m[3] * cy))
                    m[1] = int(((cy + dy) << 16) - (m[4] * cx + m[5] * cy))
                    ok, prm = Wp.get_shear_params(m)
                    if ok:
                        break
                j = jobs[n]
                j["mat"] = m
                j["alpha"], j["beta"], j["gamma"], j["delta"] = prm
                j["p_col"], j["p_row"] = bx * C3_BLOCK, by * C3_BLOCK
                j["p_width"] = j["p_height"] = C3_BLOCK
                j["ref_off"] = k * W * H
                j["pred_off"] = k * W * H + by * C3_BLOCK * W + bx * C3_BLOCK
                n += 1
    return refs, jobs


def warp_bytes(njobs, bw=16, bh=16):
    """Algorithmic bytes of one step: per block the prediction written (w*h)
    and the reference samples it covers read once (w*h; the 15 x 15 windows
    of neighbouring 8x8 units overlap and are L2 hits), plus the 72 B job."""
    return njobs * (2 * bw * bh + 72)


def cpu_baseline_warp(args):
    """orc_warp_batch (the oracle's av1_warp_affine_c restatement) on a
    1920x256 strip of the same workload on all host cores, ~cpu_seconds."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    W, Hs = args.width, 256
    refs, jobs = warp_setup(W, Hs, args.refs, 1234)
    pred = np.zeros_like(refs)
    threads = host_cores()
    sb = sb64_count(W, Hs)
    cp = dict(do_average=0, round_0=3, round_1=11, is_compound=0, use_dist_wtd_comp_avg=0,
              fwd_offset=0, bck_offset=0)
    passes = 0
    t0 = time.perf_counter()
    while True:
        O.warp_batch(refs.reshape(-1, W), W, Hs, W, pred.reshape(-1, W), W, jobs, cp,
                     threads=threads)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(passes * sb / dt, 2), "unit": "SB64/s", "cores": threads,
            "kind": "port",
            "sample": "%d passes of a %dx%d strip (%d SB64, %d blocks) through the warp step, "
                      "oracle C restatement (-O3, %d pthreads), %.1f s"
                      % (passes, W, Hs, sb, len(jobs), threads, dt)}


SCALE_STEP = 1536      # 1/1024 pel per output pixel: a reference at 1.5x the frame's size
SCALE_BORDER = 32


def scale_setup(W, H, nrefs, seed):
    """Scaled-prediction workload (av1_convolve_2d_scale, the inter predictor
    of a reference of another resolution): nrefs 8-bit references at 1.5x
    the frame's size (3 W / 2 x 3 H / 2, SCALE_BORDER pixels of edge
    replication), one LavishScaleJob per 16x16 block x reference: the
    block's position scaled by 1.5 (x_step_qn = y_step_qn = 1536) plus a
    seeded motion of +-8 reference pixels at a seeded 1/1024-pel phase."""
    import lavish_dsp.scale as Sc
    import lavish_dsp.synth as synth
    Wr, Hr, b = W * 3 // 2, H * 3 // 2, SCALE_BORDER
    refs = np.stack([synth.pad_plane(synth.frame(Wr, Hr, 8, seed + k).astype(np.uint8), b)
                     for k in range(nrefs)])
    st = refs.shape[2]
    rng = np.random.default_rng(seed)
    nbx, nby = W // C3_BLOCK, H // C3_BLOCK
    ys = np.repeat(np.arange(nby) * C3_BLOCK, nbx)
    xs = np.tile(np.arange(nbx) * C3_BLOCK, nby)
    n = len(ys)
    jobs = np.zeros(nrefs * n, Sc.JOB_DTYPE)
    for k in range(nrefs):
        sl = slice(k * n, (k + 1) * n)
        qx = xs * SCALE_STEP + rng.integers(-8 * 1024, 8 * 1024, n)
        qy = ys * SCALE_STEP + rng.integers(-8 * 1024, 8 * 1024, n)
        qx = np.clip(qx, 0, None)
        qy = np.clip(qy, 0, None)
        jobs["src_off"][sl] = k * refs[0].size + ((qy >> 10) + b) * st + (qx >> 10) + b
        jobs["subpel_x_qn"][sl] = qx & 1023
        jobs["subpel_y_qn"][sl] = qy & 1023
        jobs["dst_off"][sl] = k * W * H + ys * W + xs
    jobs["x_step_qn"] = SCALE_STEP
    jobs["y_step_qn"] = SCALE_STEP
    return refs, st, jobs


def scale_bytes(W, H, nrefs, njobs, bw=16, bh=16):
    """Algorithmic bytes of one step: every reference plane read once (the
    blocks' source windows tile it; their 7-pixel tap margins overlap and are
    L2 hits), every prediction pixel written once, the 40-byte job records."""
    return nrefs * (W * 3 // 2) * (H * 3 // 2) + njobs * (bw * bh + 40)


SCALE_CP = dict(do_average=0, round_0=3, round_1=11, is_compound=0, use_dist_wtd_comp_avg=0,
                fwd_offset=0, bck_offset=0)


def cpu_baseline_scale(args):
    """orc_convolve_2d_scale_batch (the oracle's av1_convolve_2d_scale_c
    restatement) on a 1920x256 strip of the same workload, all host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    W, Hs = args.width, 256
    refs, st, jobs = scale_setup(W, Hs, args.refs, 1234)
    tab = compound_tables()
    dst = np.zeros(args.refs * W * Hs, np.uint8)
    threads = host_cores()
    sb = sb64_count(W, Hs)
    n = 0
    t0 = time.perf_counter()
    while True:
        O.convolve_2d_scale_batch(refs.reshape(-1), st, dst, W, None, 0, C3_BLOCK, C3_BLOCK, jobs,
                                  tab, tab, SCALE_CP, threads=threads)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(n * sb / dt, 2), "unit": "SB64/s", "cores": threads, "kind": "port",
            "sample": "%d passes of a %dx%d strip (%d SB64, %d blocks) through the scaled "
                      "prediction step, oracle C restatement (-O3, %d pthreads), %.1f s"
                      % (n, W, Hs, sb, len(jobs), threads, dt)}


def main_scale(args):
    """Scaled inter prediction (av1_convolve_2d_scale, single prediction,
    8-bit, EIGHTTAP_REGULAR) of every 16x16 block of a 1080p frame from
    every reference at 1.5x resolution (lavish_convolve_2d_scale_batch),
    one frame per step."""
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.scale as Sc
    from lavish_dsp.compound import filter_params
    from lavish_dsp.inter import ConvolveParams
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    W, H = args.width, args.height
    refs, st, jobs_np = scale_setup(W, H, args.refs, 1234 + rank)
    tref = torch.from_numpy(refs.reshape(-1)).cuda()
    pred = torch.empty(args.refs * W * H, dtype=torch.uint8, device="cuda")
    tjobs = torch.from_numpy(jobs_np.view(np.uint8)).cuda()
    fp, keep = filter_params(compound_tables())
    c = SCALE_CP
    cp = ConvolveParams(c["do_average"], None, 0, c["round_0"], c["round_1"], 0,
                        c["is_compound"], c["use_dist_wtd_comp_avg"], c["fwd_offset"],
                        c["bck_offset"])
    stream = torch.cuda.current_stream()

    def step():
        Sc.convolve_2d_scale_batch(tref, st, pred, W, None, 0, C3_BLOCK, C3_BLOCK, tjobs,
                                   len(jobs_np), fp, fp, cp, 8, stream=stream)

    line = _timed_line(args, step, stream, world, rank, W, H, dtype="u8",
                       data="synthetic (seeded 1080p frame, seeded 1.5x references, "
                            "lavish_dsp/synth.py; seeded motion and phases)",
                       workload="scale: %dx%d 8-bit; av1_convolve_2d_scale (single prediction, "
                                "EIGHTTAP_REGULAR, x / y step %d/1024) of every %dx%d block x "
                                "%d refs at 1.5x resolution, %d blocks"
                                % (W, H, SCALE_STEP, C3_BLOCK, C3_BLOCK, args.refs,
                                   len(jobs_np)),
                       kernel="scale_kernel<u8, 8, 8> (lavish_convolve_2d_scale_batch)",
                       nbytes=scale_bytes(W, H, args.refs, len(jobs_np)))
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_scale(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# the temporal filter's full-pel search (temporal_filter.c:113-160): NSTEP at
# av1_init_search_range(1920) = 0, MV_COST_L1_HDRES, run_mesh_search = 1,
# good_quality_mesh_patterns[min(speed 6, MAX_MESH_SPEED)] (speed_features.c:26-33,
# 2291-2298), mesh_search_mv_diff_threshold 4, no pruning; 16x16 blocks
# (TF_BLOCK_SIZE), cost list on
MESH_PATTERNS = [(64, 16), (24, 8), (12, 4), (7, 1)]


def mesh_candidates(patterns=MESH_PATTERNS):
    """Nominal mesh candidates per job (exhaustive_mesh_search, mcomp.c:1529-1601):
    per pass ((2 range) / interval + 1)^2 positions around its centre,
    unclamped (jobs near the frame edge clamp their ranges: an upper bound)."""
    return sum((2 * r // max(iv, 1) + 1) ** 2 for r, iv in patterns)


def mesh_setup(W, H, nrefs, seed):
    import lavish_dsp.motion as M
    import lavish_dsp.synth as synth
    border = 160
    src, refs = synth.motion_planes(W, H, nrefs, border, seed=seed)
    st = src.shape[1]
    jobs = M.frame_jobs(W, H, st, border, src.size, C3_BLOCK, C3_BLOCK, nrefs)
    return src, refs, st, jobs


def cpu_baseline_mesh(args):
    """The oracle's av1_full_pixel_search (NSTEP + the mesh refinement) on a
    1920x256 strip of the same workload, all host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    W, Hs = args.width, 256
    src, refs, st, jobs = mesh_setup(W, Hs, args.refs, 1234)
    om = O.OrcMeshParams(1, 0x7FFFFFFF, 0, 4, 0, 0)
    for i, (r, iv) in enumerate(MESH_PATTERNS):
        om.range[i], om.interval[i] = r, iv
    threads = host_cores()
    sb = sb64_count(W, Hs)
    n = 0
    t0 = time.perf_counter()
    while True:
        O.full_pixel_search_batch(src.reshape(-1), refs.reshape(-1), st, C3_BLOCK, C3_BLOCK, jobs,
                                  "nstep", 0, 3, 0, 0, skip=False, cost_list=True,
                                  threads=threads, mesh=om)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(n * sb / dt, 2), "unit": "SB64/s", "cores": threads, "kind": "port",
            "sample": "%d passes of a %dx%d strip (%d SB64, %d jobs) through NSTEP + the mesh "
                      "refinement, oracle C restatement (-O3, %d pthreads), %.1f s"
                      % (n, W, Hs, sb, len(jobs), threads, dt)}


def main_mesh(args):
    """The temporal filter's full-pel motion search (NSTEP, then the
    exhaustive mesh refinement on every job: run_mesh_search = 1) of every
    16x16 block of a 1080p frame against each reference
    (lavish_full_pixel_search_batch_mesh: the search kernel, then
    mesh_kernel), one frame per step."""
    import torch
    import torch.distributed as dist
    import lavish_dsp.motion as M
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    W, H = args.width, args.height
    src, refs, st, jobs_np = mesh_setup(W, H, args.refs, 1234 + rank)
    tsrc, trefs = torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda()
    tjobs = M.to_device(jobs_np)
    cp = M.l1_cost_params(M.MV_COST_L1_HDRES)
    mesh = M.MeshParams.make(MESH_PATTERNS, run_mesh_search=1)
    nj = len(jobs_np)
    out = torch.empty(nj * M.RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    cl = torch.empty((nj, 5), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        M.full_pixel_search_batch(tsrc, trefs, C3_BLOCK, C3_BLOCK, tjobs, cp, "nstep", 0, False,
                                  True, out=out, cost_lists=cl, stream=stream, mesh=mesh)

    cand = mesh_candidates()
    nbytes = nj * cand * C3_BLOCK * C3_BLOCK
    line = _timed_line(args, step, stream, world, rank, W, H, dtype="u8",
                       data="synthetic (seeded 1080p motion planes, lavish_dsp/synth.py)",
                       workload="mesh: %dx%d 8-bit; the temporal filter's av1_full_pixel_search "
                                "(NSTEP, step_param 0, MV_COST_L1_HDRES, run_mesh_search 1, mesh "
                                "patterns %s, cost list) of every %dx%d block x %d refs, %d jobs"
                                % (W, H, MESH_PATTERNS, C3_BLOCK, C3_BLOCK, args.refs, nj),
                       kernel="diamond_kernel<16,16,NSTEP> + mesh_kernel<16,16> "
                              "(lavish_full_pixel_search_batch_mesh)",
                       nbytes=nbytes)
    # the candidates' SAD reads overlap (neighbouring positions share rows):
    # L2-served, as C3's; no HBM bound is claimed for them
    r = line["roofline"]
    r["bound"] = "l2-served SAD reads (nominal)"
    r["note"] = ("algorithmic bytes = jobs x %d nominal mesh candidates (unclamped) x 256 B "
                 "of candidate rows read by the SADs; the NSTEP walk's own reads not counted; "
                 "frac against the HBM peak for scale only" % cand)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_mesh(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _timed_line(args, step, stream, world, rank, W, H, dtype, data, workload, kernel, nbytes):
    """The contract's line for a one-launch component workload: W warmup
    steps, K timed steps bracketed by barrier + synchronize, max over ranks;
    the roofline from HIP events on the launch's stream."""
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    k_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    sb = sb64_count(W, H)
    achieved = nbytes / (k_ms * 1e-3) / 1e9
    return {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(world * sb * args.steps / elapsed, 2), "unit": "SB64/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": data,
        "config": {"workload": workload + "; %d SB64/frame" % sb,
                   "parallelism": "frame-per-rank x%d" % world},
        "roofline": {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "avg_launch_ms": round(k_ms, 4), "algorithmic_bytes_per_launch": nbytes},
    }


def main_warp(args):
    """Affine warp prediction (av1_warp_affine_c, single prediction, 8-bit)
    of every 16x16 block of a 1080p frame against every reference with its
    own local model (lavish_warp_affine_batch), one frame per step."""
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.warp as Wp
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    W, H = args.width, args.height
    refs, jobs_np = warp_setup(W, H, args.refs, 1234 + rank)
    tref = torch.from_numpy(refs.reshape(-1, W)).cuda()
    pred = torch.empty_like(tref)
    tjobs = torch.from_numpy(jobs_np.view(np.uint8)).cuda()
    cp = Wp.conv_params(3, 11)
    stream = torch.cuda.current_stream()

    def step():
        Wp.warp_affine_batch(tref, W, H, W, pred, W, tjobs, len(jobs_np), cp, 8, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    t_enq = time.perf_counter() - t0  # host time to enqueue the steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    k_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    nbytes = warp_bytes(len(jobs_np))
    sb = sb64_count(W, H)
    line = {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(world * sb * args.steps / elapsed, 2),
        "unit": "SB64/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded 1080p content, lavish_dsp/synth.py; seeded affine models)",
        "config": {
            "workload": "warp: %dx%d 8-bit; av1_warp_affine (single prediction) of every %dx%d "
                        "block x %d refs with its own local affine model, %d blocks; "
                        "%d SB64/frame" % (W, H, C3_BLOCK, C3_BLOCK, args.refs, len(jobs_np), sb),
            "parallelism": "frame-per-rank x%d" % world,
        },
        "roofline": {"bound": "hbm", "kernel": "warp_kernel<u8> (lavish_warp_affine_batch)",
                     "achieved": round(nbytes / (k_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "traffic": None, "avg_launch_ms": round(k_ms, 4),
                     "algorithmic_bytes_per_launch": nbytes},
    }
    line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBS, 4)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_warp(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def compound_setup(W, H, nrefs, seed):
    """Compound workload: the 8-bit motion planes (no border kept: candidates
    stay >= 8 px inside) and, per 16x16 block, a pair of references (k, k+1
    mod nrefs for every k) with seeded integer + sub-pel motion (+-16 px,
    1/16 pel): pass 1 jobs read ref k into the CONV_BUF, pass 2 jobs read
    ref k+1 and average (distance-weighted) into the prediction."""
    import lavish_dsp.compound as Cm
    import lavish_dsp.synth as synth
    border = 160
    _, refs = synth.motion_planes(W, H, nrefs, border, seed=seed)
    st = refs.shape[2]
    rng = np.random.default_rng(seed)
    nbx, nby = W // C3_BLOCK, H // C3_BLOCK
    ys = np.repeat(np.arange(nby) * C3_BLOCK, nbx)
    xs = np.tile(np.arange(nbx) * C3_BLOCK, nby)
    n = len(ys)
    passes = []
    for p in range(2):
        jobs = np.zeros(nrefs * n, Cm.JOB_DTYPE)
        for k in range(nrefs):
            sl = slice(k * n, (k + 1) * n)
            r = (k + p) % nrefs
            d = rng.integers(-16, 17, (n, 2))
            jobs["src_off"][sl] = r * refs[0].size + (ys + border + d[:, 0]) * st + xs + border + d[:, 1]
            jobs["dst_off"][sl] = k * W * H + ys * W + xs
            jobs["conv_off"][sl] = k * W * H + ys * W + xs
        jobs["subpel_x_qn"] = rng.integers(0, 16, len(jobs))
        jobs["subpel_y_qn"] = rng.integers(0, 16, len(jobs))
        passes.append(jobs)
    return refs, st, passes


def compound_tables():
    """EIGHTTAP_REGULAR kernels for 16-wide blocks (av1/common/filter.h), from
    the library's own table (lavish_interp_kernels, pinned to the reference
    text by tests/test_capi_cpu.py)."""
    import lavish_dsp.inter as I
    return I.interp_kernels(I.EIGHTTAP_REGULAR, 16)


COMPOUND_CP = [dict(do_average=0, round_0=3, round_1=7, is_compound=1, use_dist_wtd_comp_avg=0,
                    fwd_offset=0, bck_offset=0),
               dict(do_average=1, round_0=3, round_1=7, is_compound=1, use_dist_wtd_comp_avg=1,
                    fwd_offset=9, bck_offset=7)]


def cpu_baseline_compound(args):
    """orc_dist_wtd_batch (the oracle's av1_dist_wtd_convolve_* restatement,
    both passes) on a 1920x256 strip of the same workload, all host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    W, Hs = args.width, 256
    refs, st, passes = compound_setup(W, Hs, args.refs, 1234)
    tab = compound_tables()
    dst = np.zeros(args.refs * W * Hs, np.uint8)
    conv = np.zeros(args.refs * W * Hs, np.uint16)
    threads = host_cores()
    sb = sb64_count(W, Hs)
    n = 0
    t0 = time.perf_counter()
    while True:
        for p in range(2):
            O.dist_wtd_batch(refs.reshape(-1), st, dst, W, conv, W, C3_BLOCK, C3_BLOCK,
                             passes[p], tab, tab, COMPOUND_CP[p], threads=threads)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(n * sb / dt, 2), "unit": "SB64/s", "cores": threads, "kind": "port",
            "sample": "%d passes of a %dx%d strip (%d SB64, 2 x %d blocks) through the compound "
                      "step, oracle C restatement (-O3, %d pthreads), %.1f s"
                      % (n, W, Hs, sb, len(passes[0]), threads, dt)}


def main_compound(args):
    """Compound inter prediction of every 16x16 block x reference pair of a
    1080p frame: lavish_dist_wtd_convolve_batch twice (first prediction into
    the CONV_BUF, then the distance-weighted average into the prediction)."""
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.compound as Cm
    from lavish_dsp.inter import ConvolveParams
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    W, H = args.width, args.height
    refs, st, passes = compound_setup(W, H, args.refs, 1234 + rank)
    tref = torch.from_numpy(refs.reshape(-1)).cuda()
    dst = torch.empty(args.refs * W * H, dtype=torch.uint8, device="cuda")
    conv = torch.empty(args.refs * W * H, dtype=torch.int16, device="cuda")
    tjobs = [torch.from_numpy(p.view(np.uint8)).cuda() for p in passes]
    fp, tab = Cm.filter_params(compound_tables())
    cps = [ConvolveParams(c["do_average"], None, 0, c["round_0"], c["round_1"], 0, 1,
                          c["use_dist_wtd_comp_avg"], c["fwd_offset"], c["bck_offset"])
           for c in COMPOUND_CP]
    stream = torch.cuda.current_stream()
    nj = len(passes[0])

    def step():
        for p in range(2):
            Cm.dist_wtd_convolve_batch(tref, st, dst, W, conv, W, C3_BLOCK, C3_BLOCK, tjobs[p], nj,
                                       fp, fp, cps[p], 8, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    t_enq = time.perf_counter() - t0  # host time to enqueue the steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    k_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    # per block and pass: the source window read once, the CONV_BUF written
    # (pass 1) or read + the prediction written (pass 2), the 32 B job
    nbytes = nj * (2 * 256 + 2 * 512 + 512 + 256 + 2 * 32)
    sb = sb64_count(W, H)
    line = {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(world * sb * args.steps / elapsed, 2),
        "unit": "SB64/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded 1080p content, lavish_dsp/synth.py; seeded mvs)",
        "config": {
            "workload": "compound: %dx%d 8-bit; av1_dist_wtd_convolve (facade path per block, "
                        "EIGHTTAP_REGULAR) of every %dx%d block x %d reference pairs: first "
                        "prediction into the CONV_BUF, distance-weighted average into the "
                        "prediction; %d SB64/frame" % (W, H, C3_BLOCK, C3_BLOCK, args.refs, sb),
            "parallelism": "frame-per-rank x%d" % world,
        },
        "roofline": {"bound": "hbm", "kernel": "compound_kernel<u8> x 2 "
                     "(lavish_dist_wtd_convolve_batch)",
                     "achieved": round(nbytes / (k_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "traffic": None, "avg_launch_ms": round(k_ms / 2, 4),
                     "algorithmic_bytes_per_launch": nbytes // 2},
    }
    line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBS, 4)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_compound(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()

TPL_BORDER = 288  # AOM_BORDER_IN_PIXELS: the predictor's clamp reads stay inside


def tpl_block_bytes(W, H, nrefs, bs=16):
    """TPL block-leg bytes per frame (lavish_tpl_block_batch): the source and
    every reference's prediction read once (u8), the reconstruction written,
    a 32-byte record and nrefs int32 costs per block."""
    nb = (W // bs) * (H // bs)
    return W * H * (nrefs + 2) + nb * (32 + 4 * nrefs)


def cpu_baseline_tpl(args):
    """The oracle chain (start-mv full-pel, sub-pel, prediction, block leg) on
    a 1920x256 strip with the bench's parameters, repeated for ~cpu_seconds
    (the start-mv walk uses one thread per reference, the rest all cores)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    import lavish_dsp.inter as I
    import lavish_dsp.motion as M
    import lavish_dsp.synth as synth
    threads = host_cores()
    W, Hs, R, border = args.width, 256, args.refs, TPL_BORDER
    src, refs = synth.tpl_motion_planes(W, Hs, R, border, seed=1234)
    st = src.shape[1]
    jobs = M.frame_jobs(W, Hs, st, border, src.size, 16, 16, R, mv_border=32)
    allow_hp = args.qindex < 128
    mvj, mvc = M.default_mv_cost_tables(allow_hp)
    spb, epb = M.sad_per_bit(args.qindex), M.error_per_bit(args.rdmult)
    ij = np.concatenate([I.plane_jobs(W, Hs, 16, 16, (0, 0), ref_off=k * src.size, dst_stride=W)
                         for k in range(R)])
    n1 = len(ij) // R
    for k in range(R):
        ij["dst_off"][k * n1:(k + 1) * n1] += k * W * Hs
    org = border * st + border
    sb = sb64_count(W, Hs)
    passes = 0
    t0 = time.perf_counter()
    while True:
        # the start-mv walk is sequential per reference: one thread each
        _, fp, cl, _ = O.tpl_motion_search(src.reshape(-1), refs.reshape(-1), st, jobs, W // 16,
                                           Hs // 16, R, "fast_bigdia", 6, False, 3, 2, spb, epb,
                                           mvj, mvc, 0)
        sj = M.subpel_jobs(W, Hs, 32, 16, 16, jobs, fp)
        sub = O.subpel_search_batch(src.reshape(-1), refs.reshape(-1), st, 16, 16, sj, 2,
                                    M.FULL_PEL, allow_hp, 1, M.MV_COST_NONE, 0, None, None, cl,
                                    threads=threads)
        preds = O.build_inter_pred(refs.reshape(-1, st), org, W, Hs, 0, 0, 16, 16, ij,
                                   (R, Hs, W), mvs=sub, dst_stride=W)
        O.tpl_block_batch(src[border:border + Hs, border:border + W], preds, 16, 8, args.qindex,
                          threads=threads)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(passes * sb / dt, 2), "unit": "SB64/s", "cores": threads,
            "kind": "port",
            "sample": "%d passes of a %dx%d strip (%d SB64) through the tpl step (full-pel, "
                      "sub-pel, prediction, block leg), oracle C restatement (-O3, %d pthreads), "
                      "%.1f s" % (passes, W, Hs, sb, threads, dt)}


def main_tpl(args):
    """The TPL model's inter leg for one 1080p frame per step (TplFrame.step:
    FAST_BIGDIA full-pel with entropy costs and cost lists, sub-pel stop at
    full pel with MV_COST_NONE, EIGHTTAP_REGULAR predictions, then the block
    leg: per-reference satd, best reference, quantize error, rate, recon) --
    the cpu-used=6 tpl speed features (speed_features.c:1101,1213-1216)."""
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.motion as M
    import lavish_dsp.synth as synth
    import lavish_dsp.tpl as T
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    W, H, R = args.width, args.height, args.refs
    src, refs = synth.tpl_motion_planes(W, H, R, TPL_BORDER, seed=1234 + rank)
    tf = T.TplFrame(src, refs, W, H, TPL_BORDER, args.qindex, args.rdmult)
    stream = torch.cuda.current_stream()
    bs = T.TPL_BSIZE

    def step(ev=None):
        mark = (lambda i: ev[i].record(stream)) if ev is not None else (lambda i: None)
        mark(0)
        # mode_estimation's start mvs + FAST_BIGDIA: the device wavefront
        T.tpl_motion_search(tf.src, tf.refs, tf.jobs, tf.cols, tf.rows, tf.nrefs, tf.cost,
                            tf.search_method, tf.step_param, tf.skip_sad, tf.prune, tf.alike,
                            out=tf.mv_out, stream=stream)
        mark(1)
        M.find_best_sub_pixel_tree_batch(tf.src, tf.refs, bs, bs, tf.sub_jobs, tf.cost_none,
                                         tf.subpel_method, tf.forced_stop, tf.allow_hp, 1,
                                         fullpel=tf.fp, cost_lists=tf.cl, out=tf.sub,
                                         stream=stream)
        mark(2)
        import lavish_dsp.inter as I
        I.build_inter_pred_batch(tf.refs.view(-1, tf.stride), tf.org, W, H, bs, bs,
                                 tf.inter_jobs, dst=tf.preds.view(-1, W), dst_stride=W,
                                 bit_depth=8, mvs=tf.sub, stream=stream)
        mark(3)
        T.tpl_block_batch(tf.src_view, tf.preds, bs, 8, tf.qp, out=tf.out, recon=tf.recon,
                          ref_costs=tf.costs, stream=stream)
        mark(4)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(ev[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    K = args.steps
    legs = [sum(ev[k][i].elapsed_time(ev[k][i + 1]) for k in range(K)) / K for i in range(4)]
    names = ["fullpel_start_mv_wavefront", "subpel", "inter_pred", "tpl_block"]
    if T.tpl_motion_failures(tf.mv_out):
        raise RuntimeError("tpl motion wavefront: a wait timed out")
    blk_bytes = tpl_block_bytes(W, H, R)
    fp_res = M.results_numpy(tf.fp)
    # full-pel leg bytes: per job the source block, the var cost's 2 blocks,
    # 16 + 20 B out; every SAD block it read (results' `searches` field for
    # the pattern methods: start, in-range candidates, cost list)
    nj = len(fp_res)
    fp_bytes = nj * (3 * bs * bs + 36) + int(fp_res["searches"].astype(np.int64).sum()) * bs * bs
    sb = sb64_count(W, H)
    recs = T.records_numpy(tf.out)
    line = {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(world * sb * args.steps / elapsed, 2),
        "unit": "SB64/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded 1080p content, lavish_dsp/synth.py)",
        "config": {
            "workload": "tpl: %dx%d 8-bit frame per step; TPL inter leg of every 16x16 block x %d "
                        "refs: mode_estimation's start mvs (neighbour tpl mvs, is_alike_mv "
                        "skip_alike 2, prune_starting_mv 3: full-SAD ranking, one search) as a "
                        "device wavefront + FAST_BIGDIA full-pel (step_param 6, "
                        "MV_COST_ENTROPY default nmv context, ref_mv = the centre, cost list, mv "
                        "border 32) -> sub-pel forced stop FULL_PEL (MV_COST_NONE) -> "
                        "EIGHTTAP_REGULAR prediction -> tpl_get_satd_cost per ref, best ref, "
                        "get_quantize_error (quantize_fp qindex %d) + rate_estimator + recon; "
                        "%d SB64/frame" % (W, H, R, args.qindex, sb),
            "parallelism": "frame-per-rank x%d" % world,
        },
        "roofline": ({"bound": "hbm",
                      "kernel": "tpl_mv_kernel<true> (FAST_BIGDIA with the start-mv "
                                "candidates, lavish_tpl_motion_search wavefront; latency-bound: "
                                "%d dependent block steps)" % (tf.cols + 2 * (tf.rows - 1)),
                      "achieved": round(fp_bytes / (legs[0] * 1e-3) / 1e9, 1),
                      "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": None,
                      "avg_launch_ms": round(legs[0], 4),
                      "algorithmic_bytes_per_launch": fp_bytes}
                     if legs[0] >= legs[3] else
                     {"bound": "hbm", "kernel": "tpl_kernel<16,0,u8> (lavish_tpl_block_batch)",
                      "achieved": round(blk_bytes / (legs[3] * 1e-3) / 1e9, 1),
                      "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": None,
                      "avg_launch_ms": round(legs[3], 4),
                      "algorithmic_bytes_per_launch": blk_bytes}),
        "legs_ms": {n: round(v, 4) for n, v in zip(names, legs)},
        "tpl": {"blocks": int(len(recs)), "mean_eob": round(float(recs["eob"].mean()), 2),
                "refs_chosen": int(len(set(recs["best_ref"].tolist()))),
                "fullpel_sad_blocks_per_job": round(float(fp_res["searches"].mean()), 2),
                "wavefront": {"block_steps": tf.cols + 2 * (tf.rows - 1),
                              "us_per_block_step": round(legs[0] * 1e3 /
                                                         (tf.cols + 2 * (tf.rows - 1)), 3),
                              "jobs_started_off_zero": int(np.count_nonzero(
                                  tf.mv_out["centers"].cpu().numpy()))},
                "block_leg": {"ms": round(legs[3], 4), "algorithmic_bytes": blk_bytes,
                              "achieved_GBps": round(blk_bytes / (legs[3] * 1e-3) / 1e9, 1)}},
    }
    line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBS, 4)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_tpl(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rate_tables(seed=2024):
    """Seeded CoeffCosts cells in av1_fill_coeff_costs' magnitude and
    get_tx_type_cost per type (the timing does not depend on the values)."""
    from lavish_dsp import txb
    rng = np.random.default_rng(seed)
    return (rng.integers(30, 4000, txb.COEFF_COSTS_CELLS).astype(np.int32),
            rng.integers(0, 3000, 16).astype(np.int32))


def cpu_baseline_rate(args):
    """Oracle C4 ranked by the coefficient rate (orc_rdo_plane_rate for every
    candidate size / type) on a 3840x128 10-bit strip, ~cpu_seconds."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _c4ref
    import _oracle as O
    import lavish_dsp as L
    threads = host_cores()
    src, pred = _c4ref.planes(10, 1234, Wp=3840, Hp=128)
    blob, ttc = rate_tables()
    q = O.build_quant(10, args.qindex)
    sb = sb64_count(3840, 128)
    passes = 0
    t0 = time.perf_counter()
    while True:
        for s, m in L.C4_TYPE_MASKS.items():
            O.rdo_plane_rate(src, pred, s, m, 10, q, args.rdmult, blob, None, ttc,
                             threads=threads)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(passes * sb / dt, 2), "unit": "SB64/s", "cores": threads,
            "kind": "port",
            "sample": "%d passes of a 3840x128 10-bit strip (%d SB64) through the rate step "
                      "(RDO of all candidate sizes / types ranked by av1_cost_coeffs_txb), "
                      "oracle C restatement (-O3, %d pthreads), %.1f s"
                      % (passes, sb, threads, dt)}


def main_rate(args):
    """The coefficient rate on a 4K 10-bit frame.
    Step = C4's decision of every candidate size / type (the c4 type sets)
    ranked by av1_cost_coeffs_txb (lavish_rdo_plane_rate, rdo_kernel mode
    3), sizes back to back on the current stream.  Beside it, timed the same
    way: the same decision with rate_estimator (lavish_rdo_plane_masked,
    mode 1), and the standalone lavish_cost_coeffs_txb_batch over every
    block of each size's DCT_DCT quantization (lavish_txq_plane)."""
    import torch
    import lavish_dsp as L
    import lavish_dsp.synth as synth
    from lavish_dsp import txb
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    W = args.width if args.width != 1920 else 3840
    H = args.height if args.height != 1080 else 2160
    src_np = synth.frame(W, H, 10, 1234).astype(np.uint16)
    pred_np = synth.shifted(synth.frame(W, H, 10, 1235), 3, -2).astype(np.uint16)
    src = torch.from_numpy(src_np.view(np.int16)).cuda()
    pred = torch.from_numpy(pred_np.view(np.int16)).cuda()
    qp = L.build_quant_params(10, args.qindex, L.QUANT_FP)
    blob, ttc = rate_tables()
    costs = txb.CoeffCosts(blob)
    sizes = dict(L.C4_TYPE_MASKS)
    outs = {s: L.rdo_out(src, s) for s in sizes}
    stream = torch.cuda.current_stream()

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        t0 = time.perf_counter()
        for k in range(steps):
            ev[k][0].record(stream)
            fn()
            ev[k][1].record(stream)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, sum(a.elapsed_time(b) for a, b in ev) / steps

    def step_rate():
        for s, m in sizes.items():
            txb.rdo_plane_rate(src, pred, s, m, qp, args.rdmult, costs, None, ttc,
                               bit_depth=10, out=outs[s])

    def step_est():
        for s, m in sizes.items():
            L.rdo_plane_masked(src, pred, s, m, qp, args.rdmult, bit_depth=10, out=outs[s])

    elapsed, step_ms = timed(step_rate, args.steps, args.warmup)
    _, est_ms = timed(step_est, args.steps, args.warmup)
    # standalone coefficient rate over each size's DCT_DCT quantization
    res = (src.to(torch.int32) - pred.to(torch.int32)).to(torch.int16).contiguous()
    cc = {}
    for s in sizes:
        tq = L.txq_plane(res, s, 1, qp, bit_depth=10)
        qc, eob = tq["qcoeff"][0].contiguous(), tq["eob"][0].contiguous()
        rate = torch.empty(qc.shape[0], dtype=torch.int32, device="cuda")
        _, ms = timed(lambda: txb.cost_coeffs_txb_batch(costs, qc, eob, s, 0, out=rate),
                      args.steps, args.warmup)
        nb, n = qc.shape
        nbytes = nb * (4 * n + 2 + 4)  # qcoeff, eob in, rate out
        cc[L.TX_SIZES[s]] = {"blocks": nb, "ms": round(ms, 4), "algorithmic_bytes": nbytes,
                             "achieved_GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                             "mean_eob": round(float(eob.view(torch.uint16).float().mean()), 1)}
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    sb = sb64_count(W, H)
    nbytes = c4_algorithmic_bytes(L, W, H) - 8 * W * H  # no reconstruction in this step
    line = {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(sb * args.steps / elapsed, 2),
        "unit": "SB64/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded 4K 10-bit content, lavish_dsp/synth.py; seeded CoeffCosts)",
        "config": {
            "workload": "rate: %dx%d 10-bit frame per step; TX-type RDO (subtract, fwd txfm, "
                        "highbd quantize_fp, TX-domain block error, av1_cost_coeffs_txb rate, "
                        "RDCOST) of 64x64 DCT, 32x32 DCT+IDTX, 16x16/8x8/4x4 all types; "
                        "qindex %d, rdmult %d; %d SB64/frame" % (W, H, args.qindex,
                                                                args.rdmult, sb),
            "parallelism": "frame-per-rank x1"},
        "roofline": {"bound": "hbm", "kernel": "rdo_kernel<W,H,3> x5 sizes "
                     "(lavish_rdo_plane_rate)",
                     "achieved": round(nbytes / (step_ms * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": None,
                     "avg_launch_ms": round(step_ms, 4),
                     "algorithmic_bytes_per_launch": nbytes},
        "rate_estimator_ms": round(est_ms, 4),
        "cost_coeffs": cc,
    }
    line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBS, 4)
    if not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_rate(args)
    print(json.dumps(line), flush=True)


class RdoStep:
    """The default workload's step (C3 beside C2 on one 1080p frame): the
    device inputs, outputs and launches main() times, kept in one place so
    tests/test_gpu_bench_step.py runs exactly the timed configuration.

    workload: "rdo" (C2 + C3), "c2", "c3" or "c3sub" (C3 + the chained
    pruned_more sub-pel refinement).  serial: the legs back to back on the
    caller's stream; otherwise C3 runs on a side stream beside C2 in at most
    `c3_wg_cap` workgroups (0: uncapped; alone, C3 always runs uncapped)."""

    def __init__(self, workload="rdo", width=1920, height=1080, refs=7, border=160, qindex=128,
                 rdmult=2000, seed=1234, serial=False, c3_wg_cap=C3_WG_CAP, c3_mode=C3_MODE,
                 c3_every=C3_EVERY):
        import torch
        import lavish_dsp as L
        import lavish_dsp.motion as M
        import lavish_dsp.synth as synth
        self.L, self.M = L, M
        W, H = width, height
        self.do_c2 = workload in ("rdo", "c2")
        self.do_c3 = workload in ("rdo", "c3", "c3sub")
        self.do_sub = workload == "c3sub"
        self.overlap = self.do_c2 and self.do_c3 and not serial
        # fused: the overlapped step as one launch (C3 without the sub-pel leg)
        self.fused = self.overlap and c3_mode == "fused" and not self.do_sub
        self.split32 = c3_mode == "split32"
        self.c3_wg_cap = c3_wg_cap
        self.c3_every = c3_every
        self.stream = torch.cuda.current_stream()
        # C2 input: residual plane (each rank its own frame)
        self.res_np = synth.residual_plane(W, H, 8, seed=seed)
        self.res = torch.from_numpy(self.res_np).cuda()
        self.sizes = [s for s in range(19) if L.TX_W[s] <= 32 and L.TX_H[s] <= 32]
        self.qp = L.build_quant_params(8, qindex, L.QUANT_FP)
        self.frame = L.FrameOutputs(self.res, self.sizes)
        # the 32-point class of lavish_txq_frame (largest side 32)
        self.mask32 = sum(1 << s for s in self.sizes if max(L.TX_W[s], L.TX_H[s]) == 32)
        # C3 input: padded current frame + references, jobs for every 16x16
        # block x ref
        self.src_np, self.refs_np = synth.motion_planes(W, H, refs, border, seed=seed)
        st = self.src_np.shape[1]
        self.ref_stride = st
        self.jobs_np = M.frame_jobs(W, H, st, border, self.src_np.size, C3_BLOCK, C3_BLOCK, refs)
        self.tsrc = torch.from_numpy(self.src_np).cuda()
        self.trefs = torch.from_numpy(self.refs_np).cuda()
        self.tjobs = M.to_device(self.jobs_np)
        n = len(self.jobs_np)
        self.c3_out = torch.empty(n * M.RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        self.c3_cl = torch.empty((n, 5), dtype=torch.int32, device="cuda")
        self.allow_hp = qindex < 128
        self.mv_tables = M.default_mv_cost_tables(self.allow_hp)
        self.mv_costs = M.MvCosts(*self.mv_tables)
        self.sad_per_bit, self.error_per_bit = M.sad_per_bit(qindex), M.error_per_bit(rdmult)
        self.c3_cost = self.mv_costs.cost_params(self.sad_per_bit, self.error_per_bit, C3_COST)
        if self.do_sub:
            self.sub_jobs = M.to_device(M.subpel_jobs(W, H, border, C3_BLOCK, C3_BLOCK,
                                                      self.jobs_np,
                                                      np.zeros(n, M.RESULT_DTYPE)))
            self.sub_out = torch.empty(n * M.SUBPEL_RESULT_DTYPE.itemsize, dtype=torch.uint8,
                                       device="cuda")
        # the searches' candidate-row copy of the references (LavishRefTiles),
        # rebuilt inside every step: the frame's references are new per frame
        self.c3_tiles = M.RefTiles(self.trefs, st)
        self.side_stream = torch.cuda.Stream()
        self.fork = torch.cuda.Event()
        self.join = torch.cuda.Event()
        torch.cuda.synchronize()

    def c3(self, on):
        M = self.M
        self.c3_tiles.build(stream=on)
        M.full_pixel_search_batch(self.tsrc, self.trefs, C3_BLOCK, C3_BLOCK, self.tjobs,
                                  self.c3_cost, "diamond", 0, C3_SKIP, C3_CL, out=self.c3_out,
                                  cost_lists=self.c3_cl, stream=on, tiles=self.c3_tiles)
        if self.do_sub:  # chained on the device: starts + cost lists = the full-pel results
            M.find_best_sub_pixel_tree_batch(self.tsrc, self.trefs, C3_BLOCK, C3_BLOCK,
                                             self.sub_jobs, self.c3_cost, "pruned_more",
                                             SUB_FORCED_STOP, self.allow_hp, SUB_ITERS,
                                             fullpel=self.c3_out, cost_lists=self.c3_cl,
                                             out=self.sub_out, stream=on)

    def step(self, ev=None, ovl=None):
        """One frame.  ev = (start, c3 start, c3 end, c2 start, c2 end, end),
        each leg's pair recorded on the stream that leg runs on; ovl: run C3 on
        the side stream beside C2 (default: the run's mode)."""
        ovl = self.overlap if ovl is None else ovl
        stream = self.stream
        side = self.side_stream if ovl else stream
        if ev is not None:
            ev[0].record(stream)
        if ovl and self.fused:
            # the tiled references, then C2 + C3 as one grid (both legs' event
            # pairs bracket the whole launch)
            if ev is not None:
                ev[1].record(stream)
                ev[3].record(stream)
            self.c3_tiles.build(stream=stream)
            self.M.txq_frame_search(self.res, self.frame, self.qp, self.tsrc, self.trefs,
                                    self.tjobs, self.c3_cost, self.c3_tiles, self.c3_out,
                                    self.c3_cl, self.c3_every, use_downsampled_sad=C3_SKIP,
                                    stream=stream)
            if ev is not None:
                ev[2].record(stream)
                ev[4].record(stream)
                ev[5].record(stream)
            return
        # split32: C2's 32-point class (few, latency-bound workgroups) follows
        # C3 on the side stream, the <= 16-point class runs on the caller's
        split = ovl and self.split32 and self.do_c2
        if ovl:  # the legs are independent: C3 (TA / latency bound) beside C2 (HBM writes)
            self.fork.record(stream)
            side.wait_event(self.fork)
        if self.do_c3:
            if ev is not None:
                ev[1].record(side)
            # beside C2 the search runs in fewer workgroups (it holds fewer CU
            # slots and C2 stretches less: DESIGN.md section 5); alone, uncapped
            self.M.set_search_workgroup_cap(self.c3_wg_cap if ovl else 0)
            self.c3(side)
            if split:
                self.L.txq_frame(self.res, self.frame, self.qp, stream=side,
                                 size_mask=self.mask32)
            if ev is not None:
                ev[2].record(side)
        if self.do_c2:
            if ev is not None:
                ev[3].record(stream)
            self.L.txq_frame(self.res, self.frame, self.qp, stream=stream,
                             size_mask=~self.mask32 if split else None)
            if ev is not None:
                ev[4].record(stream)
        if ovl:
            self.join.record(side)
            stream.wait_event(self.join)
        if ev is not None:
            ev[5].record(stream)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def child_envs(n, port):
    """The environment of each of the n ranks `--gpus n` starts itself when no
    launcher set WORLD_SIZE: one process per GPU, torch.distributed's env://
    rendezvous on 127.0.0.1."""
    envs = []
    for r in range(n):
        e = dict(os.environ)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                  "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(port)})
        envs.append(e)
    return envs


def spawn_ranks(args, argv):
    """`bench.py --gpus N` without a launcher: start N fresh child processes
    (before this process touches the GPU; never an exec), each one rank with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, wait for all of them, print
    rank 0's JSON line and return non-zero if any rank failed.  --dry-run
    prints the plan (commands and rank environments) instead of starting."""
    import subprocess
    n = args.gpus
    envs = child_envs(n, free_port())
    cmd = [sys.executable, os.path.abspath(__file__)] + [a for a in argv if a != "--dry-run"]
    if args.dry_run:
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                "MASTER_PORT")
        print(json.dumps({"spawn": n, "cmd": cmd,
                          "ranks": [{k: e[k] for k in keys} for e in envs]}), flush=True)
        return 0
    procs = [subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else None)
             for r, e in enumerate(envs)]
    out0 = procs[0].communicate()[0].decode(errors="replace")
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    for ln in out0.splitlines():
        print(ln, flush=True)
    bad = [(r, rc) for r, rc in enumerate(rcs) if rc != 0]
    if bad:
        print("bench.py --gpus %d: ranks failed (rank, exit status): %s" % (n, bad),
              file=sys.stderr, flush=True)
        return 1
    return 0


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args, sys.argv[1:])
    if args.hw_queues:  # read by the HIP runtime when it starts (first device call)
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.fan_width:
        import lavish_dsp
        lavish_dsp.set_fan_width(args.fan_width)
    if args.workload in ("c4", "c4px", "c5"):
        return main_c4(args)
    if args.workload == "inter":
        return main_inter(args)
    if args.workload == "pixel":
        return main_pixel(args)
    if args.workload == "scale":
        return main_scale(args)
    if args.workload == "mesh":
        return main_mesh(args)
    if args.workload == "warp":
        return main_warp(args)
    if args.workload == "compound":
        return main_compound(args)
    if args.workload == "tpl":
        return main_tpl(args)
    if args.workload == "rate":
        return main_rate(args)
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.motion as M

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    W, H = args.width, args.height
    if args.c2_priority and args.workload == "rdo" and not args.serial:
        # C2 (the step's long leg) on a high-priority stream, C3 beside it on
        # a normal one: freed CU slots go to C2's workgroups first
        torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
    R = RdoStep(args.workload, W, H, args.refs, args.border, args.qindex, args.rdmult,
                seed=1234 + rank, serial=args.serial, c3_wg_cap=args.c3_wg_cap,
                c3_mode=args.c3_mode, c3_every=args.c3_every)
    if args.c3_static:
        R.M.set_search_schedule(False)
    do_c2, do_c3, do_sub, overlap = R.do_c2, R.do_c3, R.do_sub, R.overlap
    stream, sizes, jobs_np, c3_cost = R.stream, R.sizes, R.jobs_np, R.c3_cost
    step = R.step

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(6))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(ev[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    status = L.status()
    if status[0] != 0:
        raise RuntimeError("HIP error during bench: %s" % (status,))
    K = args.steps
    step_ms = sum(ev[k][0].elapsed_time(ev[k][5]) for k in range(K)) / K
    c3_ms = sum(ev[k][1].elapsed_time(ev[k][2]) for k in range(K)) / K if do_c3 else 0.0
    c2_ms = sum(ev[k][3].elapsed_time(ev[k][4]) for k in range(K)) / K if do_c2 else 0.0
    # the C3 results the timed region produced (its last step): the serial
    # pass below overwrites the output buffer
    c3_res = M.results_numpy(R.c3_out) if do_c3 else None
    legs_overlapped = None
    if overlap:
        # the legs share the GPU in the timed region, which stretches each; the
        # per-kernel roofline is taken from a serial pass after it (isolated
        # legs, same inputs), not from the overlapped leg spans
        legs_overlapped = ({"c2_c3_fused_launch": round(c2_ms, 4)} if R.fused else
                           {"c2_txq_frame_le16pt": round(c2_ms, 4),
                            "c3_diamond_then_c2_32pt": round(c3_ms, 4)} if R.split32 else
                           {"c2_txq_frame": round(c2_ms, 4), "c3_diamond": round(c3_ms, 4)})
        KS = max(5, K // 2)
        evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(6)) for _ in range(KS)]
        step(ovl=False)
        for k in range(KS):
            step(evs[k], ovl=False)
        torch.cuda.synchronize()
        c3_ms = sum(evs[k][1].elapsed_time(evs[k][2]) for k in range(KS)) / KS
        c2_ms = sum(evs[k][3].elapsed_time(evs[k][4]) for k in range(KS)) / KS
    c2_bytes = sum(algorithmic_bytes(L, s, W, H) for s in sizes)
    # + the tiled copy of the references: read once, written at 2x
    c3_bytes = c3_algorithmic_bytes(c3_res, len(jobs_np), C3_BLOCK, C3_BLOCK, C3_SKIP, C3_CL) \
        + R.trefs.numel() + R.c3_tiles.data.numel() if do_c3 else 0

    traffic = c3_hbm = traffic_src = None
    if os.path.exists(args.pmc_json):
        try:
            pj = json.load(open(args.pmc_json))
            traffic = pj.get("frame_hbm_bytes_per_launch")
            c3_hbm = pj.get("diamond_hbm_bytes_per_launch")
            traffic_src = "%s (round %s: %s)" % (os.path.relpath(args.pmc_json, ROOT),
                                                  pj.get("round"), pj.get("command", ""))
        except (ValueError, OSError):
            traffic = None

    # dominant kernel: the longer leg
    if do_c2 and (c2_ms >= c3_ms):
        roof = {"bound": "hbm",
                "kernel": "lavish_txq_frame (txq_multi_kernel<0> + <1>: one launch per VGPR class, 14 sizes)",
                "achieved": round(c2_bytes / (c2_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "traffic": traffic, "traffic_source": traffic_src,
                "avg_launch_ms": round(c2_ms, 4), "algorithmic_bytes_per_launch": c2_bytes}
    else:
        roof = {"bound": "hbm",
                "kernel": "ref_tiles_kernel + diamond_kernel<16,16,false,true> "
                          "(lavish_ref_tiles_build + lavish_full_pixel_search_batch_tiled)",
                "achieved": round(c3_bytes / (c3_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "traffic": None, "avg_launch_ms": round(c3_ms, 4),
                "algorithmic_bytes_per_launch": c3_bytes}
    roof["frac"] = round(roof["achieved"] / HBM_PEAK_GBS, 4)

    sb = sb64_count(W, H)
    value = world * sb * args.steps / elapsed
    legs = []
    if do_c2:
        legs.append("C2 fwd_txfm2d + quantize_fp (qindex %d) of all 14 TX sizes <=32x32 x every "
                    "valid TX type" % args.qindex)
    if do_c3:
        legs.append("C3 DIAMOND full-pel search of every %dx%d block x %d refs (downsampled SAD, "
                    "MV_COST_ENTROPY default nmv context, sadperbit %d, errorperbit %d, "
                    "cost list, step_param 0; candidate rows from the references' tiled copy, "
                    "rebuilt per step)" % (C3_BLOCK, C3_BLOCK, args.refs,
                                                  c3_cost.sad_per_bit, c3_cost.error_per_bit))
    if do_sub:
        legs.append("sub-pel refinement SUBPEL_TREE_PRUNED_MORE to %s pel (bilinear svf, "
                    "cost-list surface minimum, iters_per_step %d) chained on the device"
                    % ("1/8" if args.qindex < 128 else "1/4", SUB_ITERS))
    line = {
        "metric": metric_name(args), "workload": args.workload,
        "value": round(value, 2),
        "unit": "SB64/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded 1080p content, lavish_dsp/synth.py)",
        "config": {
            "workload": "%s: %dx%d 8-bit frame per step; %s; %d SB64/frame"
                        % (args.workload, W, H, " + ".join(legs), sb),
            "tx_sizes": [L.TX_SIZES[s] for s in sizes] if do_c2 else [],
            "parallelism": "frame-per-rank x%d" % world,
            "legs": (("C2 + C3 in one launch, a C3 unit of 8 workgroups every %d units "
                      "(lavish_txq_frame_search)" % args.c3_every) if R.fused else
                     ("C3 on a second stream beside C2 (C3 in at most %d workgroups)"
                      % args.c3_wg_cap if args.c3_wg_cap else
                      "C3 on a second stream beside C2")) if overlap else "C3 then C2, one stream",
        },
        "roofline": roof,
        "legs_ms": {"c2_txq_frame": round(c2_ms, 4), "c3_diamond": round(c3_ms, 4),
                    "step_event_ms": round(step_ms, 4),
                    "legs": "isolated (serial pass after the timed region)" if overlap
                            else "as timed"},
    }
    if legs_overlapped is not None:
        line["legs_overlapped_ms"] = legs_overlapped
    if do_c3:
        # the search's candidate re-reads are served by L2: its
        # algorithmic rate is not an HBM rate; the PMC bytes that reach HBM
        # (tiles + search + cost tables) stand beside it
        line["c3"] = {"jobs": len(jobs_np),
                      "steps_per_job": round(float(c3_res["steps"].mean()), 2),
                      "stats_from": "the timed region's last step",
                      "algorithmic_bytes": c3_bytes,
                      "algorithmic_GBps_L2_served": round(c3_bytes / (c3_ms * 1e-3) / 1e9, 1),
                      "hbm_bytes_pmc": c3_hbm,
                      "hbm_GBps_pmc": round(c3_hbm / (c3_ms * 1e-3) / 1e9, 1) if c3_hbm else None,
                      "leg_ms": round(c3_ms, 4)}
    if args.workload == "rdo" and not args.no_c4:
        # the 4K 10-bit RDO configuration (BASELINE configs[3]), timed after
        # the headline region so the driver's run records it too
        roof4, line["c4"] = c4_leg(L, max(5, args.steps // 2), max(2, args.warmup),
                                   args.rdmult, args.qindex)
        line["c4"]["roofline"] = roof4
        if rank == 0 and world == 1 and not args.no_cpu:
            a4 = argparse.Namespace(**vars(args))
            a4.workload = "c4"
            a4.cpu_seconds = max(3.0, args.cpu_seconds / 2)
            line["c4"]["cpu_baseline"] = cpu_baseline_c4(a4)
    if args.workload == "rdo" and world > 1 and not args.no_c4:
        # the SB-row shard of north_star over RCCL (BASELINE configs[4]): at
        # N > 1 the driver's scaling run measures it from this object
        line["c5"] = c5_leg(L, max(5, args.steps // 2), max(2, args.warmup), args.rdmult,
                            args.qindex, world, rank,
                            c4_ms=line.get("c4", {}).get("ms_per_frame"),
                            form="band" if args.c5_form == "band" else "tiles")
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
