#!/usr/bin/env python3
"""bench.py -- MI355X throughput of the per-block RDO hot path.

One step = one 1920x1080 luma residual plane (synthetic, seeded; SURVEY.md
section 8(d) config C2) pushed through the batched forward transform +
quantize_fp of every TX size <= 32x32 and every valid TX type (9 sizes x 16
types + 5 sizes x 2 types): the work search_tx_type's per-type loop does for
a frame (av1/encoder/tx_search.c:2148-2312).  A 1080p frame is 30 x 17 = 510
64x64 superblocks; value = superblocks processed per second by the whole job.

Multi-GPU: one process per GPU (torchrun), each rank processes its own frame
(independent units, no data-path collective): weak scaling.  Timing: barrier +
device sync on both sides of exactly `--steps` steps, max over ranks.

Extra fields: `roofline` for the dominant kernel (algorithmic bytes / average
launch duration, from HIP events on the launch stream) and `cpu_baseline`
(the oracle's C restatement on the host cores, rank 0 at N=1, bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))

METRIC = "superblocks/s (fwd_txfm+quant+SAD RDO inner loop), 1080p cpu-used=6, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--qindex", type=int, default=128)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def sb64_count(w, h):
    return ((w + 63) // 64) * ((h + 63) // 64)


def algorithmic_bytes(L, s, width, height):
    """Bytes one launch must move: the residual once, then per
    (block, type) qcoeff + dqcoeff (8 B/coefficient) + a 2-byte eob."""
    W, H = L.TX_W[s], L.TX_H[s]
    nb = (width // W) * (height // H)
    nt = bin(L.valid_type_mask(s)).count("1")
    n = L.max_eob(s)
    return nb * (2 * W * H + nt * (8 * n + 2))


def cpu_baseline(args):
    """The oracle's C restatement (oracle/liboracle.so, -O3, pthreads) on a
    bounded sample: 4 superblock rows of the same synthetic frame, repeated
    until ~cpu_seconds of wall time; reported as SB64/s."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    import lavish_dsp as L
    import lavish_dsp.synth as synth
    threads = min(16, os.cpu_count() or 1)
    res = synth.residual_plane(args.width, 256, 8)
    q = O.build_quant(8, args.qindex)
    sizes = [s for s in range(19) if L.TX_W[s] <= 32 and L.TX_H[s] <= 32]
    sb = sb64_count(args.width, 256)
    passes = 0
    t0 = time.perf_counter()
    while True:
        for s in sizes:
            O.txq_plane(res, s, L.valid_type_mask(s), q, threads=threads)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    return {"value": round(passes * sb / dt, 2), "unit": "SB64/s", "cores": threads,
            "kind": "port",
            "sample": "%d passes of a %dx256 strip (%d SB64), all 14 sizes <=32 x valid types, "
                      "quantize_fp q%d, oracle C restatement (-O3, %d pthreads), %.1f s"
                      % (passes, args.width, sb, args.qindex, threads, dt)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import lavish_dsp as L
    import lavish_dsp.synth as synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    W, H = args.width, args.height
    res = torch.from_numpy(synth.residual_plane(W, H, 8, seed=1234 + rank)).cuda()
    sizes = [s for s in range(19) if L.TX_W[s] <= 32 and L.TX_H[s] <= 32]
    qp = L.build_quant_params(8, args.qindex, L.QUANT_FP)
    frame = L.FrameOutputs(res, sizes)
    stream = torch.cuda.current_stream()

    def step():
        L.txq_frame(res, frame, qp, stream=stream)

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

    # The dominant (indeed the only) launch of a step is the frame batch
    # lavish_txq_frame: 14 per-size kernels forked over 3 streams and joined
    # back; its duration is timed with HIP events on the caller stream.
    frame_ms = sum(ev[k][0].elapsed_time(ev[k][1]) for k in range(args.steps)) / args.steps
    step_bytes = sum(algorithmic_bytes(L, s, W, H) for s in sizes)
    achieved = step_bytes / (frame_ms * 1e-3) / 1e9

    # informational: per-size kernel durations, serialized, outside the timed region
    kev = {s: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for s in sizes}
    kern_ms = {s: 0.0 for s in sizes}
    for _ in range(3):
        for s in sizes:
            kev[s][0].record(stream)
            L.txq_plane(res, s, frame.type_masks[s], qp, out=frame.outs[s], stream=stream)
            kev[s][1].record(stream)
        torch.cuda.synchronize()
        for s in sizes:
            kern_ms[s] += kev[s][0].elapsed_time(kev[s][1]) / 3

    traffic = None
    kname = "lavish_txq_frame"
    if os.path.exists(args.pmc_json):
        try:
            pmc = json.load(open(args.pmc_json))
            traffic = pmc.get("frame_hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    sb = sb64_count(W, H)
    value = world * sb * args.steps / elapsed
    line = {
        "metric": METRIC,
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
        "data": "synthetic (seeded 1080p luma residual, lavish_dsp/synth.py)",
        "config": {
            "workload": "C2: %dx%d 8-bit residual, fwd_txfm2d + quantize_fp (qindex %d) of "
                        "all 14 TX sizes <=32x32 x every valid TX type per step "
                        "(lavish_txq_frame); %d SB64/frame"
                        % (W, H, args.qindex, sb),
            "tx_sizes": [L.TX_SIZES[s] for s in sizes],
            "parallelism": "frame-per-rank x%d" % world,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kname + " (14 txq_plane_kernel<W,H> over 3 streams)",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "avg_launch_ms": round(frame_ms, 4),
            "algorithmic_bytes_per_launch": step_bytes,
        },
        "kernel_ms_serialized": {L.TX_SIZES[s]: round(kern_ms[s], 4) for s in sizes},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
