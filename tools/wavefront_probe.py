#!/usr/bin/env python3
"""Where the one-GPU C5 row wavefront's time goes (bench.py --workload c5
--c5-form wavefront): host time per step call and device time per SB row of
the 4K 10-bit C4 step, for
  graph1   one row's captured step (lavish_rdo_graph) replayed N times on one stream
  direct1  the same row through lavish_rdo_frame + reconstruct (uncaptured)
  rows     the 34 rows' graphs back to back on one stream (no events)
  wave1    shard.wavefront_frame at one chunk per row (bench.py's form)
usage: wavefront_probe.py [variant,variant,...]
Prints one JSON line per variant: host_us per call, device ms total."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "aom-av1-lavish_amd"))


def main():
    import numpy as np
    import torch
    import lavish_dsp as L
    import lavish_dsp.synth as synth
    from lavish_dsp import shard
    W, H = 3840, 2160
    src = torch.from_numpy(synth.frame(W, H, 10, 1234).astype(np.uint16).view(np.int16)).cuda()
    pred = torch.from_numpy(synth.shifted(synth.frame(W, H, 10, 1235), 3, -2)
                            .astype(np.uint16).view(np.int16)).cuda()
    qp = L.build_quant_params(10, 128, L.QUANT_FP)
    out = torch.empty_like(src)
    frames = {}
    proc_g = shard.c4_rect_processor(src, pred, qp, 2000, 10, frames, out=out, graphs=True)
    R = shard.sb_rows(H)
    for r in range(R):  # capture every row's graph
        proc_g(r * 64, min(H, r * 64 + 64), 0, W)
    torch.cuda.synchronize()
    key = (64, 128, 0, W)
    fr = frames[key]

    def timed(name, fn, n):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn_n = n
        for _ in range(fn_n):
            fn()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tt = time.perf_counter() - t0
        print(json.dumps({"variant": name, "calls": n, "host_us_per_call": round(th / n * 1e6, 1),
                          "total_ms_per_call": round(tt / n * 1e3, 4)}), flush=True)

    want = set(sys.argv[1].split(",")) if len(sys.argv) > 1 else None

    def timed_if(name, fn, n):
        if want is None or name in want:
            timed(name, fn, n)
    timed_if("graph1", lambda: fr.graph.launch(), 100)
    s, p = src[64:128], pred[64:128]
    timed_if("direct1", lambda: L.rdo_frame(s, p, fr, qp, 2000, 10), 100)
    keys = [(r * 64, min(H, r * 64 + 64), 0, W) for r in range(R)]

    def rows():
        for k in keys:
            frames[k].graph.launch()
    timed_if("rows", rows, 10)
    streams = [torch.cuda.Stream() for _ in range(4)]

    def wave1():  # the wavefront form at one chunk per row (one stream, shard.py)
        shard.wavefront_frame(H, W, 0, 1, proc_g, chunks=1, out=out, streams=streams)
    timed_if("wave1", wave1, 10)


if __name__ == "__main__":
    main()
