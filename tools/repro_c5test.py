"""Diagnostic: test_gpu_fullsize.py::test_c5_partition_rects_on_gpu's graph
cases step by step with a line per step (a host crash inside hipGraphLaunch
in its one-chunk case).  usage: repro_c5test.py CASES [destroy] [whole]
CASES: comma list of graphs:streams:chunks, e.g. 1:0:4,1:4:4,1:4:1;
destroy 0 keeps every case's graphs alive to the end; whole 0 skips the
uncaptured whole-frame step the test runs first (its reference)."""
import gc
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))


def say(*a):
    print(*a, flush=True)


def main(cases, destroy=1, whole_first=1):
    import torch
    import lavish_dsp as L
    import lavish_dsp.shard as shard
    import lavish_dsp.synth as synth
    W, H, rdmult = 3840, 2160, 1700
    src = synth.frame(W, H, 10, 1234).astype(np.uint16)
    pred = synth.shifted(synth.frame(W, H, 10, 1235), 3, -2).astype(np.uint16)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    qp = L.build_quant_params(10, 128, L.QUANT_FP)
    ref = None
    if whole_first:
        whole = L.RdoFrame(ts)
        L.rdo_frame(ts, tp, whole, qp, rdmult, 10)
        ref = whole.recon.cpu().numpy()
        say("whole frame done")
    kept = []
    for case in cases.split(","):
        graphs, nst, chunks = (int(v) for v in case.split(":"))
        say("case", case)
        out = torch.full_like(ts, -1)
        frames = {}
        direct = shard.c4_rect_processor(ts, tp, qp, rdmult, 10, frames, out=out,
                                         graphs=bool(graphs))
        streams = [torch.cuda.Stream() for _ in range(nst)] or None
        if graphs and streams:
            shard.wavefront_frame(H, W, 0, 1, direct, chunks=chunks, out=out)
            torch.cuda.synchronize()
            say("  captured", len(frames))
        for p in range(2):
            out.fill_(-1)
            shard.wavefront_frame(H, W, 0, 1, direct, chunks=chunks, out=out, streams=streams)
            torch.cuda.synchronize()
            ok = ref is None or np.array_equal(out.cpu().numpy(), ref)
            say("  pass", p, "equal" if ok else "DIFFERENT")
            if ref is None:
                ref = out.cpu().numpy()
        if not destroy:
            kept.append(frames)
        del direct, frames
        gc.collect()
        torch.cuda.synchronize()
        say("  freed")


if __name__ == "__main__":
    main(sys.argv[1], *[int(a) for a in sys.argv[2:]])
