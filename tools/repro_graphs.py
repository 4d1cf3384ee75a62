"""Stress of the captured C4 step (lavish_rdo_graph_*): the row wavefront at
world 1 with every 4K chunk a replayed graph over 4 streams, repeated with
fresh graphs each round (a diagnostic for a host crash inside hipGraphLaunch
seen once in the full GPU suite); prints a line per round."""
import gc
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(rounds=6, chunks=4, nst=4, keep=0):
    import torch
    import lavish_dsp as L
    import lavish_dsp.shard as shard
    import lavish_dsp.synth as synth
    W, H = 3840, 2160
    src = synth.frame(W, H, 10, 1234).astype(np.uint16)
    pred = synth.shifted(synth.frame(W, H, 10, 1235), 3, -2).astype(np.uint16)
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    qp = L.build_quant_params(10, 128, L.QUANT_FP)
    kept = []
    for r in range(rounds):
        t0 = time.time()
        out = torch.full_like(ts, -1)
        frames = {}
        direct = shard.c4_rect_processor(ts, tp, qp, 1700, 10, frames, out=out, graphs=True)
        streams = [torch.cuda.Stream() for _ in range(nst)] or None
        for _ in range(2):
            out.fill_(-1)
            shard.wavefront_frame(H, W, 0, 1, direct, chunks=chunks, out=out, streams=streams)
            torch.cuda.synchronize()
        if keep:
            kept.append(frames)
        del direct, frames
        gc.collect()
        print("round %d ok %.1fs graphs kept %d" % (r, time.time() - t0,
                                                     sum(len(f) for f in kept)), flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
