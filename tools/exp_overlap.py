"""C2 (txq frame) and C3 (diamond search) of one 1080p frame: each alone,
back to back on one stream, and concurrently (C3 on a second stream)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
import torch  # noqa: E402

import lavish_dsp as L  # noqa: E402
import lavish_dsp.motion as M  # noqa: E402
import lavish_dsp.synth as S  # noqa: E402

W, H, R, B = 1920, 1080, 7, 160
res = torch.from_numpy(S.residual_plane(W, H, 8, seed=1234)).cuda()
sizes = [s for s in range(19) if L.TX_W[s] <= 32 and L.TX_H[s] <= 32]
qp = L.build_quant_params(8, 128, L.QUANT_FP)
fr = L.FrameOutputs(res, sizes)
src, refs = S.motion_planes(W, H, R, B, seed=1234)
jobs = M.frame_jobs(W, H, src.shape[1], B, src.size, 16, 16, R)
ts, tr, tj = torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda(), M.to_device(jobs)
out = torch.empty(len(jobs) * M.RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
main = torch.cuda.current_stream()
side = torch.cuda.Stream()


def c2(st=None):
    L.txq_frame(res, fr, qp, stream=st)


def c3(st=None):
    M.diamond_search_batch(ts, tr, 16, 16, tj, 0, 3, True, out=out, stream=st)


def seq():
    c3(main)
    c2(main)


def conc(first_c3=True):
    e = torch.cuda.Event()
    e.record(main)
    side.wait_event(e)
    if first_c3:
        c3(side)
        c2(main)
    else:
        c2(main)
        c3(side)
    e2 = torch.cuda.Event()
    e2.record(side)
    main.wait_event(e2)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(n):
        fn()
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for name, fn in (("c2", lambda: c2(main)), ("c3", lambda: c3(main)), ("seq", seq),
                 ("conc c3-first", lambda: conc(True)), ("conc c2-first", lambda: conc(False))):
    ms = timeit(fn)
    print("%-14s ms=%.4f SB64/s=%.0f" % (name, ms, 510 / ms * 1e3), flush=True)
