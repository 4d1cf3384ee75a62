"""Quick C3 timing: diamond search of all 16x16 blocks of a 1080p frame vs R refs."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "aom-av1-lavish_amd"))
import numpy as np, torch
import lavish_dsp.motion as M, lavish_dsp.synth as S
W, H, B = 1920, 1080, 160
for R in (1, 7):
    src, refs = S.motion_planes(W, H, R, B)
    st = src.shape[1]
    for bw in (16, 8, 32, 64):
        jobs = M.frame_jobs(W, H, st, B, src.size, bw, bw, R)
        ts, tr, tj = torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda(), M.to_device(jobs)
        for skip in (0, 1):
            out = M.diamond_search_batch(ts, tr, bw, bw, tj, use_downsampled_sad=skip)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                M.diamond_search_batch(ts, tr, bw, bw, tj, use_downsampled_sad=skip, out=out)
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 5
            r = M.results_numpy(out)
            steps = r["steps"].astype(np.int64).sum(); srch = r["searches"].astype(np.int64).sum()
            rows = bw // 2 if skip and bw >= 16 else bw
            algo = len(jobs) * bw * bw + steps * 8 * rows * bw + srch * 2 * bw * bw
            print("R=%d %dx%d skip=%d jobs=%d ms=%.3f steps/job=%.1f searches/job=%.2f algoGB/s=%.0f"
                  % (R, bw, bw, skip, len(jobs), ms, steps / len(jobs), srch / len(jobs), algo / ms / 1e6), flush=True)
