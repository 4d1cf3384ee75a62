"""Diagnostic: C3 1080p GPU vs oracle under several cost settings; saves the
mismatching jobs to gpurun_out/diag_c3.npz."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O  # noqa: E402
import lavish_dsp.motion as M  # noqa: E402
import lavish_dsp.synth as synth  # noqa: E402

W, H, R, border = 1920, 1080, 7, 160
src, refs = synth.motion_planes(W, H, R, border, seed=1234)
st = src.shape[1]
jobs = M.frame_jobs(W, H, st, border, src.size, 16, 16, R)
mvj, mvc = M.default_mv_cost_tables(False)
tsrc, trefs = torch.from_numpy(src).cuda(), torch.from_numpy(refs).cuda()
tj = M.to_device(jobs)
out = {}
for name, ctype, skip, cl in (("l1", 3, True, False), ("ent_noskip_nocl", 0, False, False),
                              ("ent_skip_nocl", 0, True, False), ("ent_skip_cl", 0, True, True)):
    cp = M.MvCosts(mvj, mvc).cost_params(4, 31, ctype)
    fp, cls = M.full_pixel_search_batch(tsrc, trefs, 16, 16, tj, cp, "diamond", 0, skip, cl)
    torch.cuda.synchronize()
    got = M.results_numpy(fp)
    exp, _ = O.full_pixel_search_batch(src.reshape(-1), refs.reshape(-1), st, 16, 16, jobs,
                                       "diamond", 0, ctype, 4, 31, mvj, mvc, skip=skip,
                                       cost_list=cl, threads=16)
    bad = np.nonzero((got["best_row"] != exp["best_row"]) | (got["best_col"] != exp["best_col"])
                     | (got["bestsme"] != exp["bestsme"]))[0]
    print(name, "mismatches", len(bad), flush=True)
    out[name + "_idx"] = bad[:200]
    out[name + "_got"] = got[bad[:200]].view(np.uint8)
    out[name + "_exp"] = exp[bad[:200]].view(np.uint8)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "diag_c3.npz"), **out)
