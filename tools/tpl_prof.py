"""Per-phase clock of the TPL start-mv wavefront (diagnostic).

Runs the bench's TPL motion search (1080p x 7 refs) a few times through a
library built with -DLAVISH_TPL_PROF=1 (LAVISH_HIP_LIB) and prints wave 0's
clock per block step, by phase (see tpl_mv_kernel's LAVISH_TPL_PROF note).
Usage: LAVISH_HIP_LIB=tools/dbg/lib_tplprof.so python tools/tpl_prof.py [reps]
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
sys.path.insert(0, ROOT)


def main(reps=5):
    import torch
    import lavish_dsp as L
    import lavish_dsp.synth as synth
    import lavish_dsp.tpl as T
    import bench
    W, H, R = 1920, 1080, 7
    src, refs = synth.tpl_motion_planes(W, H, R, bench.TPL_BORDER, seed=1234)
    tf = T.TplFrame(src, refs, W, H, bench.TPL_BORDER, 128, 2000)
    lib = ctypes.CDLL(L.LIB_PATH)
    fn = lib.lavish_dbg_tpl_prof
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 16)()
    stream = torch.cuda.current_stream()

    def run():
        T.tpl_motion_search(tf.src, tf.refs, tf.jobs, tf.cols, tf.rows, tf.nrefs, tf.cost,
                            tf.search_method, tf.step_param, tf.skip_sad, tf.prune, tf.alike,
                            out=tf.mv_out, stream=stream)

    run()
    torch.cuda.synchronize()
    assert fn(buf, 1) == 0
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    assert fn(buf, 1) == 0
    v = list(buf)
    steps = max(v[7], 1)
    names = ["await", "after_wait_work", "before_wait_work", None, "publish"]
    out = {"ms_per_call_host": round(ms, 4), "blocks": steps // reps,
           "cycles_per_step": {n: round(v[i] / steps, 1) for i, n in enumerate(names) if n},
           "new_centre_after_wait_frac": round(v[3] / steps, 4),
           "walk_cycles_per_wave": round(v[5] / max(1, reps * tf.rows * tf.nrefs), 1),
           "polls_ready_first_time": v[6],
           "speculative_walk_cycles_per_step": {n: round(v[8 + i] / steps, 1) for i, n in enumerate(
               ["centres", "window_fill", "ranking_sads", "sort_cut", "searches"])},
           "searches_per_step": round(v[13] / steps, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
