# experiment: concurrency of the 14 per-size launches over several streams
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
import torch, lavish_dsp as L, lavish_dsp.synth as synth
res = torch.from_numpy(synth.residual_plane(1920, 1080, 8)).cuda()
sizes = [s for s in range(19) if L.TX_W[s] <= 32 and L.TX_H[s] <= 32]
qp = L.build_quant_params(8, 128, L.QUANT_FP)
outs = {s: L.txq_plane_out(res, s, L.valid_type_mask(s)) for s in sizes}
order = sorted(sizes, key=lambda s: -bin(L.valid_type_mask(s)).count("1") * L.TX_W[s] * L.TX_H[s])
for ns in (1, 2, 3, 4, 6):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    main = torch.cuda.current_stream()
    def step():
        ev = torch.cuda.Event(); ev.record(main)
        for st in streams: st.wait_event(ev)
        for i, s in enumerate(order):
            L.txq_plane(res, s, L.valid_type_mask(s), qp, out=outs[s], stream=streams[i % ns])
        for st in streams:
            e = torch.cuda.Event(); e.record(st); main.wait_event(e)
    for _ in range(3): step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(30): step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 30
    print("streams=%d ms/step=%.4f SB64/s=%.0f" % (ns, dt * 1e3, 510 / dt), flush=True)
