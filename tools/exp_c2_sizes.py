"""Per-size C2 timing: each txq_plane_kernel<W,H> alone over a 1080p residual
(all valid types, quantize_fp qindex 128), algorithmic GB/s per size, then the
whole frame (lavish_txq_frame) for comparison."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "aom-av1-lavish_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

import lavish_dsp as L  # noqa: E402
import lavish_dsp.synth as S  # noqa: E402
from bench import algorithmic_bytes  # noqa: E402

W, H = 1920, 1080
res = torch.from_numpy(S.residual_plane(W, H, 8, seed=1234)).cuda()
qp = L.build_quant_params(8, 128, L.QUANT_FP)
sizes = [s for s in range(19) if L.TX_W[s] <= 32 and L.TX_H[s] <= 32]
tot_ms = 0.0
for s in sizes:
    m = L.valid_type_mask(s)
    out = L.txq_plane(res, s, m, qp)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        L.txq_plane(res, s, m, qp, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    b = algorithmic_bytes(L, s, W, H)
    tot_ms += ms
    print("%-6s types=%2d ms=%.4f MB=%7.1f GB/s=%6.0f" % (L.TX_SIZES[s], bin(m).count("1"), ms,
                                                         b / 1e6, b / ms / 1e6), flush=True)
fr = L.FrameOutputs(res, sizes)
L.txq_frame(res, fr, qp)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    L.txq_frame(res, fr, qp)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
b = sum(algorithmic_bytes(L, s, W, H) for s in sizes)
print("serial sum ms=%.4f  frame ms=%.4f GB/s=%.0f" % (tot_ms, ms, b / ms / 1e6))
# raw write bandwidth reference: fill a 2.6 GB buffer
buf = torch.empty(b // 4, dtype=torch.int32, device="cuda")
buf.fill_(1)
torch.cuda.synchronize()
e0.record()
for _ in range(5):
    buf.fill_(7)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print("torch fill %d MB ms=%.4f GB/s=%.0f" % (b // 1e6, ms, b / ms / 1e6))
