"""C5 at its configuration size (3840x2160 10-bit) with the HIP C4 step in
the ranks: two processes on one GPU (gloo between them, reconstructions
moved through host memory), the band form and the row-wavefront form of
lavish_dsp/shard.py, each rank's frame equal to the single-process
whole-frame step; in the wavefront form every chunk's received edge (the 4
pixel rows above it and its above-right chunk) equals those rows of the
whole-frame reconstruction."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, RDMULT = 3840, 2160, 1700   # 34 SB rows (the last 48 px high)
CHUNKS = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _planes():
    sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
    import lavish_dsp.synth as synth
    src = synth.frame(W, H, 10, 77).astype(np.uint16)
    pred = synth.shifted(synth.frame(W, H, 10, 78), 3, -2).astype(np.uint16)
    return src, pred


def _worker(rank, world, port, q, form):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
        import torch
        import torch.distributed as dist
        import lavish_dsp as L
        import lavish_dsp.shard as shard
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        src, pred = _planes()
        ts = torch.from_numpy(src.view(np.int16)).cuda()
        tp = torch.from_numpy(pred.view(np.int16)).cuda()
        qp = L.build_quant_params(10, 128, L.QUANT_FP)
        gpu = shard.c4_rect_processor(ts, tp, qp, RDMULT, 10, {})

        aboves = []

        def rect(y0, y1, x0, x1, above=None):   # the HIP step; gloo moves host tensors
            if above is not None:
                aboves.append((y0, x0, above.numpy().view(np.uint16).copy()))
            return gpu(y0, y1, x0, x1, above=above).cpu()
        if form == "band":
            full = shard.sharded_frame(H, W, rank, world, rect)
        elif form == "band_streams":
            # bench.py --c5-form band's arrangement: band and tail on two
            # streams, each part's gather finished on its own stream
            streams = [torch.cuda.Stream(), torch.cuda.Stream()]
            full = shard.sharded_frame(H, W, rank, world, rect, streams=streams)
            torch.cuda.synchronize()
        else:
            p2p = dist.new_group(list(range(world)))
            full = shard.wavefront_frame(H, W, rank, world, rect, chunks=CHUNKS, p2p_group=p2p,
                                         dtype=torch.int16)
        q.put((rank, (full.numpy().view(np.uint16).copy(), aboves)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


@pytest.mark.parametrize("form", ["band", "band_streams", "wave"])
def test_c5_two_ranks_hip_step(form):
    import torch
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
    import lavish_dsp as L
    src, pred = _planes()
    ts = torch.from_numpy(src.view(np.int16)).cuda()
    tp = torch.from_numpy(pred.view(np.int16)).cuda()
    whole = L.RdoFrame(ts)
    L.rdo_frame(ts, tp, whole, L.build_quant_params(10, 128, L.QUANT_FP), RDMULT, 10)
    ref = whole.recon.cpu().numpy().view(np.uint16)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, form)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=150) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    C = (W + 63) // 64
    cx = [min(C * k // CHUNKS * 64, W) for k in range(CHUNKS + 1)]
    for r in range(2):
        assert not isinstance(got[r], str), got[r]
        full, aboves = got[r]
        np.testing.assert_array_equal(full, ref)
        if form == "wave":
            rows = [row for row in range(r, (H + 63) // 64, 2) if row > 0]
            assert len(aboves) == CHUNKS * len(rows)
            for y0, x0, above in aboves:
                c = cx.index(x0)
                np.testing.assert_array_equal(above, ref[y0 - 4:y0, x0:cx[min(c + 2, CHUNKS)]],
                                              err_msg="edge above (%d, %d)" % (y0, x0))
        else:
            assert aboves == []
