"""Multi-process (gloo, world_size 2 and 3, CPU) tests of the C5 SB-row
sharding: band partition, padded all-gather, and that the sharded frame is
identical to the single-process result when every rank processes its band
with the oracle's C4 pipeline (the property that makes the sharding valid:
SB rows are independent for C4)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bands_partition():
    sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
    from lavish_dsp import shard
    for H in (64, 200, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            bs = shard.bands(H, world)
            assert bs[0][0] == 0 and bs[-1][1] == H
            for (a0, a1), (b0, b1) in zip(bs, bs[1:]):
                assert a1 == b0
            for b0, b1 in bs[:-1]:
                assert b0 % 64 == 0 and b1 % 64 == 0
            rows = [(-(-(b1 - b0) // 64)) for b0, b1 in bs]
            assert max(rows) - min(rows) <= 1
    # 4K: 34 SB rows over 8 GPUs -> 5,4,4,4,4,4,4,5 style balance
    assert sum(-(-(b1 - b0) // 64) for b0, b1 in shard.bands(2160, 8)) == 34


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import torch
        import torch.distributed as dist
        from lavish_dsp import shard
        import _c4ref as T  # the oracle C4 frame composition
        dist.init_process_group("gloo", rank=rank, world_size=world)
        src, pred = T.planes(10, 5, Wp=192, Hp=200)
        masks = {4: 0x1, 3: 0x201, 2: 0xFFFF, 1: 0x3}

        def band(y0, y1):
            _, _, rec = T.oracle_frame(src[y0:y1], pred[y0:y1], 10, masks, 1500)
            return torch.from_numpy(rec.view(np.int16).copy())
        full = shard.sharded_frame(200, rank, world, band)
        q.put((rank, full.numpy().view(np.uint16).copy()))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_frame_matches_single_process(world):
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _c4ref as T
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    src, pred = T.planes(10, 5, Wp=192, Hp=200)
    _, _, ref = T.oracle_frame(src, pred, 10, {4: 0x1, 3: 0x201, 2: 0xFFFF, 1: 0x3}, 1500)
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
        np.testing.assert_array_equal(got[r], ref)
