"""Multi-process (gloo, CPU) tests of the C5 sharding (lavish_dsp/shard.py):
the balanced band partition, the band form with its overlapped per-part
all-gathers, the tile form (one grid tile per rank, one gather), and the
row-wavefront form with point-to-point edges and the
per-wave row all-gather -- each rank processing its rectangles with the
oracle's C4 pipeline, the sharded frame identical to the single-process
result (the property that makes the sharding valid: SBs are independent
for C4), world sizes 2, 3 and 8."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MASKS = {4: 0x1, 3: 0x201, 2: 0xFFFF, 1: 0x3}
GEOM = (200, 256)   # 4 SB rows (the last 8 px high) x 4 SB columns


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard():
    sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
    from lavish_dsp import shard
    return shard


def test_bands_partition():
    shard = _shard()
    for H in (64, 200, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            bs = shard.bands(H, world)
            assert bs[0][0] == 0 and bs[-1][1] == H
            for (a0, a1), (b0, b1) in zip(bs, bs[1:]):
                assert a1 == b0
    assert sum(-(-(b1 - b0) // 64) for b0, b1 in shard.bands(2160, 8)) == 34


@pytest.mark.parametrize("H,W", [(2160, 3840), (1080, 1920), (200, 256), (64, 64)])
def test_partition_covers_and_balances(H, W):
    """Every pixel in exactly one rectangle; at 4K and 1080p every world in
    1..8 within 7% of perfect balance (whole-row bands: 85% at 4K x 8)."""
    shard = _shard()
    for world in range(1, 9):
        cov = np.zeros((H, W), np.int32)
        work = []
        for band, tail in shard.partition(H, W, world):
            w = 0
            for r in (band, tail):
                if r is not None:
                    y0, y1, x0, x1 = r
                    assert y0 % 64 == 0 and x0 % 64 == 0
                    cov[y0:y1, x0:x1] += 1
                    w += (y1 - y0) * (x1 - x0)
            work.append(w)
        assert (cov == 1).all(), world
        if H >= 1080:
            assert np.mean(work) / max(work) > 0.93, (world, work)
    # 4K on 8 GPUs: 4 rows + a quarter row (15 SBs) each
    parts = shard.partition(2160, 3840, 8)
    assert all(b[1] - b[0] == 256 and t[3] - t[2] == 960 for b, t in parts)


def _worker(rank, world, port, q, form):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import torch
        import torch.distributed as dist
        from lavish_dsp import shard
        import _c4ref as T  # the oracle C4 frame composition
        dist.init_process_group("gloo", rank=rank, world_size=world)
        H, W = GEOM
        src, pred = T.planes(10, 5, Wp=W, Hp=H)
        done = []
        aboves = []

        def rect(y0, y1, x0, x1, above=None):
            done.append((y0, y1, x0, x1))
            if above is not None:  # the received edge, as the chunk got it
                aboves.append((y0, x0, above.numpy().view(np.uint16).copy()))
            _, _, rec = T.oracle_frame(np.ascontiguousarray(src[y0:y1, x0:x1]),
                                       np.ascontiguousarray(pred[y0:y1, x0:x1]), 10, MASKS, 1500,
                                       threads=1)
            return torch.from_numpy(rec.view(np.int16).copy())
        log = []
        if form == "band":
            full = shard.sharded_frame(H, W, rank, world, rect)
        elif form == "tiles":
            full = shard.tiled_frame(H, W, rank, world, rect)
        else:
            p2p = dist.new_group(list(range(world)))
            full = shard.wavefront_frame(H, W, rank, world, rect, chunks=3, p2p_group=p2p,
                                         dtype=torch.int16, log=log)
        q.put((rank, full.numpy().view(np.uint16).copy(), done, (log, aboves)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None, None))


def _run(world, form):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, form)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, full, done, log = q.get(timeout=300)
        got[r] = (full, done, log)
    for p in procs:
        p.join(timeout=60)
    return got


def _reference():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "aom-av1-lavish_amd"))
    import _c4ref as T
    H, W = GEOM
    src, pred = T.planes(10, 5, Wp=W, Hp=H)
    return T.oracle_frame(src, pred, 10, MASKS, 1500)[2]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_band_form_matches_single_process(world):
    got = _run(world, "band")
    ref = _reference()
    shard = _shard()
    parts = shard.partition(*GEOM, world)
    for r in range(world):
        full, done, _ = got[r]
        assert not isinstance(full, str), full
        np.testing.assert_array_equal(full, ref)
        assert done == [x for x in parts[r] if x is not None]  # band, then tail


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tile_form_matches_single_process(world):
    """One grid tile per rank, one gather: every rank ends with the
    single-process frame and computed exactly its tile."""
    got = _run(world, "tiles")
    ref = _reference()
    rects = _shard().grid_partition(*GEOM, world)
    for r in range(world):
        full, done, _ = got[r]
        assert not isinstance(full, str), full
        np.testing.assert_array_equal(full, ref)
        assert done == [rects[r]]


@pytest.mark.parametrize("H,W", [(2160, 3840), (1080, 1920), (200, 256), (288, 352)])
def test_grid_partition_covers_and_balances(H, W):
    """Every pixel in exactly one tile, tiles on SB boundaries; at 4K the
    tiles of G = 2, 4, 8 hold exactly R C / G SBs."""
    shard = _shard()
    R, C = shard.sb_rows(H), shard.sb_cols(W)
    for world in range(1, 9):
        try:
            rects = shard.grid_partition(H, W, world)
        except ValueError:
            assert all(world % gr or gr > R or world // gr > C for gr in range(1, world + 1))
            continue
        assert len(rects) == world
        cov = np.zeros((H, W), np.int32)
        for y0, y1, x0, x1 in rects:
            assert y0 % 64 == 0 and x0 % 64 == 0 and y1 > y0 and x1 > x0
            cov[y0:y1, x0:x1] += 1
        assert (cov == 1).all(), world
    for world in (2, 4, 8):
        sbs = [-(-(y1 - y0) // 64) * -(-(x1 - x0) // 64)
               for y0, y1, x0, x1 in shard.grid_partition(2160, 3840, world)]
        assert sbs == [2040 // world] * world


def test_partition_narrow_frames():
    """A leftover row is cut into at most its SB columns: on frames narrower
    than the rank count no tail is empty, surplus ranks get none, and every
    pixel is still covered once."""
    shard = _shard()
    for W in (64, 128, 320):
        for R in range(1, 12):
            H = 64 * R - 8
            for world in range(1, 9):
                cov = np.zeros((H, W), np.int32)
                for band, tail in shard.partition(H, W, world):
                    for rc in (band, tail):
                        if rc is not None:
                            y0, y1, x0, x1 = rc
                            assert y1 > y0 and x1 > x0, (W, H, world, rc)
                            cov[y0:y1, x0:x1] += 1
                assert (cov == 1).all(), (W, H, world)


@pytest.mark.parametrize("world", [2, 3])
def test_wavefront_form_matches_single_process(world):
    """Row r on rank r % G, 3 column chunks per row: every rank ends with the
    single-process frame, and the edge traffic follows the wavefront: rank g
    receives row r - 1's chunks in order before (and only as far as) each
    chunk of row r needs them."""
    got = _run(world, "wave")
    ref = _reference()
    H, W = GEOM
    R = (H + 63) // 64
    C = (W + 63) // 64
    cx = [min(C * k // 3 * 64, W) for k in range(4)]
    for r in range(world):
        full, done, logs = got[r]
        assert not isinstance(full, str), full
        np.testing.assert_array_equal(full, ref)
        log, aboves = logs
        # every chunk below row 0 got the row above's bottom 4 pixel rows over
        # its own columns and the next chunk's (above-right), exactly as the
        # single-process reconstruction has them
        assert len(aboves) == sum(3 for y0, _, x0, _ in done if y0 > 0 and x0 == 0)
        for y0, x0, above in aboves:
            c = cx.index(x0)
            x1 = cx[min(c + 2, 3)]
            np.testing.assert_array_equal(above, ref[y0 - 4:y0, x0:x1], err_msg=str((y0, x0)))
        rows = [y0 // 64 for y0, _, _, _ in done]
        assert rows == sorted(rows) and all(row % world == r for row in rows)
        if world > 1:
            for row in range(r, R, world):
                if row == 0:
                    continue
                recv = [c for k, rr, c in log if k == "recv" and rr == row - 1]
                assert recv == [0, 1, 2], (row, recv)
            # chunk c of a row is computed only after chunks <= c + 1 of the row above arrived
            seen = 0
            for k, rr, c in log:
                if k == "recv":
                    seen = c + 1
                elif rr > 0:
                    assert seen >= min(c + 2, 3) or rr == 0
