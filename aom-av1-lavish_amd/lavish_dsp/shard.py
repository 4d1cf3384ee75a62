"""C5: the C4 RDO step sharded over GPUs by superblock rows.

For C4 as defined (residual / prediction given) every TX block and every
64x64 superblock decision lies inside one SB, so any set of SBs is an
independent unit; what the ranks must exchange is the reconstruction: the
next SB row's intra prediction reads the reconstructed row above, the next
frame's inter prediction the whole frame (north_star: "an RCCL/xGMI
all-gather of the reconstructed row for next-row intra prediction").  Two
forms, both one process per GPU over torch.distributed (RCCL on the GPUs,
gloo on the CPU for the tests):

tiles (the one-step form, `tiled_frame`):
  One rectangle per rank, a gr x gc grid of whole-SB tiles with the
  smallest largest tile (`grid_partition`; at 4K exactly R C / G SBs per
  rank for G = 2, 4, 8), computed as a single C4 step and all-gathered once.
  A small rank share is latency-bound (a step costs about one decision
  wave's lifetime whatever its width), so one step per rank, not a band's
  and a tail's, is what the per-rank time scales with.

band (`sharded_frame`):
  The frame's R SB rows are dealt as floor(R / G) contiguous full rows per
  rank plus the R mod G leftover rows cut into G equal column segments
  (one each), so every rank holds exactly R / G SB rows of work: at 4K
  (34 rows) and 8 GPUs 4 rows + a quarter row each, no 34/40 = 85% cap of
  whole-row bands.  Each rank computes its band, then its tail segment, and
  all-gathers each part as soon as it is computed -- the band's gather
  (equal-sized on every rank) runs on a communication stream while the tail
  segment computes (`async_op`), then the tail segments are gathered.
  (`partition` gives the rectangles.)

row wavefront (the full-encoder-faithful form, `wavefront_frame`,
SURVEY 8(e)(ii) and ethread.c:113-160):
  SB row r runs on rank r mod G, in column chunks; before chunk c of row r
  the rank needs the bottom edge (the last `edge_rows` pixel rows, what the
  next row's intra predictors read) of row r - 1 up to chunk c + 1 (the
  above-right dependency), which rank (r - 1) mod G sends point-to-point as
  soon as it finishes each chunk; the received edges are written into the
  receiver's reconstruction above its row.  After every wave of G rows the
  wave's reconstructed rows are all-gathered (one SB row per rank: the
  per-row all-gather of north_star), on the communication stream, while the
  next wave computes.

process_rect(y0, y1, x0, x1) -> the reconstructed [y1 - y0, x1 - x0] region
is the per-rank work (the GPU C4 step in `c4_rect_processor`; the CPU tests pass
their own); the bookkeeping and the exchanges are plain torch.distributed.
"""

SB = 64


def sb_rows(height):
    return (height + SB - 1) // SB


def sb_cols(width):
    return (width + SB - 1) // SB


def bands(height, world):
    """Pixel-row bands [(y0, y1)] of whole SB rows, one per rank, contiguous,
    balanced to +-1 SB row (the round-2 partition; kept for reference)."""
    n = sb_rows(height)
    out = []
    for r in range(world):
        r0 = n * r // world
        r1 = n * (r + 1) // world
        out.append((min(r0 * SB, height), min(r1 * SB, height)))
    return out


def partition(height, width, world):
    """Per rank: (band, tail) pixel rectangles (y0, y1, x0, x1) or None.
    band: floor(R / G) whole SB rows, contiguous, rank-major; tail: rank g's
    column segment of the L = R mod G leftover rows -- leftover row i is cut
    into n_i = G (i + 1) // L - G i // L segments (whole SBs, widths within
    one SB), so the G segments go one per rank.  When L divides G every rank
    gets exactly R / G rows of work (4K: 34 rows = 8 x (4 + 1/4)).  A leftover
    row is never cut finer than its C SB columns (ranks beyond get no tail)."""
    R, C = sb_rows(height), sb_cols(width)
    full = R // world
    L = R - full * world
    out = []
    for g in range(world):
        band = (g * full * SB, min((g + 1) * full * SB, height), 0, width) if full else None
        tail = None
        if L:
            row = next(i for i in range(L) if g < world * (i + 1) // L)
            first = world * row // L
            # at most one segment per SB column: on a frame narrower than
            # the segment count the surplus ranks get no tail
            segs = min(world * (row + 1) // L - first, C)
            k = g - first
            if k < segs:
                c0, c1 = C * k // segs, C * (k + 1) // segs
                y0 = (full * world + row) * SB
                tail = (y0, min(y0 + SB, height), c0 * SB, min(c1 * SB, width))
        out.append((band, tail))
    return out


def grid_partition(height, width, world):
    """The tile form's rectangles: one (y0, y1, x0, x1) per rank, rank-major
    over a gr x gc grid (gr * gc = world) of whole-SB tiles -- SB rows and SB
    columns dealt as evenly as integers allow.  The grid is the factorisation
    with the smallest largest tile (ties: fewer column cuts, so rows stay
    long): at 4K (34 x 60 SBs) 2 x 1, 2 x 2, 2 x 4 tiles of exactly R C / G
    SBs for G = 2, 4, 8."""
    R, C = sb_rows(height), sb_cols(width)
    best = None
    for gr in range(1, world + 1):
        if world % gr:
            continue
        gc = world // gr
        if gr > R or gc > C:
            continue
        biggest = -(-R // gr) * -(-C // gc)
        if best is None or biggest < best[0] or (biggest == best[0] and gc < best[2]):
            best = (biggest, gr, gc)
    if best is None:
        raise ValueError("a %dx%d frame has fewer SBs than %d ranks in any grid" %
                         (width, height, world))
    _, gr, gc = best
    out = []
    for i in range(gr):
        r0, r1 = R * i // gr, R * (i + 1) // gr
        for j in range(gc):
            c0, c1 = C * j // gc, C * (j + 1) // gc
            out.append((r0 * SB, min(r1 * SB, height), c0 * SB, min(c1 * SB, width)))
    return out


def _gather_rects(local, rects, full, group, async_op):
    """All-gather equally shaped per-rank regions (local: this rank's
    [h, w] tensor; rects: every rank's (y0, y1, x0, x1), None for none)
    into `full`; regions are zero-padded to the largest one.  Returns a
    finisher (call it to wait and unpack)."""
    import torch
    import torch.distributed as dist
    world = len(rects)
    hmax = max((r[1] - r[0]) for r in rects if r is not None)
    wmax = max((r[3] - r[2]) for r in rects if r is not None)
    send = torch.zeros((hmax, wmax), dtype=full.dtype, device=full.device)
    if local is not None:
        send[:local.shape[0], :local.shape[1]] = local
    recv = torch.empty((world * hmax, wmax), dtype=full.dtype, device=full.device)
    work = None
    if world > 1:
        # moved as bytes: neither RCCL nor gloo gathers int16 as a dtype
        work = dist.all_gather_into_tensor(recv.view(torch.uint8), send.view(torch.uint8),
                                           group=group, async_op=async_op)
    else:
        recv.copy_(send)

    def finish():
        if work is not None and async_op:
            work.wait()
        for g, r in enumerate(rects):
            if r is None:
                continue
            y0, y1, x0, x1 = r
            full[y0:y1, x0:x1] = recv[g * hmax:g * hmax + (y1 - y0), :x1 - x0]
    return finish


def sharded_frame(height, width, rank, world, process_rect, group=None, like=None,
                  streams=None):
    """The band form: run process_rect on this rank's band, start its
    all-gather asynchronously, run the tail segment, gather the tails, and
    return the whole reconstructed frame (identical on every rank).
    streams (device work, optional): two streams; the band and its gather go
    on the first, the tail and its gather on the second, so the two parts
    (independent SBs) compute side by side -- the tail segment's few waves
    would otherwise run after the band's kernels; the caller's stream then
    waits for both."""
    import torch
    parts = partition(height, width, world)
    band, tail = parts[rank]
    if world == 1:  # one rank: the band is the frame, nothing to exchange
        return process_rect(*band)
    full = None
    fin = []
    caller = torch.cuda.current_stream() if streams else None
    if streams:
        start = torch.cuda.Event()
        start.record(caller)
    for phase, rect in enumerate((band, tail)):
        rects = [p[phase] for p in parts]
        if all(r is None for r in rects):
            continue
        if streams:
            st = streams[phase]
            st.wait_event(start)
            with torch.cuda.stream(st):
                local = process_rect(*rect) if rect is not None else None
                if full is None:
                    ref = local if local is not None else like
                    with torch.cuda.stream(caller):  # allocated on the caller's stream
                        full = torch.empty((height, width), dtype=ref.dtype, device=ref.device)
                    st.wait_stream(caller)
                fin.append((phase, _gather_rects(local, rects, full, group, async_op=True)))
        else:
            local = process_rect(*rect) if rect is not None else None
            if full is None:
                ref = local if local is not None else like
                full = torch.empty((height, width), dtype=ref.dtype, device=ref.device)
            fin.append((phase, _gather_rects(local, rects, full, group, async_op=True)))
    if streams:
        # each finisher on the stream its phase ran on (a skipped phase 0
        # leaves the tail's gather first in `fin`, still on streams[1])
        for phase, f in fin:
            with torch.cuda.stream(streams[phase]):
                f()
        for st in streams:
            caller.wait_stream(st)
    else:
        for _, f in fin:
            f()
    return full


def tiled_frame(height, width, rank, world, process_rect, group=None, like=None):
    """The tile form: this rank's one grid_partition rectangle (a single C4
    step, so a rank pays one step's latency, not a band's and a tail's),
    then one all-gather of the equally padded tiles into the whole
    reconstructed frame (identical on every rank)."""
    import torch
    rects = grid_partition(height, width, world)
    local = process_rect(*rects[rank])
    if world == 1:
        return local
    full = torch.empty((height, width), dtype=local.dtype, device=local.device)
    _gather_rects(local, rects, full, group, async_op=False)()
    return full


def wavefront_frame(height, width, rank, world, process_rect, chunks=4, edge_rows=4,
                    p2p_group=None, gather_group=None, dtype=None, device=None, log=None,
                    out=None, streams=None):
    """The row-wavefront form: SB row r on rank r % G, processed in `chunks`
    column chunks; chunk c of row r waits for the bottom `edge_rows` pixel
    rows of row r - 1 up to chunk c + 1 (point-to-point from rank
    (r - 1) % G, which sends each chunk's edge when it is done) and hands
    them to the chunk: process_rect(y0, y1, x0, x1, above=E) with E the
    [edge_rows, x0 : x1 + the next chunk] pixels above the chunk (None on row
    0) -- what the next row's intra prediction reads (above and above-right);
    after each wave of G rows the wave's rows are all-gathered.  Returns the
    whole reconstructed frame (identical on every rank).  The edges and the
    gathers must use different process groups (communicators): a rank's
    receive for the next wave must not queue behind its pending gather of
    this one, which waits for the sender.  out: the frame buffer to fill
    (process_rect may return views of it, then nothing is copied).  log:
    optional list that receives ('recv', row, chunk) / ('send', row, chunk)
    events.  streams (world 1, device work): the rows are dealt round-robin
    over these streams and each chunk waits, through events, only for the
    row above's chunk it depends on -- the wavefront's diagonal parallelism
    on one GPU (the reference's row threads, ethread.c:113-160); the rows
    overlap on the device only when process_rect replays graphs (see
    _wavefront_streams)."""
    import torch
    import torch.distributed as dist
    R, C = sb_rows(height), sb_cols(width)
    chunks = max(1, min(chunks, C))
    cx = [min(C * k // chunks * SB, width) for k in range(chunks + 1)]
    full = out if out is not None else torch.zeros((height, width), dtype=dtype, device=device)
    if world == 1 and streams:
        return _wavefront_streams(height, width, process_rect, chunks, cx, edge_rows, full,
                                  streams, log)
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    pending = []   # outstanding sends
    gathers = []
    for w0 in range(0, R, world):
        wave = list(range(w0, min(w0 + world, R)))
        mine = w0 + rank if w0 + rank < R else None
        if mine is not None:
            y0, y1 = mine * SB, min((mine + 1) * SB, height)
            edges = []   # the row above's bottom edge, chunk by chunk as received
            for c in range(chunks):
                # above-right: the row above's chunks 0 .. c + 1 (ethread.c
                # sync_range; the reference's own row-above dependency)
                need = min(c + 2, chunks) if mine > 0 else 0
                while len(edges) < need:
                    got = len(edges)
                    if world > 1:
                        edge = torch.empty((edge_rows, cx[got + 1] - cx[got]), dtype=full.dtype,
                                           device=full.device)
                        # on RCCL the wait orders the caller's stream after the
                        # receive and returns: the host goes on queueing chunks
                        # (gloo, the CPU tests, waits on the host)
                        dist.irecv(edge.view(torch.uint8), src=prv, group=p2p_group).wait()
                    else:  # the row above is this rank's own, already in the frame
                        edge = full[y0 - edge_rows:y0, cx[got]:cx[got + 1]]
                    edges.append(edge)
                    if log is not None:
                        log.append(("recv", mine - 1, got))
                above = (torch.cat(edges[c:need], 1) if need - c > 1 else edges[c]) \
                    if mine > 0 else None
                rec = process_rect(y0, y1, cx[c], cx[c + 1], above=above)
                dst = full[y0:y1, cx[c]:cx[c + 1]]
                if rec.data_ptr() != dst.data_ptr():
                    dst.copy_(rec)
                if mine + 1 < R and world > 1:
                    e = rec[rec.shape[0] - edge_rows:].contiguous()
                    pending.append((dist.isend(e.view(torch.uint8), dst=nxt, group=p2p_group),
                                    e))
                    if log is not None:
                        log.append(("send", mine, c))
        if world == 1:
            continue  # every row is already in the frame
        # the wave's rows: one SB row per rank (the per-row all-gather)
        rects = [(r * SB, min((r + 1) * SB, height), 0, width) for r in wave] + \
            [None] * (world - len(wave))
        local = full[mine * SB:min((mine + 1) * SB, height)].clone() if mine is not None else None
        gathers.append(_gather_rects(local, rects, full, gather_group, async_op=True))
    for f in gathers:
        f()
    for work, _ in pending:
        work.wait()
    return full


def _wavefront_streams(height, width, process_rect, chunks, cx, edge_rows, full, streams, log):
    """wavefront_frame at world 1 over several streams: row r on
    streams[r % len(streams)]; chunk c of row r waits for the event of row
    r - 1's chunk min(c + 1, chunks - 1) (chunks of a row complete in order
    on its stream), reads its edge rows from the frame, and records its own
    event; the caller's stream then waits for every row.  Device concurrency
    between rows needs process_rect to replay captured graphs
    (c4_rect_processor(graphs=True)): the direct calls share the library's
    per-thread fan-out streams and reconstruction scratch, which serialise
    the rows again (results are the same either way).

    With one chunk per row every row waits for the whole row above, so the
    rows are a chain: they go in order on streams[0], whose stream order is
    the dependency -- no events (a cross-queue event wait costs ~15 us of
    device time per row: 3.43 -> 2.99 ms per 4K frame on one box,
    tools/wavefront_probe.py)."""
    import torch
    R = sb_rows(height)
    caller = torch.cuda.current_stream()
    start = torch.cuda.Event()
    start.record(caller)
    if chunks == 1:
        st = streams[0]
        st.wait_event(start)
        with torch.cuda.stream(st):
            for r in range(R):
                y0, y1 = r * SB, min((r + 1) * SB, height)
                above = None
                if r > 0:
                    above = full[y0 - edge_rows:y0, 0:cx[1]]
                    if log is not None:
                        log.append(("recv", r - 1, 0))
                rec = process_rect(y0, y1, 0, cx[1], above=above)
                dst = full[y0:y1, 0:cx[1]]
                if rec.data_ptr() != dst.data_ptr():
                    dst.copy_(rec)
        caller.wait_stream(st)
        return full
    prev = None   # the row above's per-chunk events
    for r in range(R):
        st = streams[r % len(streams)]
        st.wait_event(start)
        y0, y1 = r * SB, min((r + 1) * SB, height)
        evs = []
        with torch.cuda.stream(st):
            for c in range(chunks):
                above = None
                if r > 0:
                    need = min(c + 2, chunks)
                    st.wait_event(prev[need - 1])
                    above = full[y0 - edge_rows:y0, cx[c]:cx[need]]
                    if log is not None:
                        log.append(("recv", r - 1, need - 1))
                rec = process_rect(y0, y1, cx[c], cx[c + 1], above=above)
                dst = full[y0:y1, cx[c]:cx[c + 1]]
                if rec.data_ptr() != dst.data_ptr():
                    dst.copy_(rec)
                e = torch.cuda.Event()
                e.record(st)
                evs.append(e)
        prev = evs
    for st in streams:
        caller.wait_stream(st)
    return full


def c4_rect_processor(src, pred, qp, rdmult, bit_depth, frames, out=None, graphs=False):
    """process_rect for the GPU path: lavish_rdo_frame + reconstruct on the
    rectangle [y0, y1) x [x0, x1) of device planes (views keep the planes'
    stride).  `frames` caches the RdoFrame output buffers per rectangle.  out
    (optional, a frame-sized plane with src's stride): each rectangle's
    reconstruction is written straight into its view of it.  `above` (the
    wavefront's received edge) is accepted and not read: C4 as defined takes
    its prediction as input, so no intra predictor consumes it here.  graphs:
    each rectangle's step is captured once into a HIP graph
    (lavish_rdo_graph_create) and replayed with one launch per call."""
    import lavish_dsp as L

    def run(y0, y1, x0, x1, above=None):
        s, p = src[y0:y1, x0:x1], pred[y0:y1, x0:x1]
        key = (y0, y1, x0, x1)
        if key not in frames:
            # a rectangle lower / narrower than a candidate size holds none of
            # its blocks: leave the size out (the per-SB decision skips sizes
            # that do not tile the SB, so the result is the whole frame's)
            masks = {t: m for t, m in L.C4_TYPE_MASKS.items()
                     if L.TX_W[t] <= x1 - x0 and L.TX_H[t] <= y1 - y0}
            frames[key] = L.RdoFrame(s, masks,
                                     recon=out[y0:y1, x0:x1] if out is not None else None)
            if graphs:
                frames[key].graph = L.RdoGraph(s, p, frames[key], qp, rdmult, bit_depth)
        fr = frames[key]
        if graphs:
            fr.graph.launch()
        else:
            L.rdo_frame(s, p, fr, qp, rdmult, bit_depth)
        return fr.recon
    return run


def c4_band_processor(src, pred, qp, rdmult, bit_depth, frames):
    """process_band(y0, y1) over whole-width bands (kept for callers of the
    round-2 interface)."""
    run = c4_rect_processor(src, pred, qp, rdmult, bit_depth, frames)
    return lambda y0, y1: run(y0, y1, 0, src.shape[1])
