"""C4 reference compositions shared by the GPU tests and the gloo sharding
tests (test infrastructure: the oracle's per-size decisions, the per-SB
TX-size choice and the oracle reconstruction)."""
import numpy as np

import _oracle as O


def planes(bd, seed, Wp=384, Hp=192):
    import lavish_dsp.synth as synth
    src = synth.frame(Wp, Hp, bd, seed)
    pred = synth.shifted(synth.frame(Wp, Hp, bd, seed + 1), 3, -2)
    return src.astype(np.uint16), pred.astype(np.uint16)


def oracle_frame(src, pred, bd, masks, rdmult, threads=8, px=False):
    """C4 frame reference: per-size oracle decisions (px: pixel-domain
    distortion), the per-SB TX-size choice (lowest summed rd cost, ties to
    the larger size) and the reconstruction with the oracle's inverse
    transform."""
    H, W = src.shape
    q = O.build_quant(bd, 128)
    per = {s: O.rdo_plane(src, pred, s, m, bd, q, rdmult, threads=threads, px=px)
           for s, m in masks.items()}
    sizes = sorted(masks, key=lambda s: -O.TX_W[s] * O.TX_H[s])
    sbw, sbh = (W + 63) // 64, (H + 63) // 64
    choice = np.full(sbw * sbh, 255, np.uint8)
    for sy in range(sbh):
        for sx in range(sbw):
            best = None
            for s in sizes:
                bw_, bh_ = O.TX_W[s], O.TX_H[s]
                y1, x1 = min(64, H - sy * 64), min(64, W - sx * 64)
                if y1 % bh_ or x1 % bw_:
                    continue
                nbx = W // bw_
                tot = 0
                for y in range(0, y1, bh_):
                    for x in range(0, x1, bw_):
                        tot = min(tot + int(per[s][0]["rdcost"][((sy * 64 + y) // bh_) * nbx
                                                                + (sx * 64 + x) // bw_]),
                                  2 ** 63 - 1)  # saturating, as orc_rdo_reconstruct
                if tot < (2 ** 63 - 1 if best is None else best[0]):
                    best = (tot, s)
            if best is not None:
                choice[sy * sbw + sx] = best[1]
    recon = pred.copy()
    for s in sizes:
        bw_, bh_ = O.TX_W[s], O.TX_H[s]
        rec, qc, dq = per[s]
        nbx = W // bw_
        for blk in range(len(rec)):
            by, bx = divmod(blk, nbx)
            y, x = by * bh_, bx * bw_
            if choice[(y // 64) * sbw + x // 64] != s or rec["eob"][blk] == 0:
                continue
            recon[y:y + bh_, x:x + bw_] = O.inv_txfm2d_add(dq[blk], recon[y:y + bh_, x:x + bw_],
                                                           int(rec["best_type"][blk]), s, bd)
    return per, choice, recon




def oracle_frame_c(src, pred, bd, masks, rdmult, threads=8, px=False):
    """oracle_frame with the SB decision and reconstruction in C
    (orc_rdo_reconstruct); used as bench.py's C4 CPU baseline."""
    import ctypes
    H, W = src.shape
    q = O.build_quant(bd, 128)
    sizes = sorted(masks, key=lambda s: -O.TX_W[s] * O.TX_H[s])
    per = {s: O.rdo_plane(src, pred, s, masks[s], bd, q, rdmult, threads=threads, px=px)
           for s in sizes}
    L = O.lib()
    vp = ctypes.c_void_p
    L.orc_rdo_reconstruct.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp,
                                      vp, ctypes.c_int, ctypes.c_int, vp]
    sz = np.array(sizes, np.int32)
    recs = (vp * len(sizes))(*[per[s][0].ctypes.data for s in sizes])
    dqs = (vp * len(sizes))(*[per[s][2].ctypes.data for s in sizes])
    pred = np.ascontiguousarray(pred, dtype=np.uint16)
    recon = np.empty_like(pred)
    choice = np.zeros(((W + 63) // 64) * ((H + 63) // 64), np.uint8)
    L.orc_rdo_reconstruct(len(sizes), O.P(sz), ctypes.cast(recs, vp), ctypes.cast(dqs, vp), W, H,
                          O.P(pred), O.P(recon), W, bd, O.P(choice))
    return per, choice, recon
