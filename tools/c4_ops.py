#!/usr/bin/env python3
"""Algorithmic int32 operation counts of the C4 step (DESIGN.md section 5,
"C4 algorithmic ops"), written to profiles/c4_ops.json for bench.py.

The 1-D transform counts come from the reference's own straight-line bodies
(av1/encoder/av1_fwd_txfm1d.c, av1/common/av1_inv_txfm1d.c), executed by
tests/golden/gen_golden.py's StraightLineEval with a counting integer: every
C `+`, `-`, `*` on a data value is one op, `half_btf` (av1_txfm.h:80-102:
two products, their sum, the rounding add and the shift) is 5, `round_shift`
(add + shift) 2, `clamp_value` (min + max) 2, `range_check_value` 0.  The
identity kernels are loops, counted from their bodies (fwd :1064-1094, inv
:1029-1060).  The per-element 2-D terms follow fwd_txfm2d_c
(av1_fwd_txfm2d.c:56-124) and inv_txfm2d_add_c (av1_inv_txfm2d.c:234-316);
the per-coefficient terms highbd_quantize_fp_helper_c (av1_quantize.c:
174-194, its branch-free form), aom_satd (avg.c:509-516),
av1_highbd_block_error (rdopt.c:664-682) and rate_estimator (tpl_model.c:
214-226).  64-bit adds / shifts / products count 2.

Needs /root/reference (run here, not on the GPU box).
usage: c4_ops.py [OUT_JSON]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gen_golden as G  # noqa: E402

COUNT = [0]


class Op:
    """A data value whose arithmetic counts one op per operator."""

    def _c(self, other=None):
        COUNT[0] += 1
        return Op()

    __add__ = __radd__ = __sub__ = __rsub__ = __mul__ = __rmul__ = _c
    __rshift__ = __lshift__ = __and__ = __or__ = __xor__ = _c

    def __neg__(self):  # `-a + b` is one subtraction
        return self

    def __pos__(self):
        return self


def _half_btf(w0, in0, w1, in1, bit):
    COUNT[0] += 5
    return Op()


def _round_shift(v, bit):
    COUNT[0] += 2
    return Op()


def _clamp_value(v, bit):
    COUNT[0] += 2
    return Op()


G.half_btf = _half_btf
G.round_shift = _round_shift
G.clamp_value = _clamp_value
G.range_check_value = lambda v, bit: v
G.wrap32 = lambda v: v

# identity kernels: ops per element (fwd av1_fwd_txfm1d.c:1064-1094, inv
# av1_inv_txfm1d.c:1029-1060): x NewSqrt2 + round_shift = 3, x 2 / x 4 = 1
IDENT = {4: 3, 8: 1, 16: 3, 32: 1}

TX_W = [4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64]
TX_H = [4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16]
# tx type -> (vertical, horizontal) 1-D kind: 0 DCT, 1 ADST, 2 FLIPADST, 3 IDTX
VTX = [0, 1, 0, 1, 2, 0, 2, 1, 2, 3, 0, 3, 1, 3, 2, 3]
HTX = [0, 0, 1, 1, 0, 2, 2, 2, 1, 3, 3, 0, 3, 1, 3, 2]


def one_d_counts():
    txfm_c = G.read("av1/common/av1_txfm.c")
    cospi = G.extract_array(txfm_c, "av1_cospi_arr_data")
    sinpi = G.extract_array(txfm_c, "av1_sinpi_arr_data")
    fwd1d = G.read("av1/encoder/av1_fwd_txfm1d.c")
    inv1d = G.read("av1/common/av1_inv_txfm1d.c")
    out = {"fwd": {}, "inv": {}}
    for side, src, pre in (("fwd", fwd1d, "f"), ("inv", inv1d, "i")):
        for kind, sizes in (("dct", (4, 8, 16, 32, 64)), ("adst", (4, 8, 16))):
            for n in sizes:
                ev = G.StraightLineEval(G.function_body(src, "av1_%s%s%d" % (pre, kind, n)),
                                        cospi, sinpi)
                COUNT[0] = 0
                ev.run([Op() for _ in range(n)], 12, [32] * 16)
                out[side]["%s%d" % (kind, n)] = COUNT[0]
        for n, per in IDENT.items():
            out[side]["identity%d" % n] = per * n
    return out


def kind_name(k, n):
    return ("dct%d" if k == 0 else "adst%d" if k in (1, 2) else "identity%d") % n


def shift_ops(bit):
    """av1_round_shift_array(arr, n, bit) per element (av1_txfm.c:71-87):
    round_shift 2, the clamped left shift 3 (shift + clamp64), none 0"""
    return 0 if bit == 0 else (2 if bit > 0 else 3)


def main(out_path):
    oned = one_d_counts()
    tables = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_tables.json")))
    fwd_shift, inv_shift = tables["fwd_shift"], tables["inv_shift"]
    sizes = {}
    for s in range(19):
        W, H = TX_W[s], TX_H[s]
        rect2 = W == 2 * H or H == 2 * W
        KW, KH = min(W, 32), min(H, 32)   # stored coefficient columns / rows
        sh = fwd_shift[s]
        # forward: per column (H-point, every column), per row (W-point, only
        # the KH rows whose coefficients are kept: the 64-point sizes zero the
        # rest, av1_fwd_txfm2d.c:236-312)
        col = {}
        for k in range(4):
            if H == 64 and k != 0:
                continue
            if H == 32 and k in (1, 2):
                continue
            col[k] = W * (H * shift_ops(-sh[0]) + oned["fwd"][kind_name(k, H)] +
                          H * shift_ops(-sh[1]))
        row = {}
        for k in range(4):
            if W == 64 and k != 0:
                continue
            if W == 32 and k in (1, 2):
                continue
            row[k] = KH * (oned["fwd"][kind_name(k, W)] + W * shift_ops(-sh[2]) +
                           (W * 3 if rect2 else 0))
        ish = inv_shift[s]
        # inverse: rows over the KH stored rows (the rest are zero in, zero
        # out), columns over every column, + highbd_clip_pixel_add
        irow = {k: KH * ((W * 3 if rect2 else 0) + W * 2 + oned["inv"][kind_name(k, W)] +
                         W * shift_ops(-ish[0])) for k in col_kinds(W)}
        icol = {k: W * (H * 2 + oned["inv"][kind_name(k, H)] + H * shift_ops(-ish[1]) + H * 3)
                for k in col_kinds(H)}
        sizes[s] = {"W": W, "H": H, "n": KW * KH, "fwd_col": col, "fwd_row": row,
                    "inv_row": irow, "inv_col": icol}
    res = {
        "source": "tools/c4_ops.py (reference 1-D bodies executed with a counting integer)",
        "one_d": oned,
        "per_pixel": {"subtract": 1},
        "per_coefficient": {"quantize_fp": 21, "satd": 2, "block_error": 9,
                            "rate_estimator": 9},
        "per_block_type": {"dist_shift_rdcost_select": 17},
        "per_block_decide": 3,
        "sizes": sizes,
        "vtx": VTX, "htx": HTX,
    }
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", out_path)
    for k, v in sorted(oned["fwd"].items()):
        print("fwd", k, v, "inv", oned["inv"][k])


def col_kinds(n):
    return (0,) if n == 64 else (0, 3) if n == 32 else (0, 1, 2, 3)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "c4_ops.json"))
