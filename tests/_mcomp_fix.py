"""Helpers over tests/golden/fix_mcomp.npz (av1_full_pixel_search executed
from the reference by tests/golden/gen_fixtures.py): the fixture jobs as
LavishDiamondJob records grouped into the batches one call can serve."""
import numpy as np

MS_METHODS = ["diamond", "bigdia", "fast_bigdia"]   # fixture "cases" column 0
MS_JOB = np.dtype([("src_off", "<i8"), ("ref_off", "<i8"), ("start_row", "<i2"),
                   ("start_col", "<i2"), ("ref_mv_row", "<i2"), ("ref_mv_col", "<i2"),
                   ("col_min", "<i2"), ("col_max", "<i2"), ("row_min", "<i2"),
                   ("row_max", "<i2")], align=True)


def mcomp_groups(F):
    """Fixture jobs grouped by (case, block size, lambdas) -- the parameters
    one batch call shares -- as (case row, bw, bh, epb, spb, JOB records,
    expected rows)."""
    J = {n: i for i, n in enumerate(F["job_fields"])}
    jobs = F["jobs"]
    W, H, BORDER, NREF = (int(v) for v in F["geom"])
    stride = F["src"].shape[1]
    plane = F["refs"][0].size
    org = BORDER * stride + BORDER
    key = lambda r: tuple(int(r[J[k]]) for k in ("case", "bw", "bh", "error_per_bit",
                                                   "sad_per_bit"))
    groups = {}
    for r in jobs:
        groups.setdefault(key(r), []).append(r)
    for (ci, bw, bh, epb, spb), rows in sorted(groups.items()):
        rows = np.array(rows)
        rec = np.zeros(len(rows), MS_JOB)
        off = org + rows[:, J["by"]] * stride + rows[:, J["bx"]]
        rec["src_off"], rec["ref_off"] = off, off + rows[:, J["ref"]] * plane
        for f in ("start_row", "start_col", "ref_mv_row", "ref_mv_col", "col_min", "col_max",
                  "row_min", "row_max"):
            rec[f] = rows[:, J[f]]
        yield F["cases"][ci], bw, bh, epb, spb, rec, rows, J


def subpel_groups(F, mc):
    """fix_subpel.npz jobs grouped by (case, block size, error_per_bit), as
    (case row, bw, bh, epb, JOB records (start = full-pel best x 8, subpel
    limits), cost lists int32 [n][5], expected rows, field index); mc: the
    fix_mcomp.npz dict (planes and geometry)."""
    J = {n: i for i, n in enumerate(F["job_fields"])}
    W, H, BORDER, NREF = (int(v) for v in mc["geom"])
    stride = mc["src"].shape[1]
    plane = mc["refs"][0].size
    org = BORDER * stride + BORDER
    groups = {}
    for r in F["jobs"]:
        key = tuple(int(r[J[k]]) for k in ("case", "bw", "bh", "error_per_bit"))
        groups.setdefault(key, []).append(r)
    for (ci, bw, bh, epb), rows in sorted(groups.items()):
        rows = np.array(rows)
        rec = np.zeros(len(rows), MS_JOB)
        off = org + rows[:, J["by"]] * stride + rows[:, J["bx"]]
        rec["src_off"], rec["ref_off"] = off, off + rows[:, J["ref"]] * plane
        for f in ("start_row", "start_col", "ref_mv_row", "ref_mv_col", "col_min", "col_max",
                  "row_min", "row_max"):
            rec[f] = rows[:, J[f]]
        cls = (np.ascontiguousarray(rows[:, J["cl0"]:J["cl4"] + 1].astype(np.int32))
               if "cl0" in J else None)  # (fix_subpel_up: SUBPEL_TREE takes no cost list)
        yield F["cases"][ci], bw, bh, epb, rec, cls, rows, J
