"""CPU: the C restatement of the per-SB TX-size decision + reconstruction
(orc_rdo_reconstruct, bench.py's C4 baseline) equals the numpy composition
the GPU tests use."""
import numpy as np

import _c4ref


def test_c_reconstruct_matches_numpy():
    src, pred = _c4ref.planes(10, 3, Wp=200, Hp=136)
    masks = {4: 0x1, 3: 0x201, 2: 0xFFFF, 1: 0x11, 0: 0x3}
    _, ch1, rec1 = _c4ref.oracle_frame(src, pred, 10, masks, 1800, threads=4)
    _, ch2, rec2 = _c4ref.oracle_frame_c(src, pred, 10, masks, 1800, threads=4)
    np.testing.assert_array_equal(ch1, ch2)
    np.testing.assert_array_equal(rec1, rec2)
    assert (rec1 != pred).any()
