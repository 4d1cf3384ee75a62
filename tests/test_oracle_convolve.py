"""CPU checks of the inter-prediction restatement (oracle/oracle_convolve.c):
its kernels against the reference's own tables (parsed from
av1/common/filter.h into tests/golden/ref_tables.json), the block-size filter
choice (filter.h:253-259), the single-prediction rounding
(get_conv_params_no_round), an independent pure-Python statement of the
convolve functions on small blocks, and exact invariants."""
import json
import os

import numpy as np
import pytest

import _oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
TABLES = json.load(open(os.path.join(HERE, "golden", "ref_tables.json")))["interp_filters"]
NAMES8 = ["av1_sub_pel_filters_8", "av1_sub_pel_filters_8smooth", "av1_sub_pel_filters_8sharp",
          "av1_bilinear_filters"]
NAMES4 = ["av1_sub_pel_filters_4", "av1_sub_pel_filters_4smooth", "av1_sub_pel_filters_4",
          "av1_bilinear_filters"]


@pytest.mark.parametrize("f", range(5))
@pytest.mark.parametrize("size", [2, 4, 8, 16, 128])
def test_kernels_match_reference_tables(f, size):
    for sp in range(16):
        k = O.interp_kernel(f, size, sp)
        if f == 4:
            exp = TABLES["av1_sub_pel_filters_12sharp"][sp]
        elif size <= 4:
            exp = TABLES[NAMES4[f]][sp]
        else:
            exp = TABLES[NAMES8[f]][sp]
        assert list(k) == exp
        assert int(np.sum(k)) == 128


def test_conv_rounds():
    assert O.conv_rounds(8) == (3, 11)
    assert O.conv_rounds(10) == (3, 11)
    assert O.conv_rounds(12) == (5, 9)


def _rpot(v, n):
    return (v + ((1 << n) >> 1)) >> n


def _py_convolve(src, off, ss, w, h, path, fx, fy, r0, r1, bd):
    """convolve.c:76-188 / 687-787 as plain Python loops."""
    flat = src.reshape(-1).astype(np.int64)
    mx = (1 << bd) - 1
    out = np.zeros((h, w), np.int64)
    tx, ty = len(fx), len(fy)
    foh, fov = tx // 2 - 1, ty // 2 - 1
    for y in range(h):
        for x in range(w):
            if path == 0:
                v = flat[off + y * ss + x]
            elif path == 1:
                s = sum(int(fx[k]) * int(flat[off + y * ss + x - foh + k]) for k in range(tx))
                v = _rpot(_rpot(s, r0), 7 - r0)
            elif path == 2:
                s = sum(int(fy[k]) * int(flat[off + (y - fov + k) * ss + x]) for k in range(ty))
                v = _rpot(s, 7)
            else:
                ob = bd + 14 - r0
                s = 1 << ob
                for k in range(ty):
                    hs = 1 << (bd + 6)
                    for m in range(tx):
                        hs += int(fx[m]) * int(flat[off + (y - fov + k) * ss + x - foh + m])
                    im = _rpot(hs, r0)
                    im = ((im + 32768) & 0xFFFF) - 32768
                    s += int(fy[k]) * im
                v = _rpot(_rpot(s, r1) - ((1 << (ob - r1)) + (1 << (ob - r1 - 1))),
                          14 - r0 - r1)
            out[y, x] = min(max(v, 0), mx)
    return out


@pytest.mark.parametrize("bd,dt", [(8, np.uint8), (10, np.uint16), (12, np.uint16)])
@pytest.mark.parametrize("path", [0, 1, 2, 3])
@pytest.mark.parametrize("f", [0, 1, 2, 3, 4])
def test_oracle_vs_python(bd, dt, path, f):
    rng = np.random.default_rng(bd * 100 + path * 10 + f)
    plane = rng.integers(0, 1 << bd, size=(24, 24)).astype(dt)
    r0, r1 = O.conv_rounds(bd)
    w, h = 8, 4
    off = 8 * 24 + 8
    sx, sy = int(rng.integers(1, 16)), int(rng.integers(1, 16))
    fx, fy = O.interp_kernel(f, w, sx), O.interp_kernel(f, h, sy)
    got = O.convolve_block(plane, off, 24, w, h, path, fx, fy, r0, r1, bd)
    exp = _py_convolve(plane, off, 24, w, h, path, fx, fy, r0, r1, bd)
    np.testing.assert_array_equal(got.astype(np.int64), exp)


@pytest.mark.parametrize("bd,dt", [(8, np.uint8), (12, np.uint16)])
def test_constant_plane_is_preserved(bd, dt):
    # every kernel sums to 128 and the 2-D offsets cancel: a flat plane stays flat
    r0, r1 = O.conv_rounds(bd)
    for c in (0, 1, (1 << bd) - 1, 77):
        plane = np.full((40, 40), c, dt)
        for f in range(5):
            for path in (1, 2, 3):
                fx, fy = O.interp_kernel(f, 16, 5), O.interp_kernel(f, 16, 11)
                out = O.convolve_block(plane, 12 * 40 + 12, 40, 16, 16, path, fx, fy, r0, r1, bd)
                assert (out == c).all()


def _bordered(W, H, B, dt, bd, seed):
    rng = np.random.default_rng(seed)
    stride = W + 2 * B
    plane = rng.integers(0, 1 << bd, size=(H + 2 * B, stride)).astype(dt)
    return plane, B * stride + B


def test_batch_positions_and_clamp():
    # init_subpel_params: integer mv -> copy of the shifted block; a huge mv is
    # clamped to (size + AOM_INTERP_EXTEND) / -(border - AOM_INTERP_EXTEND)
    W, H, B = 64, 48, 288
    plane, org = _bordered(W, H, B, np.uint8, 8, 3)
    stride = plane.shape[1]
    jobs = np.zeros(3, O.INTER_JOB)
    jobs["pix_row"], jobs["pix_col"] = [16, 16, 0], [8, 8, 0]
    jobs["mv_row"], jobs["mv_col"] = [8 * 3, 16000, -16000], [-8 * 5, 16000, -16000]
    jobs["dst_off"] = [0, 16, 32]
    out = O.build_inter_pred(plane, org, W, H, 0, 0, 16, 16, jobs, (16, 48))
    flat = plane.reshape(-1)

    def blk(r, c):
        return flat[org + r * stride + c + np.arange(16)[:, None] * stride + np.arange(16)]
    np.testing.assert_array_equal(out[:, :16], blk(16 + 3, 8 - 5))
    # clamp: pos = (H + 4) << 10 exactly -> integer position, copy path
    np.testing.assert_array_equal(out[:, 16:32], blk(H + 4, W + 4))
    np.testing.assert_array_equal(out[:, 32:], blk(-(B - 4), -(B - 4)))


def test_batch_chroma_subsampling_phase():
    # with ss = 1 the mv is in 1/16 chroma pel: odd mvs reach odd phases
    W, H, B = 32, 32, 144
    plane, org = _bordered(W, H, B, np.uint8, 8, 4)
    stride = plane.shape[1]
    r0, r1 = O.conv_rounds(8)
    jobs = np.zeros(1, O.INTER_JOB)
    jobs["pix_row"], jobs["pix_col"] = 8, 8
    jobs["mv_row"], jobs["mv_col"] = 3, 17
    out = O.build_inter_pred(plane, org, W, H, 1, 1, 8, 8, jobs, (8, 8))
    fx, fy = O.interp_kernel(0, 8, 1), O.interp_kernel(0, 8, 3)
    exp = O.convolve_block(plane, org + 8 * stride + 9, stride, 8, 8, 3, fx, fy, r0, r1, 8)
    np.testing.assert_array_equal(out, exp)
