"""Self-check of the fixture pin: re-derive a sample of the committed golden
fixtures from the reference's own C text at test time
(tests/golden/cinterp.py over /root/reference), so the npz -> reference link
does not rest on gen_fixtures.py having been run once.

Only in the dev container: /root/reference does not exist on the GPU box, so
every test here skips there.  CPU only, a few seconds."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
REF = os.environ.get("LAVISH_REFERENCE", "/root/reference")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "av1")),
                                reason="reference sources absent (GPU box)")


@pytest.fixture(scope="module")
def G():
    sys.path.insert(0, GOLD)
    import gen_fixtures
    return gen_fixtures


def test_fwd_txfm_rederived(G):
    """av1_fwd_txfm2d_8x16_c re-executed on fix_txfm's stored inputs."""
    tu = G.tu_txfm()
    F = dict(np.load(os.path.join(GOLD, "fix_txfm.npz")))
    s = 7
    fn = tu.func("av1_fwd_txfm2d_%s_c" % G.TX_NAMES[s])
    W, H = G.TX_W[s], G.TX_H[s]
    for t in (0, 5, 12):
        for k in (0, 3, 7):
            blk, bd = F["in_%d_%d" % (s, t)][k], int(F["bd_%d_%d" % (s, t)][k])
            padded = np.zeros((H, W + 3), np.int16)
            padded[:, :W] = blk
            o = tu.buffer("int32_t", [0x5A5A5A5A] * (W * H))
            fn(tu.buffer("int16_t", padded.reshape(-1).tolist()), o, W + 3, t, bd)
            np.testing.assert_array_equal(np.array(o.buf, np.int32), F["out_%d_%d" % (s, t)][k])


def test_quantizer_rederived(G):
    """av1_build_quantizer (bd 8, sharpness 0) and av1_quantize_fp_32x32_c at
    qindex 128 re-executed on fix_quant's stored coefficients."""
    tu = G.tu_quant()
    Q = dict(np.load(os.path.join(GOLD, "fix_qparams.npz")))
    rows = G.build_quantizer(tu, 8, 0)
    for f, v in rows.items():
        np.testing.assert_array_equal(v, Q["%s_bd8_sh0" % f])
    F = dict(np.load(os.path.join(GOLD, "fix_quant.npz")))
    ci = [i for i, c in enumerate(G.QUANT_CASES) if c[0] == "av1_quantize_fp_32x32_c"][0]
    name, s, ls, hb, kind = G.QUANT_CASES[ci]
    scan, iscan = G.dct_scan(tu, s)
    n = G.max_eob(s)
    q = 128
    key = "%d_%d_q%d" % (ci, 8, q)
    for k in range(2):
        c = F["coeff_" + key][k]
        qp, dp = tu.buffer("int32_t", [77] * n), tu.buffer("int32_t", [77] * n)
        ep = tu.buffer("uint16_t", 1)
        i16 = lambda a: tu.buffer("int16_t", a.tolist())
        tu.func(name)(tu.buffer("int32_t", c.tolist()), n, i16(rows["y_zbin"][q]),
                      i16(rows["y_round_fp"][q]), i16(rows["y_quant_fp"][q]),
                      i16(rows["y_quant_shift"][q]), qp, dp, i16(rows["y_dequant_QTX"][q]), ep,
                      i16(scan), i16(iscan))
        np.testing.assert_array_equal(np.array(qp.buf, np.int32), F["qcoeff_" + key][k])
        np.testing.assert_array_equal(np.array(dp.buf, np.int32), F["dqcoeff_" + key][k])
        assert ep.buf[0] == F["eob_" + key][k]


def test_txfeat_rederived(G):
    """av1_get_horver_correlation_full_c on fix_txfeat's stored 16x16 blocks
    (float bit patterns)."""
    from cinterp import TU, reference_defines
    tu = TU(REF, ["aom/aom_integer.h", "aom_ports/mem.h", "aom_dsp/aom_dsp_common.h",
                  "av1/encoder/rdopt.c"], reference_defines(REF))
    if not tu.has_func("av1_get_horver_correlation_full_c"):
        tu = TU(REF, ["av1/encoder/encoder.h", "av1/encoder/rdopt.c"], reference_defines(REF))
    F = dict(np.load(os.path.join(GOLD, "fix_txfeat.npz")))
    hv = tu.func("av1_get_horver_correlation_full_c")
    done = 0
    for k, (s, w, h, kind, off) in enumerate(F["rows"]):
        if (w, h) != (16, 16):
            continue
        blk = F["blocks"][off:off + w * h]
        hc, vc = tu.buffer("float", 1), tu.buffer("float", 1)
        hv(tu.buffer("int16_t", blk.tolist()), w, w, h, hc, vc)
        got = np.array([hc.buf[0], vc.buf[0]], np.float32).view(np.int32)
        np.testing.assert_array_equal(got, F["features"][k][32:34])
        done += 1
    assert done >= 5
