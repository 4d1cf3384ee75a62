"""CPU tests of the product boundary (no GPU needed):
* liblavish_hip.so loads and exports every function include/lavish_dsp.h
  declares;
* host-side tables of the product (scan orders, quantizer rows, device
  constant header) equal the reference's (tests/golden/ref_tables.json) and
  the oracle's.
No compute call touches the GPU here."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

import _oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLES = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_tables.json")))


def _header_functions():
    """Function names declared by include/lavish_dsp.h after the C
    preprocessor has expanded its prototype macros."""
    import subprocess
    out = subprocess.run(["gcc", "-E", "-P", "-x", "c", os.path.join(ROOT, "include", "lavish_dsp.h")],
                         check=True, capture_output=True, text=True).stdout
    names = set(re.findall(r"\b(lavish_\w+|av1_\w+_hip|aom_\w+_hip)\s*\(", out))
    return sorted(names)


def test_library_exports_every_header_symbol():
    import lavish_dsp
    L = lavish_dsp.lib()
    missing = [n for n in _header_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert len(_header_functions()) >= 500


def test_scan_orders_match_reference():
    import lavish_dsp
    for s in range(19):
        for t in range(16):
            sc, isc = lavish_dsp.scan_order(s, t)
            sname, iname = TABLES["scan_orders"][s][t]
            np.testing.assert_array_equal(sc, TABLES["scans"][sname])
            np.testing.assert_array_equal(isc, TABLES["scans"][iname])


@pytest.mark.parametrize("bd", [8, 10, 12])
@pytest.mark.parametrize("sharp", [0, 3, -2])
def test_quant_params_match_oracle(bd, sharp):
    import lavish_dsp
    for q in range(0, 256, 5):
        o = O.quant_arrays(O.build_quant(bd, q, sharp))
        fp = lavish_dsp.build_quant_params(bd, q, lavish_dsp.QUANT_FP, sharp).as_dict()
        b = lavish_dsp.build_quant_params(bd, q, lavish_dsp.QUANT_B, sharp).as_dict()
        np.testing.assert_array_equal(fp["round"], o["round_fp"])
        np.testing.assert_array_equal(fp["quant"], o["quant_fp"])
        np.testing.assert_array_equal(b["round"], o["round"])
        np.testing.assert_array_equal(b["quant"], o["quant"])
        for k in ("zbin", "quant_shift", "dequant"):
            np.testing.assert_array_equal(fp[k], o[k])
            np.testing.assert_array_equal(b[k], o[k])


def test_device_constant_tables_match_reference():
    src = open(os.path.join(ROOT, "aom-av1-lavish_amd", "csrc", "txfm_consts.h")).read()
    def table(name):
        body = src[src.index(name + "["):]
        body = body[body.index("{"):body.index("};")]
        return [int(v) for v in re.findall(r"-?\d+", body)]
    assert table("kCospi") == [v for row in TABLES["cospi"] for v in row]
    assert table("kSinpi") == [v for row in TABLES["sinpi"] for v in row]


def test_qlookup_header_matches_reference():
    src = open(os.path.join(ROOT, "aom-av1-lavish_amd", "csrc", "qlookup_tables.h")).read()
    for cname, key in [("kDcQ8", "dc_qlookup_QTX"), ("kDcQ10", "dc_qlookup_10_QTX"),
                       ("kDcQ12", "dc_qlookup_12_QTX"), ("kAcQ8", "ac_qlookup_QTX"),
                       ("kAcQ10", "ac_qlookup_10_QTX"), ("kAcQ12", "ac_qlookup_12_QTX")]:
        body = src[src.index(cname + "[256]"):]
        body = body[body.index("{") + 1:body.index("}")]
        assert [int(v) for v in re.findall(r"-?\d+", body)] == TABLES[key]


def test_warp_tables_match_reference():
    """kWarpedFilter / kDivLut of the product's and the oracle's warp_tables.h
    against av1_warped_filter / div_lut parsed from the reference
    (av1/common/warped_motion.c:29-166, tests/golden/ref_tables.json)."""
    for path in (os.path.join(ROOT, "aom-av1-lavish_amd", "csrc", "warp_tables.h"),
                 os.path.join(ROOT, "oracle", "warp_tables.h")):
        src = open(path).read()
        body = src[src.index("kWarpedFilter[193][8]"):]
        body = body[body.index("{") + 1:body.index("};")]
        vals = [int(v) for v in re.findall(r"-?\d+", body)]
        assert vals == [v for row in TABLES["warped_filter"] for v in row]
        body = src[src.index("kDivLut[257]"):]
        body = body[body.index("{") + 1:body.index("};")]
        assert [int(v) for v in re.findall(r"-?\d+", body)] == TABLES["div_lut"]


def test_product_does_not_reference_oracle():
    """The product tree must not include, link or load anything in oracle/."""
    pk = os.path.join(ROOT, "aom-av1-lavish_amd")
    for dirpath, _, files in os.walk(pk):
        for f in files:
            if f.endswith((".hip", ".h", ".py", ".cpp")) or f == "Makefile":
                txt = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "oracle" not in txt.replace("oracle/ never", ""), os.path.join(dirpath, f)


@pytest.mark.parametrize("bd", [8, 10, 12])
@pytest.mark.parametrize("sharp", [0, 3, -3])
def test_quant_params_match_reference_execution(bd, sharp):
    """lavish_build_quant_params against av1_build_quantizer as the
    reference's own code computes it (tests/golden/fix_qparams.npz, made by
    executing av1/encoder/av1_quantize.c:602-686), every qindex."""
    import lavish_dsp
    F = dict(np.load(os.path.join(ROOT, "tests", "golden", "fix_qparams.npz")))
    for q in range(256):
        fp = lavish_dsp.build_quant_params(bd, q, lavish_dsp.QUANT_FP, sharp).as_dict()
        b = lavish_dsp.build_quant_params(bd, q, lavish_dsp.QUANT_B, sharp).as_dict()
        row = lambda f: F["%s_bd%d_sh%d" % (f, bd, sharp)][q, :2]
        np.testing.assert_array_equal(fp["round"], row("y_round_fp"))
        np.testing.assert_array_equal(fp["quant"], row("y_quant_fp"))
        np.testing.assert_array_equal(b["round"], row("y_round"))
        np.testing.assert_array_equal(b["quant"], row("y_quant"))
        for d in (fp, b):
            np.testing.assert_array_equal(d["zbin"], row("y_zbin"))
            np.testing.assert_array_equal(d["quant_shift"], row("y_quant_shift"))
            np.testing.assert_array_equal(d["dequant"], row("y_dequant_QTX"))


def test_shear_params_host_matches_reference():
    """lavish_get_shear_params (host code of the product, no GPU) against
    av1_get_shear_params executed from the reference (fix_warp.npz)."""
    lib = ctypes.CDLL(os.path.join(ROOT, "aom-av1-lavish_amd", "liblavish_hip.so"))
    lib.lavish_get_shear_params.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.lavish_get_shear_params.restype = ctypes.c_int
    F = np.load(os.path.join(ROOT, "tests", "golden", "fix_warp.npz"))
    n_ok = 0
    for row in F["shear"]:
        m = np.ascontiguousarray(row[1:7], np.int32)
        out = np.zeros(4, np.int16)
        ok = lib.lavish_get_shear_params(m.ctypes.data_as(ctypes.c_void_p),
                                         out.ctypes.data_as(ctypes.c_void_p))
        assert (ok,) + tuple(int(v) for v in out) == tuple(int(v) for v in (row[0], *row[7:11]))
        n_ok += ok
    assert n_ok > len(F["shear"]) // 2


@pytest.mark.parametrize("f", range(5))
@pytest.mark.parametrize("size", [2, 4, 8, 16, 128])
def test_interp_kernels_match_reference_tables(f, size):
    """lavish_interp_kernels = av1_get_interp_filter_params_with_block_size
    (filter.h:253-259) over the reference's own kernel tables (filter.h)."""
    import lavish_dsp.inter as I
    names8 = ["av1_sub_pel_filters_8", "av1_sub_pel_filters_8smooth",
              "av1_sub_pel_filters_8sharp", "av1_bilinear_filters"]
    names4 = ["av1_sub_pel_filters_4", "av1_sub_pel_filters_4smooth", "av1_sub_pel_filters_4",
              "av1_bilinear_filters"]
    F = TABLES["interp_filters"]
    exp = F["av1_sub_pel_filters_12sharp"] if f == 4 else \
        (F[names4[f]] if size <= 4 else F[names8[f]])
    np.testing.assert_array_equal(I.interp_kernels(f, size), np.array(exp, np.int16))


def test_swar_nz_mag_identity():
    """The rate mode of rdo_kernel (csrc/rdo.hip, MODE 3) forms get_nz_mag's
    clipped neighbour sums for 8 positions per 32-bit word: each 4-bit level
    clipped to 3 as (x & 3) | 3 * (bit 2 | bit 3), then the class's five
    neighbour words (nibble shifts across words) added without carries.
    Check that arithmetic against the per-position sum for random level maps
    of every class and row width."""
    import numpy as np
    rng = np.random.default_rng(7)
    M = 0xFFFFFFFF

    def words(levels):  # 4-bit levels (clipped to 15) -> packed words, 8 per word
        n = (len(levels) + 7) // 8
        w = [0] * n
        for c, v in enumerate(levels):
            w[c >> 3] |= min(int(v), 15) << (4 * (c & 7))
        return w

    def min3w(w):
        out = []
        for x in w:
            f = ((x >> 2) | (x >> 3)) & 0x11111111
            out.append((x & 0x33333333) | f | ((f << 1) & M))
        return out

    def sh(m, w, k):
        return ((m[w] >> (4 * k)) | (((m[w + 1] << (32 - 4 * k)) & M) if w + 1 < len(m) else 0)) & M

    for KW in (4, 8, 16, 32):
        for _ in range(200):
            rows = [rng.integers(0, 20, KW) * (rng.random(KW) < 0.5) for _ in range(5)]
            m = [min3w(words(r)) for r in rows]
            NW = len(m[0])
            nib = lambda d, c: min(int(rows[d][c]), 15) if c < KW else 0
            for cls in range(3):
                for w in range(NW):
                    base = sh(m[0], w, 1) + m[1][w]
                    s = (base + sh(m[1], w, 1) + sh(m[0], w, 2) + m[2][w] if cls == 0 else
                         base + sh(m[0], w, 2) + sh(m[0], w, 3) + sh(m[0], w, 4) if cls == 1 else
                         base + m[2][w] + m[3][w] + m[4][w]) & M
                    for k in range(8):
                        c = 8 * w + k
                        if c >= KW:
                            continue
                        mn = lambda v: min(v, 3)
                        exp = mn(nib(0, c + 1)) + mn(nib(1, c))
                        exp += (mn(nib(1, c + 1)) + mn(nib(0, c + 2)) + mn(nib(2, c)) if cls == 0
                                else mn(nib(0, c + 2)) + mn(nib(0, c + 3)) + mn(nib(0, c + 4))
                                if cls == 1 else mn(nib(2, c)) + mn(nib(3, c)) + mn(nib(4, c)))
                        assert (s >> (4 * k)) & 15 == exp, (KW, cls, c)


def _kernel_resources_by_name():
    import shutil
    import sys
    if not os.path.exists("/opt/rocm/lib/llvm/bin/clang-offload-bundler") or \
            shutil.which("c++filt") is None:
        pytest.skip("ROCm code-object tools not present")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_resources as KR
    lib = os.path.join(ROOT, "aom-av1-lavish_amd", "liblavish_hip.so")
    res = KR.kernel_resources(lib)
    dm = dict(zip(sorted(res), KR.demangled(sorted(res))))
    return {dm[n]: v for n, v in res.items()}


def test_benched_kernels_no_scratch():
    """Code-object metadata of the kernels on the benched paths (the
    library's gfx950 images, tools/kernel_resources.py): the C3 search, the
    C2 multi-size kernels and every inverse tile kernel use no scratch."""
    by = _kernel_resources_by_name()
    checked = 0
    for name, v in by.items():
        if any(k in name for k in ("diamond_lj_kernel", "txq_multi_kernel", "inv_tile_kernel",
                                   "ref_tiles_kernel", "mvcost_dec_kernel", "sb_decide_kernel")):
            assert v.get("private_segment_fixed_size", 0) == 0, name
            checked += 1
    assert checked >= 80


@pytest.mark.xfail(strict=False, reason="perf-regression pin, not correctness: exact VGPR / "
                   "spill counts move with the toolchain")
def test_rdo_decision_kernels_spill_pin():
    """The C4 decision kernels' registers, spills, scratch and LDS as
    profiles/r06_rdo_kernel_resources.json recorded them (round 6: all
    spill-free at their occupancy requests but the 32x32 split-form build,
    14 VGPRs) -- a
    toolchain or code change that moves them shows here (XFAIL) and calls
    for re-measuring the occupancy requests (profiles/r04_v2_rdo_occupancy_ab.json
    measured the requests against spill-free ones in round 4)."""
    by = _kernel_resources_by_name()
    pin = json.load(open(os.path.join(ROOT, "profiles", "r06_rdo_kernel_resources.json")))
    for name, v in pin["kernels"].items():
        got = by[name]
        for k in ("vgpr_count", "vgpr_spill_count", "private_segment_fixed_size",
                  "group_segment_fixed_size"):
            assert got.get(k) == v.get(k), (name, k, got.get(k), v.get(k))


@pytest.mark.xfail(strict=False, reason="perf-regression pin, not correctness: exact SGPR "
                   "spill counts move with the toolchain")
def test_search_kernels_sgpr_spill_pin():
    """SGPR spills of the latency-bound search kernels as round 6 left them
    (DESIGN.md §4): diamond_lj_kernel 21 (parked at entry, none reloaded in
    the step loop), tpl_mv_kernel<false> / <true> 130 / 142 (kernel
    arguments parked in VGPR lanes, none reloaded in the candidate rounds).
    A change that raises them shows here (XFAIL) and calls for checking
    where the new reloads land."""
    by = _kernel_resources_by_name()
    pin = {"diamond_lj_kernel<4>": 21, "diamond_lj_dyn_kernel<4>": 21,
           "tpl_mv_kernel<false>": 130, "tpl_mv_kernel<true>": 142}
    seen = set()
    for name, v in by.items():
        for k, n in pin.items():
            if k in name:
                assert v.get("sgpr_spill_count", 0) <= n, (name, v.get("sgpr_spill_count"))
                seen.add(k)
    assert seen == set(pin)
