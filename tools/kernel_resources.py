#!/usr/bin/env python3
"""Per-kernel resources of liblavish_hip.so's gfx950 code object: VGPR /
AGPR / SGPR counts, spill counts, scratch (private segment) and LDS (group
segment) bytes, from the AMDGPU metadata note (llvm-readelf --notes) of the
device image in the library's .hip_fatbin section.

usage: kernel_resources.py [LIB] [OUT_JSON]   (prints a summary; writes JSON
when OUT_JSON is given).  Used by tests/test_capi_cpu.py to check that no
kernel of the C4 decision path touches scratch."""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
KEYS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
        "private_segment_fixed_size", "group_segment_fixed_size")


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _notes(co):
    return subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                          capture_output=True, text=True).stdout


def kernel_resources(lib):
    """{mangled kernel name: {key: int}} for every kernel in lib's gfx950
    images (the .hip_fatbin section holds one offload bundle per
    translation unit, back to back)."""
    notes = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat,
                        lib, os.path.join(d, "junk")], check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, a in enumerate(starts):
            b = starts[i + 1] if i + 1 < len(starts) else len(data)
            one, co = os.path.join(d, "b%d" % i), os.path.join(d, "co%d" % i)
            open(one, "wb").write(data[a:b])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o",
                            "--input=" + one, "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            "--output=" + co, "--unbundle"], check=True, capture_output=True)
            notes.append(_notes(co))
    out = {}
    # the metadata lists one mapping per kernel ("  - .agpr_count: ..." starts one)
    for block in re.split(r"\n\s+- \.", "\n".join(notes)):
        m = re.search(r"\.?name:\s+(\S+)", block)
        if m is None or ".symbol:" not in block:
            continue
        vals = {}
        for k in KEYS:
            mm = re.search(r"(?:^|\s|\.)" + k + r":\s+(\d+)", block)
            if mm:
                vals[k] = int(mm.group(1))
        out[m.group(1)] = vals
    return out


def demangled(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    except OSError:
        return list(names)
    return r.stdout.split("\n") if r.returncode == 0 else list(names)


def main(lib=None, out=None):
    lib = lib or os.path.join(ROOT, "aom-av1-lavish_amd", "liblavish_hip.so")
    res = kernel_resources(lib)
    names = sorted(res)
    dm = demangled(names)
    table = {d or n: res[n] for n, d in zip(names, dm)}
    for k, v in table.items():
        if "rdo_kernel" in k or "inv_tile_kernel<64" in k or v.get("private_segment_fixed_size"):
            print("%-90s vgpr %3d agpr %3d scratch %4d spill %d/%d" % (
                k[:90], v.get("vgpr_count", -1), v.get("agpr_count", -1),
                v.get("private_segment_fixed_size", -1), v.get("vgpr_spill_count", -1),
                v.get("sgpr_spill_count", -1)))
    if out:
        with open(out, "w") as f:
            json.dump({"library": os.path.relpath(lib, ROOT), "kernels": table}, f, indent=1,
                      sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
