"""bench.py's launcher contract on the CPU (no GPU touched).

`bench.py --gpus N` without WORLD_SIZE starts N fresh child processes itself
(one rank per GPU, env:// rendezvous on 127.0.0.1) and exits non-zero when
any rank fails; --dry-run prints that plan instead of starting it.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return e


def test_gpus_dry_run_plans_n_children():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "3"],
                         env=_env(), capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    plan = json.loads(out.stdout.strip().splitlines()[-1])
    assert plan["spawn"] == 2
    assert plan["cmd"][1] == BENCH and "--dry-run" not in plan["cmd"]
    assert plan["cmd"][2:] == ["--gpus", "2", "--steps", "3"]
    ranks = plan["ranks"]
    assert [r["RANK"] for r in ranks] == ["0", "1"]
    assert [r["LOCAL_RANK"] for r in ranks] == ["0", "1"]
    assert all(r["WORLD_SIZE"] == "2" and r["MASTER_ADDR"] == "127.0.0.1" for r in ranks)
    assert len({r["MASTER_PORT"] for r in ranks}) == 1


def test_gpus_eight_dry_run():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--dry-run"], env=_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    plan = json.loads(out.stdout.strip().splitlines()[-1])
    assert [r["RANK"] for r in plan["ranks"]] == [str(r) for r in range(8)]


def test_launcher_world_size_is_respected():
    """Under a launcher (WORLD_SIZE set) bench.py is one rank and starts
    nothing: with --dry-run it does not print a spawn plan."""
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "-c",
                          "import sys; sys.argv=['bench.py','--gpus','2','--dry-run'];"
                          "import importlib.util as u; s=u.spec_from_file_location('b', %r);"
                          "b=u.module_from_spec(s); s.loader.exec_module(b);"
                          "a=b.parse(); print(a.gpus > 1 and 'WORLD_SIZE' not in __import__('os').environ)"
                          % BENCH], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "False"


def test_failed_rank_fails_the_run():
    """Children that cannot run (here: no GPU) make the parent exit non-zero."""
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("needs a host without a GPU")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0",
                          "--no-cpu", "--no-c4"], env=_env(), capture_output=True, text=True,
                         timeout=300)
    assert out.returncode != 0
    assert "ranks failed" in out.stderr


def test_hw_queues_out_of_range_is_refused():
    """--hw-queues outside 0..32 is rejected by argparse before any GPU work
    (the runtime refused it only after the run had started)."""
    out = subprocess.run([sys.executable, BENCH, "--hw-queues", "-1", "--dry-run"], env=_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 2
    assert "--hw-queues" in out.stderr


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_cli_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_c4_counts_staleness_check():
    """bench.c4_roofline keeps profiles/c4_valu.json's issued-VALU / traffic
    fields only while every counted kernel still has the resource signature
    it was counted with (counters of rewritten kernels
    had been printed as current)."""
    import shutil
    import pytest
    if not shutil.which("c++filt") or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"):
        pytest.skip("no llvm tools")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_resources as KR
    b = _bench_module()
    lib = os.path.join(ROOT, "aom-av1-lavish_amd", "liblavish_hip.so")
    res = KR.kernel_resources(lib)
    names = sorted(res)
    name, mangled = next((d, n) for n, d in zip(names, KR.demangled(names)) if "rdo_kernel<4, 4" in d)
    short = name.replace("void ", "").replace("lavish::(anonymous namespace)::", "").split("(")[0]
    good = {"round": 6, "kernels": {short: {"signature": res[mangled]}}}
    assert b.c4_counts_stale(good) is None
    bad = {"round": 6, "kernels": {short: {"signature": dict(res[mangled], vgpr_count=1)}}}
    assert "changed" in b.c4_counts_stale(bad)
    gone = {"round": 6, "kernels": {"no_such_kernel<1>": {"signature": res[mangled]}}}
    assert b.c4_counts_stale(gone)
    assert b.c4_counts_stale({"valu_instr_per_step": 1, "kernels": {}})
