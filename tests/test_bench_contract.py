"""The bench line's contract, checked on CPU against the committed round
evidence (profiles/r*_bench.json, written by `python bench.py` on the GPU
box): the keys the driver reads, the roofline and cpu_baseline objects, and
the arithmetic between them (value = mults per step / time; frac =
achieved / peak; the rocprofv3 kernel stats of the same tree agree with the
in-bench launch time)."""
import csv
import glob
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILES = os.path.join(ROOT, "profiles")


def round_key(path):
    m = re.search(r"r(\d+)([a-z]?)_bench\.json$", os.path.basename(path))
    return (int(m.group(1)), m.group(2)) if m else (-1, "")


def latest_bench():
    files = [f for f in glob.glob(os.path.join(PROFILES, "r*_bench.json")) if round_key(f)[0] >= 0]
    if not files:
        pytest.skip("no committed bench line")
    return max(files, key=round_key)


def test_bench_line_keys_and_arithmetic():
    path = latest_bench()
    d = json.load(open(path))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, (path, k)
    assert d["unit"] == "mults/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["vs_baseline"] is None  # BASELINE.md publishes no number for this metric
    assert d["dtype"] == "int64"
    assert "workload" in d["config"]
    # value is the whole job's mults per second: 1024^3 multiplications per step
    mults = 1024 ** 3 * d["n_gpus"]
    assert d["value"] == pytest.approx(mults / (d["ms_per_step"] / 1e3), rel=1e-6)
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "mfma" and r["unit"] == "TOP/s"
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-9)
    assert 0 < r["frac"] < 1
    # achieved = the launch's algorithmic int8 ops / its measured duration
    assert r["achieved"] == pytest.approx(r["ops_per_launch"] / (r["launch_ms"] / 1e3) / 1e12, rel=1e-6)
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0


def test_rocprof_summary_agrees_with_bench_launch_time():
    """The committed kernel stats of the same tag time the share GEMM as the
    bench's own HIP events did (the roofline's launch duration)."""
    path = latest_bench()
    stats = path.replace("_bench.json", "_kernel_stats.csv")
    if not os.path.exists(stats):
        pytest.skip("no kernel stats beside " + os.path.basename(path))
    d = json.load(open(path))
    avg_ms = None
    for row in csv.DictReader(open(stats)):
        if "k_share_gemm16s" in row["Name"]:
            avg_ms = float(row["AverageNs"]) / 1e6
    assert avg_ms is not None, "no share-GEMM row in " + stats
    assert avg_ms == pytest.approx(d["roofline"]["launch_ms"], rel=0.1)


def _pmc_summary():
    import importlib.util
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "scripts", "pmc_summary.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _latest_with(pattern):
    files = [f for f in glob.glob(os.path.join(PROFILES, pattern))
             if re.search(r"r(\d+)([a-z]?)", os.path.basename(f))]
    if not files:
        pytest.skip("no " + pattern)
    key = lambda f: (lambda m: (int(m.group(1)), m.group(2)))(re.search(r"r(\d+)([a-z]?)", os.path.basename(f)))
    return max(files, key=key)


def test_binary_traffic_sums_every_level_kernel():
    """The binary roofline's traffic (pmc_*.json bin_gates) is the sum of every
    gate-level kernel's PMC bytes: each k_bin_* kernel the committed kernel
    stats name is counted by pmc_summary.py and present in the PMC table."""
    ps = _pmc_summary()
    pmc_path = _latest_with("pmc_r*.json")
    pmc = json.load(open(pmc_path))
    if "msb" not in pmc.get("kernels", {}):
        pytest.skip("no msb kernel table in " + pmc_path)
    table = pmc["kernels"]["msb"]
    tag = re.search(r"pmc_(r\d+[a-z]?)\.json", os.path.basename(pmc_path)).group(1)
    stats = os.path.join(PROFILES, tag + "_kernel_stats.csv")
    if os.path.exists(stats):
        for row in csv.DictReader(open(stats)):
            m = re.search(r"\b(k_bin_[A-Za-z0-9_]+)", row["Name"])
            if m:
                assert ps.is_level_kernel(m.group(1)), m.group(1) + " is a gate kernel the traffic sum leaves out"
                assert m.group(1) in table, m.group(1) + " has no PMC bytes in " + pmc_path
    want = sum(v["read_bytes"] + v["write_bytes"] for k, v in table.items() if k.startswith("k_bin_"))
    assert want > 0
    # 4 profiled steps of three parties (scripts/gpu_profile.sh)
    assert pmc["bin_gates"]["hbm_bytes_per_step_per_party"] == pytest.approx(want / 12, rel=1e-9)
    assert ps.bin_level_bytes(table) == pytest.approx(want, rel=1e-12)
