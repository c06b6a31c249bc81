"""GPU: bench.py keeps its output contract (the driver parses it): exactly one JSON line with the
required keys, `roofline` (bound / achieved / peak / unit / frac / traffic, frac = achieved / peak)
and `cpu_baseline` (value / unit / cores / kind / sample).  Runs the quick configs[2] workload and
a small GPU verify_batch (N4; its single-thread pairing chains report the bound "latency")."""

import json
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("extra", [["--workload", "msm"],
                                   ["--workload", "verify", "--log-trace", "6", "--vector-len", "1"]])
def test_bench_json_contract(extra):
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), *extra, "--steps", "3", "--warmup", "1"],
                         cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is False and d["scaling"] in ("weak", "strong")
    assert "workload" in d["config"]
    r = d["roofline"]
    assert r["bound"] in ("hbm", "mfma", "valu", "latency") and r["unit"] in ("GB/s", "TFLOP/s")
    if r["bound"] == "valu":  # the binding integer roofline beside the HBM figures
        v = r["valu"]
        assert v["unit"] == "mulmod/s" and 0 < v["frac"] <= 1.2 and r["hbm_frac"] == r["frac"]
    assert r["peak"] == 8000.0 and r["achieved"] > 0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert "traffic" in r
    c = d["cpu_baseline"]
    assert c["value"] > 0 and c["cores"] >= 1 and c["kind"] in ("reference", "port") and c["sample"]


@pytest.mark.parametrize("gpus,extra", [
    (2, ["--workload", "ntt4", "--log-ntt", "16"]),
    # the driver's multi-GPU configuration of the headline (lane-sharded prove), small trace
    (2, ["--log-trace", "8", "--vector-len", "2"]),
    (4, ["--log-trace", "8", "--vector-len", "8"]),
])
def test_bench_self_launch_ranks(gpus, extra):
    """`bench.py --gpus N` with no launcher starts its own N ranks (here gloo ranks sharing cuda:0,
    EON_BENCH_BACKEND=gloo EON_BENCH_ONE_DEVICE=1) and rank 0 prints n_gpus N."""
    import os

    env = dict(os.environ, EON_BENCH_BACKEND="gloo", EON_BENCH_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), *extra,
                          "--steps", "2", "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=240,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == gpus and d["steps"] == 2 and d["cpu_baseline"] is None
    assert d["value"] > 0 and d["roofline"]["achieved"] > 0
    # the per-rank evidence of an N > 1 line: every rank's record, here all on the one device
    ranks = d["ranks"]
    assert [r["rank"] for r in ranks] == list(range(gpus))
    assert d["distinct_gpus"] == 1 and all(r["device"] == 0 and r["pci_bus_id"] for r in ranks)
    assert all(r["collective"] == "torch" and r["ms_per_step"] > 0 for r in ranks)
    assert max(r["ms_per_step"] for r in ranks) <= d["ms_per_step"] + 1e-3
    if "--workload" not in extra:  # the prove's stages, per rank
        assert all("commit to trace data" in r["stage_ms"] for r in ranks)
