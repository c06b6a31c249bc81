"""CPU: bench.py's launch logic (no GPU call happens on these paths)."""

import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _run(args, **env):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env)
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, cwd=ROOT, capture_output=True, text=True,
                          timeout=120, env=e)


def test_world_size_mismatch_is_an_error():
    out = _run(["--gpus", "4"], WORLD_SIZE="1")
    assert out.returncode == 2 and "WORLD_SIZE=1" in out.stderr
    assert out.stdout.strip() == ""


def test_zero_gpus_rejected():
    out = _run(["--gpus", "0"])
    assert out.returncode == 2


def test_self_launch_builds_the_launcher_command(monkeypatch):
    sys.path.insert(0, str(ROOT))
    import bench

    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "2"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.main() == 7  # the launcher's status is the exit status
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "2"]


def test_collective_choice():
    """The N > 1 prove uses the driver's RCCL communicator by default, torch.distributed when the
    ranks share a device or the backend is gloo, and whatever --collective names."""
    import bench

    assert bench.choose_collective("auto", {}) == "rccl"
    assert bench.choose_collective("auto", {"EON_BENCH_BACKEND": "nccl"}) == "rccl"
    assert bench.choose_collective("auto", {"EON_BENCH_ONE_DEVICE": "1"}) == "torch"
    assert bench.choose_collective("auto", {"EON_BENCH_BACKEND": "gloo"}) == "torch"
    assert bench.choose_collective("torch", {}) == "torch"
    assert bench.choose_collective("rccl", {"EON_BENCH_ONE_DEVICE": "1"}) == "rccl"
    args = bench.make_parser().parse_args([])
    assert args.collective == "auto" and not args.no_clock_probe
