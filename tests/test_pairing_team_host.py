"""CPU: the team-parallel Fq12 lanes of the verifier's pairings (plonky3_eon_amd/csrc/pairing_team.h)
compiled for the host (tests/team_check.cpp): each operation's six per-lane COMPUTE halves, run
in turn on the published slots, rebuild exactly the tower's sequential result (pairing.h: f12_mul,
f12_sqr, f12_cyc_sqr, f12_mul_line, the vertical-line product, f12_frob<1,2,3>, f12_conj) on
random elements.  The kernels that exchange the slots (pairing.hip k_miller_team /
k_final_exp_team) are pinned against the pairing oracle on the GPU (tests/test_gpu_pairing.py)."""

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"


def test_team_lanes_match_tower(tmp_path):
    if not Path(HIPCC).exists() or shutil.which("g++") is None:
        pytest.skip("hipcc not available")
    exe = tmp_path / "team_check"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                    "-I", str(ROOT / "plonky3_eon_amd" / "csrc"), str(ROOT / "tests" / "team_check.cpp"),
                    "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe), "40"], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok 40", out.stdout + out.stderr
