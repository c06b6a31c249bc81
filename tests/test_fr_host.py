"""CPU: the prove driver's host Fr arithmetic (plonky3_eon_amd/host/fr_host.h), which the
Fiat-Shamir transcript's Poseidon2 permutations run on (SURVEY.md 8(f) N2,
challenger/src/duplex_challenger.rs): the portable CIOS product, the MULX/ADCX/ADOX product (when
the CPU has BMI2 + ADX, and with EON_HOST_NO_ADX=1 forcing the portable one), the lazy addition
and the halving, checked with big integers on random and contract-edge operands (< 2r):
mul = a b 2^-256 mod r with the result < 2r, add = a + b mod r below 2r, half = a / 2 mod r below
2r, fr_mul canonical.  tests/fr_host_check.cpp prints the cases."""

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
RINV = pow(2, -256, R)


def _val(s: str) -> int:
    return sum(int(w, 16) << (64 * i) for i, w in enumerate(s.split(",")))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    out = tmp_path_factory.mktemp("frhost") / "fr_host_check"
    subprocess.run([cxx, "-O2", "-std=c++17", "-I", str(ROOT / "include"), "-I",
                    str(ROOT / "plonky3_eon_amd" / "host"), str(ROOT / "tests" / "fr_host_check.cpp"), "-o",
                    str(out)], check=True, capture_output=True)
    return out


def _check(exe, env_extra):
    env = dict(os.environ, **env_extra)
    p = subprocess.run([str(exe), "3000"], check=True, capture_output=True, text=True, env=env)
    counts = {}
    for line in p.stdout.splitlines():
        op, a, b, r = line.split()
        a, b, r = _val(a), _val(b), _val(r)
        counts[op] = counts.get(op, 0) + 1
        if op == "mul":
            assert r < 2 * R and r % R == a * b * RINV % R, (hex(a), hex(b))
        elif op == "fr_mul":
            assert r < R and r == a * b * RINV % R, (hex(a), hex(b))
        elif op == "add":
            assert r < 2 * R and r % R == (a + b) % R
        elif op == "half":
            assert r < 2 * R and (2 * r) % R == a % R
        else:
            raise AssertionError(op)
    return counts, p.stderr


def test_host_fr_default(exe):
    counts, err = _check(exe, {})
    assert counts["add"] == counts["half"] == 3064
    if "adx=1" in err:  # both products checked
        assert counts["mul"] == 3 * 3064


def test_host_fr_portable(exe):
    counts, err = _check(exe, {"EON_HOST_NO_ADX": "1"})
    assert "adx=0" in err and counts["mul"] == 3064
