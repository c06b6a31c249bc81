"""CPU: the host-side Fq inverse msm.hip converts MSM results with (plonky3_eon_amd/csrc/fq_host.h;
binary extended Euclid): inverse(x 2^256) = x^-1 2^256 mod q for canonical and
non-canonical inputs, and 0 for a = 0 mod q (0, q, 2q -- the loop must end instead of spinning on
u = 0), against Python's pow; plus the CIOS product it relies on."""

import random
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 1 << 256


def _hex(v: int) -> str:
    return ",".join("%x" % ((v >> (64 * i)) & ((1 << 64) - 1)) for i in range(4))


def _val(s: str) -> int:
    return sum(int(w, 16) << (64 * i) for i, w in enumerate(s.split(",")))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    out = tmp_path_factory.mktemp("fqhost") / "fq_host_check"
    subprocess.run([cxx, "-O2", "-std=c++17", "-I", str(ROOT / "plonky3_eon_amd" / "csrc"),
                    str(ROOT / "tests" / "fq_host_check.cpp"), "-o", str(out)], check=True, capture_output=True)
    return out


def test_inverse_and_product(exe):
    rng = random.Random(5)
    cases = [0, Q, 2 * Q, 1, 2, Q - 1, Q + 1, R - 1, R % Q, (R * R) % Q]
    cases += [rng.randrange(Q) for _ in range(200)] + [rng.randrange(R) for _ in range(50)]
    out = subprocess.run([str(exe)], input="".join(_hex(a) + "\n" for a in cases), capture_output=True, text=True,
                         check=True, timeout=60).stdout.split("\n")
    for a, line in zip(cases, out):
        inv_s, sq_s = line.split()
        inv, sq = _val(inv_s), _val(sq_s)
        if a % Q == 0:
            assert inv == 0, (a, inv)
        else:
            # a = x 2^256: the result must be x^-1 2^256 = 2^512 / a
            assert inv == (pow(a, Q - 2, Q) * R * R) % Q, a
        if a < Q:  # the CIOS product's contract: canonical operands
            assert sq == (a * a * pow(R, -1, Q)) % Q, a
