"""CPU: the radix-2^29 Montgomery products (plonky3_eon_amd/csrc/field29.h: mul29 with eight
unmasked reduction multipliers, sqr29, mul29_sum2; and the NTT's Shoup product mul29_shoup with
its table pair shoup_pair29) compiled for the host and run on operands at
the edges of their contracts (tests/field29_check.cpp), checked against big integers:
r = a b 2^-261 mod p, r < 2p, limbs normalised.  The device code is the same C++ (its inline-asm
multiply-add is the host expression's one-instruction form), so an overflowing column sum or a
broken output bound fails here without a GPU."""

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"
P = {"fq": 21888242871839275222246405745257275088696311157297823662689037894645226208583,
     "fr": 21888242871839275222246405745257275088548364400416034343698204186575808495617}
RINV = {k: pow(2, -261, p) for k, p in P.items()}


def limbs(s: str) -> tuple[int, list[int]]:
    ls = [int(x, 16) for x in s.split(",")]
    return sum(v << (29 * i) for i, v in enumerate(ls)), ls


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    if not Path(HIPCC).exists() or shutil.which("g++") is None:
        pytest.skip("hipcc not available")
    exe = tmp_path_factory.mktemp("f29") / "field29_check"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                    "-I", str(ROOT / "plonky3_eon_amd" / "csrc"), str(ROOT / "tests" / "field29_check.cpp"),
                    "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe), "1500"], check=True, capture_output=True, text=True).stdout
    return [line.split() for line in out.splitlines() if line]


def check_out(field, want, r_str):
    p = P[field]
    r, rl = limbs(r_str)
    assert all(x < (1 << 29) for x in rl), rl
    assert r < 2 * p
    assert r % p == want % p


def test_products_at_contract_edges(results):
    seen = set()
    for f, op, *v in results:
        p, rinv = P[f], RINV[f]
        if op == "shoup":
            # twiddle pair from T = w 2^261 mod p, then r = y w mod p with r < 3p, exact
            (t, _), (y, _), (w, _), (wq, _), (r, rl) = (limbs(x) for x in v[:5])
            assert w < p and (w << 261) % p == t
            assert wq == (w << 261) // p
            assert all(x < (1 << 29) for x in rl)
            assert r < 3 * p and r % p == (y * w) % p
        elif op == "mul":
            (a, al), (b, bl) = limbs(v[0]), limbs(v[1])
            assert max(al + bl) < (1 << 30)
            check_out(f, a * b * rinv, v[2])
        elif op == "sqr":
            a, al = limbs(v[0])
            check_out(f, a * a * rinv, v[1])
        else:
            (a, _), (b, bl), (c, _), (d, _) = (limbs(x) for x in v[:4])
            assert max(bl) < (1 << 31)
            check_out(f, (a * b + c * d) * rinv, v[4])
        seen.add((f, op))
    assert seen == {(f, o) for f in P for o in ("mul", "sqr", "sum2")} | {("fr", "shoup")}
    # the widened operands really reach past 2^29 (the case the column bounds are about)
    assert any(max(limbs(v[0])[1]) >= (1 << 29) for f, op, *v in results if op == "mul")
    assert any(max(limbs(v[1])[1]) >= (1 << 30) for f, op, *v in results if op == "sum2")
