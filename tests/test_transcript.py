"""The Fiat-Shamir transcript of libeonprove -- Poseidon2Bn254<3>, the
DuplexChallenger and the compressed G1 observation -- against the oracle's restatement
(oracle/pyoracle.py: p2_permute, DuplexChallenger, g1_compressed).  Host code only: runs on CPU.

Pinning: the permutation is pinned to the AIR's own trace generation (its last three columns are
the permutation output, poseidon2-air/src/generation.rs), itself checked against the constraint
set; the challenger follows duplex_challenger.rs line by line; the compressed G1 bytes are
halo2curves' encoding, absent here -- parity unpinned (documented choice)."""

import numpy as np
import pytest

from oracle import coracle as C
from oracle import pyoracle as O
from plonky3_eon_amd import _lib

native = pytest.importorskip("plonky3_eon_amd.native")
if not native.PROVE_LIB_PATH.exists():
    pytest.skip("libeonprove.so not built", allow_module_level=True)


def lim(x):
    return np.array(O.int_to_limbs(O.to_mont(x % O.P)), dtype=np.uint64)


def unlim(a):
    return O.from_mont(O.limbs_to_int([int(v) for v in a]))


def consts(seed, hf, pr):
    py = O.p2_constants(seed, hf, pr)
    k = native.Poseidon2Constants([[lim(x) for x in r] for r in py[0]], [lim(x) for x in py[1]],
                                  [[lim(x) for x in r] for r in py[2]])
    return py, k


def test_oracle_permutation_is_the_air_trace_output():
    py = O.p2_constants(7, 4, 56)
    for seed in range(3):
        rng = O.SplitMix64(seed)
        inp = [O.from_mont(rng.fr_mont()) for _ in range(3)]
        row = O.p2_trace_row(inp, py)
        assert O.p2_permute(inp, py) == row[-3:]
        assert all(c == 0 for c in O.p2_constraints(row, py))


@pytest.mark.parametrize("hf,pr", [(4, 56), (2, 22), (0, 3), (1, 0)])
def test_permutation_matches_oracle(hf, pr):
    py, k = consts(100 + hf + pr, hf, pr)
    rng = np.random.default_rng(hf * 100 + pr)
    for _ in range(8):
        st = [int(rng.integers(0, 2**62)) * int(rng.integers(1, 2**62)) % O.P for _ in range(3)]
        got = native.poseidon2_permute(k, np.stack([lim(x) for x in st]))
        assert [unlim(r) for r in got] == O.p2_permute(st, py)


def test_permutation_matches_trace_generation_in_c():
    """The same constants through the C oracle's trace generation (the AIR path): last 3 columns."""
    py, k = consts(5, 4, 56)
    ck = C.P2Constants(k.begin, k.partial, k.end)
    inputs = C.random_fr(9, 6).reshape(2, 3, 4)
    tr = C.p2_generate_trace(inputs, 1, ck)
    for j in range(2):
        np.testing.assert_array_equal(native.poseidon2_permute(k, inputs[j]), tr[j, -3:])


def test_challenger_observe_sample_sequences():
    py, k = consts(11, 4, 56)
    ch, ref = native.Challenger(k), O.DuplexChallenger(py)
    rng = np.random.default_rng(3)
    for step in range(60):
        op = rng.integers(0, 3)
        if op < 2:
            n = int(rng.integers(1, 4))
            vals = [int(rng.integers(0, 2**63)) * int(rng.integers(1, 2**63)) % O.P for _ in range(n)]
            ch.observe(np.stack([lim(v) for v in vals]))
            for v in vals:
                ref.observe(v)
        else:
            assert unlim(ch.sample()) == ref.sample(), f"step {step}"
        assert [unlim(r) for r in ch.state()] == ref.state
    ch.close()


def test_challenger_sample_before_observe_and_twice():
    py, k = consts(12, 4, 56)
    ch, ref = native.Challenger(k), O.DuplexChallenger(py)
    for _ in range(5):  # empty input buffer: duplex on an empty output, then pop twice
        assert unlim(ch.sample()) == ref.sample()


def _g1_points(n, seed):
    rng = np.random.default_rng(seed)
    g = (1, 2)
    pts = [O.g1_mul(g, int(rng.integers(1, 2**62))) for _ in range(n)]
    return pts + [O.INF, O.g1_neg(pts[0])]


def test_g1_compressed_bytes_match_oracle():
    for p in _g1_points(6, 1):
        abi = np.frombuffer(O.g1_to_bytes(p), dtype=np.uint64)
        b = native.g1_to_bytes(abi)
        assert b == O.g1_compressed(p)
        if p is not O.INF:
            assert int.from_bytes(b, "little") & ((1 << 254) - 1) == p[0]
    # y and -y differ only in the sign bit
    p = _g1_points(1, 2)[0]
    a = native.g1_to_bytes(np.frombuffer(O.g1_to_bytes(p), dtype=np.uint64))
    b = native.g1_to_bytes(np.frombuffer(O.g1_to_bytes(O.g1_neg(p)), dtype=np.uint64))
    assert a[:31] == b[:31] and (a[31] ^ b[31]) == 0x80


def test_challenger_observes_commitments_like_oracle():
    py, k = consts(13, 4, 56)
    ch, ref = native.Challenger(k), O.DuplexChallenger(py)
    pts = _g1_points(5, 3)
    abi = np.stack([np.frombuffer(O.g1_to_bytes(p), dtype=np.uint64) for p in pts])
    ch.observe(lim(17))
    ref.observe(17)
    ch.observe_g1(abi)
    ref.observe_g1(pts)
    assert unlim(ch.sample()) == ref.sample()
    assert [unlim(r) for r in ch.state()] == ref.state


def test_errors():
    py, k = consts(14, 2, 3)
    ch = native.Challenger(k)
    bad = np.array(O.int_to_limbs(O.P), dtype=np.uint64)  # r itself is not canonical
    with pytest.raises(_lib.EonError):
        ch.observe(bad)
    kb = native.Poseidon2Constants(np.stack([bad] * 3).reshape(1, 3, 4), np.zeros((0, 4), np.uint64),
                                   np.zeros((1, 3, 4), np.uint64))
    with pytest.raises(_lib.EonError):
        native.Challenger(kb)
