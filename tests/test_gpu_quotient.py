"""GPU parity of the Poseidon2-AIR trace generation, selectors_on_coset and quotient_values
(eon-uni-stark/src/prover.rs:539-709) against the C restatement oracle."""

import numpy as np
import pytest

from oracle import coracle as C
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu
HF, PR = 4, 56


def lim(x):
    return np.array(O.int_to_limbs(O.to_mont(x)), dtype=np.uint64)


@pytest.fixture(scope="module")
def consts():
    py = O.p2_constants(77, HF, PR)
    return C.P2Constants([[lim(x) for x in r] for r in py[0]], [lim(x) for x in py[1]],
                         [[lim(x) for x in r] for r in py[2]])


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda:0")


def host(t):
    return t.cpu().numpy().view(np.uint64)


def make_air(consts, vl, ctx):
    from plonky3_eon_amd.air import Poseidon2Air

    return Poseidon2Air(consts.begin, consts.partial, consts.end, vl, ctx)


@pytest.mark.parametrize("vl,n", [(1, 64), (8, 256), (2, 2)])
def test_trace_generation(gpu_ctx, consts, vl, n):
    inputs = C.random_fr(n + vl, n * 3).reshape(n, 3, 4)
    air = make_air(consts, vl, gpu_ctx)
    assert air.width == 164 * vl
    got = host(air.generate_trace(dev(inputs)))
    np.testing.assert_array_equal(got, C.p2_generate_trace(inputs, vl, consts))


@pytest.mark.parametrize("log_n,log_q", [(3, 4), (4, 6), (10, 11)])
def test_selectors(gpu_ctx, log_n, log_q):
    from plonky3_eon_amd.air import selectors_on_coset

    got = host(selectors_on_coset(log_n, log_q, 5, ctx=gpu_ctx))
    np.testing.assert_array_equal(got, C.selectors_on_coset(log_n, log_q, C.fr_from_u64(5)))


@pytest.mark.parametrize("vl,log_n", [(1, 3), (8, 3), (8, 6), (1, 9)])
def test_quotient_values(gpu_ctx, consts, vl, log_n):
    n = 1 << log_n
    inputs = C.random_fr(log_n * 10 + vl, n * vl * 3).reshape(n * vl, 3, 4)
    trace = C.p2_generate_trace(inputs, vl, consts)
    lde = C.coset_lde_batch(trace, 1, C.fr_from_u64(5))
    alpha = C.random_fr(5, 1)[0]
    want = C.p2_quotient_values(lde, log_n, 1, vl, consts, alpha)
    air = make_air(consts, vl, gpu_ctx)
    got = host(air.quotient_values(dev(lde), log_n, 1, alpha))
    np.testing.assert_array_equal(got, want)


# ---- worst-case inputs for the lazy bounds of the quotient kernels --------------------------
# k_p2_quotient defers its reductions on analytic bounds (quotient.hip: external-layer outputs
# < 8p, S-box inputs < 10p, constraint values < 34p, acc < 36p; mul29 needs a b < 167 p^2).  Those
# bounds are reached with the largest residues: every trace cell, round constant and alpha stored
# as p - 1 (the largest canonical Montgomery residue), or p - 1 next to 0 (alternating patterns,
# so sums and differences see both extremes).  Checked against the C oracle, which reduces after
# every operation.

P = O.P
PM1 = np.array(O.int_to_limbs(P - 1), dtype=np.uint64)


def extreme_matrix(kind: str, rows: int, width: int, seed: int = 0) -> np.ndarray:
    out = np.zeros((rows, width, 4), dtype=np.uint64)
    if kind == "pm1":
        out[:] = PM1
    elif kind == "alt":  # checkerboard of p - 1 and 0
        out[(np.add.outer(np.arange(rows), np.arange(width)) % 2) == 0] = PM1
    elif kind == "alt_rows":  # local row p - 1, next row 0 (and back)
        out[::2] = PM1
    elif kind == "rand":  # full-range canonical residues (no top-limb mask)
        out[:] = C.random_fr(seed, rows * width).reshape(rows, width, 4)
    elif kind == "rand_pm1":  # random cells, one in four forced to p - 1
        out[:] = C.random_fr(seed, rows * width).reshape(rows, width, 4)
        out[np.random.default_rng(seed).random((rows, width)) < 0.25] = PM1
    else:
        raise ValueError(kind)
    return out


@pytest.fixture(scope="module")
def consts_pm1():
    """Every round constant stored as p - 1."""
    return C.P2Constants([[PM1.copy() for _ in range(3)] for _ in range(HF)], [PM1.copy() for _ in range(PR)],
                         [[PM1.copy() for _ in range(3)] for _ in range(HF)])


@pytest.mark.parametrize("vl", [1, 8])
@pytest.mark.parametrize("kind", ["pm1", "alt", "alt_rows", "rand_pm1"])
@pytest.mark.parametrize("kconsts", ["random", "pm1"])
def test_quotient_values_extreme(gpu_ctx, consts, consts_pm1, vl, kind, kconsts):
    k = consts if kconsts == "random" else consts_pm1
    log_n, log_qd = 3, 1
    q = 1 << (log_n + log_qd)
    lde = extreme_matrix(kind, q, 164 * vl, seed=31 + vl)
    air = make_air(k, vl, gpu_ctx)
    for alpha in (PM1, C.random_fr(17, 1)[0]):
        want = C.p2_quotient_values(lde, log_n, log_qd, vl, k, alpha)
        got = host(air.quotient_values(dev(lde), log_n, log_qd, alpha))
        np.testing.assert_array_equal(got, want)
