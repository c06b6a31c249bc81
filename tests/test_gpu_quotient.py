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
