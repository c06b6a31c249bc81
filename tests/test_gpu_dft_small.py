"""GPU parity of the TwoAdicSubgroupDft<Fr> entry points against the Python oracle
(oracle/pyoracle.py: NaiveDft + trait defaults, dft/src/naive.rs, dft/src/traits.rs)."""

import numpy as np
import pytest

from oracle import pyoracle as O
from plonky3_eon_amd import Radix2Dit, Radix2DitParallel
from plonky3_eon_amd.field import ints_to_limbs, limbs_to_ints

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[0, 1, 3])
def ctx_passes(request):
    """Contexts whose NTT plans are capped at 1 or 3 stages per pass, so that multi-pass
    schedules (twiddle offsets, in-place later passes) are exercised at oracle-sized inputs."""
    import os

    from conftest import gpu_available
    if not gpu_available():
        pytest.skip("no GPU")
    from plonky3_eon_amd import Context

    os.environ["EON_NTT_MAX_STAGES"] = str(request.param)
    try:
        return Context(0)
    finally:
        os.environ.pop("EON_NTT_MAX_STAGES", None)


def to_np(mat):
    h = len(mat)
    w = len(mat[0]) if h else 0
    return ints_to_limbs([x for row in mat for x in row]).reshape(h, w, 4)


def from_np(arr):
    h, w = arr.shape[0], arr.shape[1]
    vals = limbs_to_ints(arr)
    return [vals[r * w:(r + 1) * w] for r in range(h)]


CASES = [(0, 1), (1, 1), (1, 3), (2, 2), (3, 3), (4, 1), (4, 5), (5, 8), (6, 9), (7, 16), (8, 3), (10, 1)]


@pytest.mark.parametrize("log_h,w", CASES)
def test_dft_idft(ctx_passes, log_h, w):
    gpu_ctx = ctx_passes
    m = O.random_matrix(100 + log_h * 7 + w, 1 << log_h, w)
    x = to_np(m)
    d = Radix2Dit(gpu_ctx)
    assert from_np(d.dft_batch(x)) == O.dft(m)
    assert from_np(d.idft_batch(x)) == O.idft(m)
    assert from_np(Radix2DitParallel(gpu_ctx).dft_batch(x).storage) == O.bit_reverse_rows(O.dft(m))


@pytest.mark.parametrize("log_h,w", CASES)
def test_coset(ctx_passes, log_h, w):
    gpu_ctx = ctx_passes
    m = O.random_matrix(200 + log_h * 7 + w, 1 << log_h, w)
    x = to_np(m)
    s = O.GENERATOR
    d = Radix2Dit(gpu_ctx)
    assert from_np(d.coset_dft_batch(x, s)) == O.coset_dft(m, s)
    assert from_np(d.coset_idft_batch(x, s)) == O.coset_idft(m, s)
    assert from_np(Radix2DitParallel(gpu_ctx).coset_dft_batch(x, s).storage) == O.bit_reverse_rows(O.coset_dft(m, s))


@pytest.mark.parametrize("log_h,w,b", [(0, 1, 1), (0, 2, 3), (1, 1, 1), (2, 3, 2), (4, 3, 1), (5, 8, 2), (6, 9, 1), (7, 4, 3)])
def test_coset_lde(ctx_passes, log_h, w, b):
    gpu_ctx = ctx_passes
    m = O.random_matrix(300 + log_h * 7 + w, 1 << log_h, w)
    x = to_np(m)
    for s in (1, O.GENERATOR, 7 * O.two_adic_generator(log_h + b) % O.P):
        want = O.coset_lde(m, b, s)
        assert from_np(Radix2Dit(gpu_ctx).coset_lde_batch(x, b, s)) == want
        assert from_np(Radix2DitParallel(gpu_ctx).coset_lde_batch(x, b, s).storage) == O.bit_reverse_rows(want)


@pytest.mark.parametrize("log_h,w,b", [(0, 1, 1), (1, 2, 2), (3, 3, 1), (5, 8, 2), (6, 9, 1), (7, 4, 3)])
def test_coset_dft_padded(ctx_passes, log_h, w, b):
    """coset_dft of the zero-padded coefficients (coset_lde_batch without its idft;
    KzgPcs::get_evaluations_on_domain from committed coefficients)."""
    gpu_ctx = ctx_passes
    m = O.random_matrix(400 + log_h * 7 + w, 1 << log_h, w)
    padded = m + [[0] * w for _ in range(((1 << log_h) << b) - (1 << log_h))]
    x = to_np(m)
    for s in (1, O.GENERATOR, 11 * O.two_adic_generator(log_h + b) % O.P):
        want = O.coset_dft(padded, s)
        assert from_np(Radix2Dit(gpu_ctx).coset_dft_padded_batch(x, b, s)) == want
        assert from_np(Radix2DitParallel(gpu_ctx).coset_dft_padded_batch(x, b, s).storage) == O.bit_reverse_rows(want)
