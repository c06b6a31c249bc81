"""GPU parity of the DFT entry points against the C restatement oracle at mid sizes
(BASELINE configs[0]: 2^12 NTT, widths 1/3/64), and size-independent properties at the full
BASELINE configs[1] size (2^20 x 64 LDE)."""

import numpy as np
import pytest

from oracle import coracle as C
from plonky3_eon_amd import Radix2Dit, Radix2DitParallel

pytestmark = pytest.mark.gpu

GEN = None


def gen():
    global GEN
    if GEN is None:
        GEN = C.fr_from_u64(5)
    return GEN


@pytest.mark.parametrize("log_h,w", [(12, 1), (12, 3), (12, 64), (14, 5), (16, 2), (11, 17)])
def test_c1_ops_vs_c_oracle(gpu_ctx, log_h, w):
    x = C.random_fr(10 * log_h + w, (1 << log_h) * w).reshape(1 << log_h, w, 4)
    d = Radix2Dit(gpu_ctx)
    np.testing.assert_array_equal(d.dft_batch(x), C.dft_batch(x))
    np.testing.assert_array_equal(d.idft_batch(x), C.idft_batch(x))
    np.testing.assert_array_equal(d.coset_dft_batch(x, gen()), C.coset_dft_batch(x, gen()))
    np.testing.assert_array_equal(d.coset_idft_batch(x, gen()), C.coset_idft_batch(x, gen()))
    np.testing.assert_array_equal(Radix2DitParallel(gpu_ctx).dft_batch(x).storage, C.r2dp_dft_batch(x))
    for b in (1, 2):
        want_nat = C.coset_lde_batch(x, b, gen())
        np.testing.assert_array_equal(d.coset_lde_batch(x, b, gen()), want_nat)
        # Radix2DitParallel's own two-half schedule (restated) vs the GPU bit-reversed storage
        np.testing.assert_array_equal(Radix2DitParallel(gpu_ctx).coset_lde_batch(x, b, gen()).storage,
                                      C.r2dp_coset_lde_batch(x, b, gen()))


def test_kzg_get_evaluations_on_domain_equivalence(gpu_ctx):
    """KzgPcs::get_evaluations_on_domain (Horner at every point, kzg/src/pcs.rs:267-287) equals
    the GPU coset LDE in natural order (commit/src/testing.rs:93-105 model)."""
    log_n, w, qd = 8, 3, 1
    evals = C.random_fr(77, (1 << log_n) * w).reshape(1 << log_n, w, 4)
    coeffs = C.idft_batch(evals)  # KzgPcs::commit keeps coset_idft(evals, shift 1)
    want = C.kzg_evaluations_on_domain(coeffs, log_n + qd, gen())
    got = Radix2Dit(gpu_ctx).coset_lde_batch(evals, qd, gen())
    np.testing.assert_array_equal(got, want)


def test_errors(gpu_ctx):
    from plonky3_eon_amd import EonError

    d = Radix2Dit(gpu_ctx)
    with pytest.raises(EonError):  # log2_strict_usize panics on non-powers of two
        d.dft_batch(np.zeros((3, 2, 4), dtype=np.uint64))
    with pytest.raises(EonError):  # beyond TWO_ADICITY = 28
        d.lde_batch(np.zeros((2, 1, 4), dtype=np.uint64), 28)
    # width 0 is a no-op
    assert d.dft_batch(np.zeros((4, 0, 4), dtype=np.uint64)).shape == (4, 0, 4)


@pytest.mark.slow
def test_c2_full_size_properties(gpu_ctx):
    """configs[1] size on device: coset_idft(coset_lde(x)) == idft(x) zero-padded (exact
    round trip through the big domain), plus Horner spot checks of LDE rows."""
    import torch

    log_n, w, b = 20, 64, 1
    n = 1 << log_n
    dev = torch.device("cuda", 0)
    xh = C.random_fr(2020, n * w).reshape(n, w, 4)
    x = torch.from_numpy(xh.view(np.int64)).to(dev)
    d = Radix2Dit(gpu_ctx)
    lde = d.coset_lde_batch(x, b, gen())
    back = d.coset_idft_batch(lde, gen())
    coeffs = d.idft_batch(x)
    assert torch.equal(back[:n], coeffs)
    assert int(torch.count_nonzero(back[n:])) == 0
    # bit-reversed storage is a row permutation of the natural result
    st = Radix2DitParallel(gpu_ctx).coset_lde_batch(x, b, gen()).storage
    lg = log_n + b
    idx = torch.arange(n << b, device=dev)
    rev = torch.zeros_like(idx)
    for i in range(lg):
        rev |= ((idx >> i) & 1) << (lg - 1 - i)
    assert torch.equal(st[rev], lde)
    # Horner spot checks (eval_poly, kzg/src/util.rs:63-68) on host coefficients
    ch = coeffs.cpu().numpy().view(np.uint64)
    lh = lde.cpu().numpy().view(np.uint64)
    g = C.two_adic_generator(lg)
    for k, col in [(0, 0), (1, 5), (n + 3, 63), ((n << b) - 1, 17)]:
        pt = C.fr_mul(gen(), C.fr_pow(g, k))
        np.testing.assert_array_equal(lh[k, col], C.eval_poly_col(ch, col, pt))


@pytest.mark.slow
@pytest.mark.parametrize("order", ["natural", "bitrev"])
def test_c2_full_size_bit_exact(gpu_ctx, order):
    """configs[1] at its full size, element for element: the GPU coset LDE of a 2^20 x 64 matrix
    (added_bits 1, shift GENERATOR = 5) equals the C restatement's -- natural order against
    coset_lde_batch (Radix2Dit, dft/src/radix_2_dit.rs:61-122 via the trait default
    dft/src/traits.rs:226-249), bit-reversed storage against Radix2DitParallel's own two-half
    schedule (dft/src/radix_2_dit_parallel.rs:169-228).  The oracle takes ~8 s on 16 threads."""
    import torch

    log_n, w, b = 20, 64, 1
    n = 1 << log_n
    xh = C.random_fr(2021 + (order == "bitrev"), n * w).reshape(n, w, 4)
    x = torch.from_numpy(xh.view(np.int64)).to("cuda:0")
    if order == "natural":
        got = Radix2Dit(gpu_ctx).coset_lde_batch(x, b, gen()).cpu().numpy().view(np.uint64)
        want = C.coset_lde_batch(xh, b, gen())
    else:
        got = Radix2DitParallel(gpu_ctx).coset_lde_batch(x, b, gen()).storage
        got = got.cpu().numpy().view(np.uint64) if hasattr(got, "cpu") else got
        want = C.r2dp_coset_lde_batch(xh, b, gen())
    del x
    assert got.shape == want.shape == (n << b, w, 4)
    bad = np.flatnonzero((got != want).any(axis=(1, 2)))
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:8]}"


# p - 1 as raw limbs: the largest canonical representation, the worst case of the lazy NTT bounds
# (DIT outputs grow by < 3p per stage, DIF sums are reduced every other stage)
P_MINUS_1 = np.array([0x43E1F593F0000000, 0x2833E84879B97091, 0xB85045B68181585D, 0x30644E72E131A029],
                     dtype=np.uint64)


@pytest.mark.parametrize("pattern", ["all_max", "alternating", "max_rows_then_random"])
@pytest.mark.parametrize("log_h,w", [(12, 8), (11, 3), (15, 1)])
def test_extreme_inputs_vs_c_oracle(gpu_ctx, log_h, w, pattern):
    n = 1 << log_h
    x = np.zeros((n, w, 4), dtype=np.uint64)
    if pattern == "all_max":
        x[:] = P_MINUS_1
    elif pattern == "alternating":
        x[::2] = P_MINUS_1
    else:
        x[:] = C.random_fr(3 * log_h + w, n * w).reshape(n, w, 4)
        x[: n // 2] = P_MINUS_1
    d = Radix2Dit(gpu_ctx)
    np.testing.assert_array_equal(d.dft_batch(x), C.dft_batch(x))
    np.testing.assert_array_equal(d.idft_batch(x), C.idft_batch(x))
    np.testing.assert_array_equal(d.coset_dft_batch(x, gen()), C.coset_dft_batch(x, gen()))
    np.testing.assert_array_equal(d.coset_idft_batch(x, gen()), C.coset_idft_batch(x, gen()))
    np.testing.assert_array_equal(Radix2DitParallel(gpu_ctx).dft_batch(x).storage, C.r2dp_dft_batch(x))
    for b in (1, 2):
        np.testing.assert_array_equal(d.coset_lde_batch(x, b, gen()), C.coset_lde_batch(x, b, gen()))
        np.testing.assert_array_equal(Radix2DitParallel(gpu_ctx).coset_lde_batch(x, b, gen()).storage,
                                      C.r2dp_coset_lde_batch(x, b, gen()))
        padded = np.concatenate([x, np.zeros(((n << b) - n, w, 4), dtype=np.uint64)])
        np.testing.assert_array_equal(d.coset_dft_padded_batch(x, b, gen()), C.coset_dft_batch(padded, gen()))
