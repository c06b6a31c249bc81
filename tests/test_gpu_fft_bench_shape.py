"""GPU parity at the reference's own DFT benchmark shape (dft/benches/fft.rs:11-27,87-114): 256
columns, log sizes 14..22, dft_batch / idft_batch / coset_lde_batch(1, GENERATOR) for Radix2Dit
(natural order) and Radix2DitParallel (bit-reversed storage).

* 2^14 x 256: every output element against the C restatement (oracle/eon_oracle.c).
* 2^22 x 256 (34 GB in, 69 GB out, device-resident): columns are independent polynomials, so a
  sample of columns is checked against the C restatement run on those columns alone, plus the
  exact round trip idft(dft(x)) == x over the whole matrix.
"""

import numpy as np
import pytest

from oracle import coracle as C
from plonky3_eon_amd import Radix2Dit, Radix2DitParallel

pytestmark = pytest.mark.gpu

COLS = 256  # BATCH_SIZE, dft/benches/fft.rs:15


def dev_random_fr(n: int, w: int, seed: int):
    """canonical Fr Montgomery limbs drawn on the device (top limb below p's): the 2^22 x 256
    input would take minutes to draw and copy from the host"""
    import torch

    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    x = torch.randint(-(2**63), 2**63 - 1, (n, w, 4), dtype=torch.int64, device="cuda:0", generator=g)
    x[..., 3] &= 0x2FFFFFFFFFFFFFFF
    return x


def bitrev_index(lg: int) -> np.ndarray:
    i = np.arange(1 << lg, dtype=np.int64)
    r = np.zeros_like(i)
    for b in range(lg):
        r |= ((i >> b) & 1) << (lg - 1 - b)
    return r


def host(t):
    return t.contiguous().cpu().numpy().view(np.uint64)


def test_fft_bench_shape_2e14_full(gpu_ctx):
    x = C.random_fr(1414, (1 << 14) * COLS).reshape(1 << 14, COLS, 4)
    gen = C.fr_from_u64(5)
    d, dp = Radix2Dit(gpu_ctx), Radix2DitParallel(gpu_ctx)
    np.testing.assert_array_equal(d.dft_batch(x), C.dft_batch(x))
    np.testing.assert_array_equal(dp.dft_batch(x).storage, C.r2dp_dft_batch(x))
    np.testing.assert_array_equal(d.idft_batch(x), C.idft_batch(x))
    np.testing.assert_array_equal(d.coset_lde_batch(x, 1, gen), C.coset_lde_batch(x, 1, gen))
    np.testing.assert_array_equal(dp.coset_lde_batch(x, 1, gen).storage, C.r2dp_coset_lde_batch(x, 1, gen))


@pytest.mark.slow
def test_fft_bench_shape_2e22(gpu_ctx):
    import torch

    log_n = 22
    n = 1 << log_n
    gen = C.fr_from_u64(5)
    x = dev_random_fr(n, COLS, 2222)
    cols = [0, 97, 255]
    d, dp = Radix2Dit(gpu_ctx), Radix2DitParallel(gpu_ctx)

    # coset_lde(1, GENERATOR), natural order: one column against the C restatement, and the
    # whole matrix through the exact round trip coset_idft(coset_lde(x)) == idft(x) zero-padded
    nat = d.coset_lde_batch(x, 1, gen)
    nat_cols = host(nat[:, cols])
    np.testing.assert_array_equal(nat_cols[:, 1:2], C.coset_lde_batch(host(x[:, 97:98]), 1, gen))
    back = d.coset_idft_batch(nat, gen)
    del nat
    assert int(torch.count_nonzero(back[n:])) == 0
    coeffs = d.idft_batch(x)
    assert torch.equal(back[:n], coeffs)
    del back, coeffs
    # Radix2DitParallel: bit-reversed storage of the same evaluations
    st = host(dp.coset_lde_batch(x, 1, gen).storage[:, cols])
    np.testing.assert_array_equal(st, nat_cols[bitrev_index(log_n + 1)])
    # dft_batch: one column against the C restatement, idft(dft(x)) == x over the whole matrix
    y = d.dft_batch(x)
    np.testing.assert_array_equal(host(y[:, 0:1]), C.dft_batch(host(x[:, 0:1])))
    assert torch.equal(d.idft_batch(y), x)
    del y
    torch.cuda.empty_cache()
