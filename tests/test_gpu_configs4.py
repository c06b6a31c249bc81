"""BASELINE configs[4] at full size on one GPU (world 1) through the multi-GPU entry points
(include/eon.h: eon_fourstep_dft_dev, eon_msm_sharded_dev): the same code the 8-GPU run executes,
minus the exchanges (which the gloo multi-rank tests cover at small sizes).

* (i) forward DFT of one 2^26 column as a four-step 2^13 x 2^13 transform: every output equals the
  single-network eon_dft_batch_dev's, and spot rows equal the C oracle's Horner evaluation
  X[k] = sum_j x_j w^(jk) (dft/src/traits.rs:61 / kzg/src/util.rs:63-68).
* (ii) MSM of 2^24 terms over the alpha = 12345 SRS: sum_i s_i alpha^i G = [f(alpha)] G with
  f(alpha) from the C oracle's Horner loop (a size-independent identity, as
  bn254/src/curve.rs:598-628's group-law checks).
"""

import ctypes

import numpy as np
import pytest

from oracle import coracle as C

pytestmark = pytest.mark.gpu


def test_fourstep_dft_2_26_world1(gpu_ctx):
    import torch

    from plonky3_eon_amd import _lib as L

    log_n = 26
    n = 1 << log_n
    x = C.random_fr(2626, n).reshape(n, 4)
    xt = torch.from_numpy(x.view(np.int64)).to("cuda:0")
    ctx = gpu_ctx
    ctx.set_stream(torch.cuda.current_stream(xt.device).cuda_stream)
    four = torch.empty_like(xt)
    ctx.check(ctx.lib.eon_fourstep_dft_dev(ctx.handle, ctypes.c_void_p(xt.data_ptr()),
                                           ctypes.c_void_p(four.data_ptr()), log_n, L.EON_FOURSTEP_NATURAL, None))
    one = torch.empty_like(xt)
    ctx.check(ctx.lib.eon_dft_batch_dev(ctx.handle, ctypes.c_void_p(xt.data_ptr()), ctypes.c_void_p(one.data_ptr()),
                                        n, 1, L.EON_ORDER_NATURAL))
    torch.cuda.synchronize()
    assert torch.equal(four, one), "four-step 2^26 DFT != single-network DFT"
    got = four.cpu().numpy().view(np.uint64)
    w = C.two_adic_generator(log_n)
    for k in (1, n - 1, 12345678):
        want = C.eval_poly_col(x.reshape(n, 1, 4), 0, C.fr_pow(w, k))
        np.testing.assert_array_equal(got[k], want, err_msg=f"X[{k}]")


def test_msm_2_24_world1_kzg_identity(gpu_ctx):
    import torch

    from plonky3_eon_amd import _lib as L
    from plonky3_eon_amd.msm import MsmBases, srs_powers

    n = 1 << 24
    pts = srs_powers(n, 12345, gpu_ctx)
    bases = MsmBases(pts, gpu_ctx, precompute=True)
    del pts
    s = C.random_fr(2424, n).reshape(n, 4)
    st = torch.from_numpy(s.view(np.int64)).to("cuda:0")
    out = L.eon_g1_affine()
    ctx = gpu_ctx
    ctx.set_stream(torch.cuda.current_stream(st.device).cuda_stream)
    ctx.check(ctx.lib.eon_msm_sharded_dev(ctx.handle, bases._h, ctypes.c_void_p(st.data_ptr()), n, None,
                                          ctypes.byref(out)))
    got = np.array(list(out.x) + list(out.y), dtype=np.uint64)
    f_alpha = C.eval_poly_col(s.reshape(n, 1, 4), 0, C.fr_from_u64(12345))
    np.testing.assert_array_equal(got, C.g1_mul(C.g1_generator(), f_alpha))
    bases.close()
