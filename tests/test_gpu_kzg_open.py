"""GPU parity of the KZG opening as an MSM of the committed coefficients against opening bases
(eon_msm_g1_columns_prepare_dev / eon_msm_g1_columns_prepared / eon_kzg_opening_bases_create)
against the oracle's route, the reference's: quotient_and_eval per column
(kzg/src/util.rs:100-111) then commit_column of the quotient over the SRS (kzg/src/util.rs:37-40,
kzg/src/pcs.rs:305-316), with the C Pippenger restatement as the MSM."""

import numpy as np
import pytest

from oracle import coracle as C
from plonky3_eon_amd import EonError
from plonky3_eon_amd.msm import MsmBases, srs_powers

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda:0")


@pytest.mark.parametrize("log_n,width", [(1, 2), (4, 3), (10, 5)])
def test_opening_witnesses_match_synthetic_division(gpu_ctx, log_n, width):
    n = 1 << log_n
    pts = srs_powers(n + 1, 12345, gpu_ctx)  # max_degree n, as KzgPcs's SRS
    srs = MsmBases(pts, gpu_ctx, precompute=True)
    coeffs = C.random_fr(31 + log_n, n * width).reshape(n, width, 4)
    cm, prep = srs.prepare_columns(_dev(coeffs))
    np.testing.assert_array_equal(cm, srs.msm_columns(coeffs))
    points = [C.fr_from_u64(0), C.fr_from_u64(1), C.random_fr(77, 1)[0], C.random_fr(78, 1)[0]]
    # four points at once: z = 0 and z != 0 mixed, over the three construction streams
    hs = srs.opening_bases_many(n, points)
    got = prep.msm([srs] + hs)
    np.testing.assert_array_equal(got[0], cm)  # the prepared digits reproduce the commitments
    for t, z in enumerate(points):
        for j in range(width):
            q, _ = C.quotient_and_eval(coeffs[:, j], z)
            want = C.g1_msm(pts[: n - 1], q) if n > 1 else np.zeros(8, np.uint64)
            np.testing.assert_array_equal(got[t + 1, j], want, err_msg=f"point {t} column {j}")
    prep.close()
    for h in hs:
        h.close()


def test_opening_bases_edge_cases(gpu_ctx):
    n = 16
    pts = srs_powers(n, 7, gpu_ctx)
    srs = MsmBases(pts, gpu_ctx, precompute=True)
    # n - 1 SRS points are enough; n + 1 would need n
    srs.opening_bases(n + 1, C.fr_from_u64(3)).close()
    with pytest.raises(EonError):
        srs.opening_bases(n + 2, C.fr_from_u64(3))
    # a single-row column has an empty quotient: the witness is the identity
    c1 = C.random_fr(5, 2).reshape(1, 2, 4)
    _, prep = srs.prepare_columns(_dev(c1), want_commitments=False)
    h = srs.opening_bases(1, C.fr_from_u64(9))
    np.testing.assert_array_equal(prep.msm([h]), np.zeros((1, 2, 8), np.uint64))
    # bases of another window layout are refused
    plain = MsmBases(pts, gpu_ctx, precompute=False)
    with pytest.raises(EonError):
        prep.msm([plain])


@pytest.mark.parametrize("rows,width,npts", [(1, 3, 1), (255, 2, 5), (257, 4, 4), (256 * 32 + 5, 3, 6),
                                             (256 * 32 * 3, 2, 2)])
def test_eval_columns_multi_point(gpu_ctx, rows, width, npts):
    """eon_eval_columns_dev (every point's f_j(z) in one pass, block/chunk carries) against the
    oracle's quotient_and_eval values, ragged heights and more points than one pass holds."""
    import ctypes

    import torch

    from plonky3_eon_amd import _lib
    from plonky3_eon_amd.field import fr_to_abi

    coeffs = C.random_fr(rows + npts, rows * width).reshape(rows, width, 4)
    points = [C.fr_from_u64(0)] + list(C.random_fr(rows + 7, npts - 1)) if npts > 1 else [C.fr_from_u64(5)]
    out = torch.zeros((npts, width, 4), dtype=torch.int64, device="cuda:0")
    zs = (_lib.eon_fr * npts)(*[fr_to_abi(z) for z in points])
    gpu_ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    gpu_ctx.check(gpu_ctx.lib.eon_eval_columns_dev(gpu_ctx.handle, ctypes.c_void_p(_dev(coeffs).data_ptr()), rows,
                                                   width, zs, npts, ctypes.c_void_p(out.data_ptr())))
    got = out.cpu().numpy().view(np.uint64)
    for t, z in enumerate(points):
        for j in range(width):
            _, v = C.quotient_and_eval(coeffs[:, j], z)
            np.testing.assert_array_equal(got[t, j], v, err_msg=f"point {t} column {j}")


def test_eval_columns_edge_cases(gpu_ctx):
    """Empty columns evaluate to 0 (kzg/src/util.rs:101-103), no points is a no-op, a
    non-canonical point is refused."""
    import ctypes

    import torch

    from plonky3_eon_amd import _lib
    from plonky3_eon_amd.field import fr_to_abi

    lib, h = gpu_ctx.lib, gpu_ctx.handle
    out = torch.full((2, 3, 4), 7, dtype=torch.int64, device="cuda:0")
    zs = (_lib.eon_fr * 2)(fr_to_abi(C.fr_from_u64(3)), fr_to_abi(C.fr_from_u64(4)))
    gpu_ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    gpu_ctx.check(lib.eon_eval_columns_dev(h, None, 0, 3, zs, 2, ctypes.c_void_p(out.data_ptr())))
    assert int(out.abs().sum().item()) == 0
    out.fill_(7)
    c = _dev(C.random_fr(3, 4 * 3).reshape(4, 3, 4))
    gpu_ctx.check(lib.eon_eval_columns_dev(h, ctypes.c_void_p(c.data_ptr()), 4, 3, zs, 0,
                                           ctypes.c_void_p(out.data_ptr())))
    torch.cuda.synchronize()
    assert bool((out == 7).all())
    bad = _lib.eon_fr()
    for i, v in enumerate([0x43E1F593F0000001, 0x2833E84879B97091, 0xB85045B68181585D, 0x30644E72E131A029]):
        bad.l[i] = v  # r itself
    with pytest.raises(EonError):
        gpu_ctx.check(lib.eon_eval_columns_dev(h, ctypes.c_void_p(c.data_ptr()), 4, 3, ctypes.byref(bad), 1,
                                               ctypes.c_void_p(out.data_ptr())))
