"""The multi-batch MSM pipeline at full size (eon_msm_g1_columns_dev: batches of <= 2^29 digit
pairs alternating over two compute streams with three workspaces and a sort stream): 520 columns
of 2^17 scalars are 3 batches.  Columns are col_j = s + j t, so MSM(col_j) = S + j T must hold for
every column (a cross-batch ordering race breaks it with overwhelming probability); col_0 and
col_1 are checked against the C Pippenger restatement."""

import numpy as np
import pytest

from oracle import coracle as C

pytestmark = pytest.mark.gpu


def test_multibatch_columns_linear(gpu_ctx):
    import torch

    from plonky3_eon_amd.distributed import combine_partials
    from plonky3_eon_amd.msm import MsmBases, srs_powers

    n, width = 1 << 17, 520
    srs = srs_powers(n, 4242, gpu_ctx)
    bases = MsmBases(srs, gpu_ctx, precompute=True)
    st = torch.from_numpy(np.stack([C.random_fr(31, n).reshape(n, 4), C.random_fr(32, n).reshape(n, 4)])
                          .view(np.int64)).to("cuda:0")
    mat = torch.empty((n, width, 4), dtype=torch.int64, device="cuda:0")
    for j in range(width):
        mat[:, j] = combine_partials(gpu_ctx, st, [1, j])
    got = bases.msm_columns(mat)
    s_host = st[0].cpu().numpy().view(np.uint64)
    t_host = st[1].cpu().numpy().view(np.uint64)
    S = C.g1_msm(srs, s_host)
    np.testing.assert_array_equal(got[0], S)
    s_plus_t = C.g1_msm(srs, mat[:, 1].contiguous().cpu().numpy().view(np.uint64))
    np.testing.assert_array_equal(got[1], s_plus_t)
    T = C.g1_msm(srs, t_host)
    acc = S
    for j in range(1, width):
        acc = C.g1_add(acc, T)
        assert np.array_equal(got[j], acc), f"column {j}"
