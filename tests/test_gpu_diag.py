"""Diagnostics and context housekeeping on the GPU: the in-kernel clock probe bench.py reports
(eon_diag_clock_probe) and eon_ctx_trim, which gives the context's cached idle buffers back
between proofs without changing any result."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_clock_probe_reads_a_plausible_clock(gpu_ctx):
    r = gpu_ctx.clock_probe(launches=4, iters=64)
    # MI355X: max shader clock 2400 MHz; a loaded chip holds well above 500 MHz
    assert 500 < r["clock_mhz_min"] <= r["clock_mhz_median"] <= r["clock_mhz_max"] < 2600, r
    # 2^20 threads x 2 chains x 64 products per launch: the rate is of the order of the measured
    # product peak (1.80e11/s at 2.1 GHz), far from 0 and below the issue limit
    assert 2e10 < r["products_per_s"] < 4e11, r
    assert r["ms_per_launch"] > 0


def test_clock_probe_rejects_bad_arguments(gpu_ctx):
    import ctypes

    from plonky3_eon_amd import _lib

    out = _lib.eon_clock_probe()
    assert gpu_ctx.lib.eon_diag_clock_probe(gpu_ctx.handle, 0, 10, ctypes.byref(out)) == _lib.EON_E_ARG
    assert gpu_ctx.lib.eon_diag_clock_probe(gpu_ctx.handle, 1, 0, ctypes.byref(out)) == _lib.EON_E_ARG
    assert gpu_ctx.lib.eon_diag_clock_probe(gpu_ctx.handle, 1, 10, None) == _lib.EON_E_ARG


def test_trim_between_msms_keeps_results(gpu_ctx):
    """Fixed-base tables come from the context's pool; closing the bases returns them to it and
    eon_ctx_trim empties it.  The MSM before and after a trim equals the oracle's."""
    from oracle import coracle as C
    from plonky3_eon_amd.msm import MsmBases

    n = 1 << 12
    pts = C.g1_srs(n, C.fr_from_u64(12345))
    scal = C.random_fr(3, n)
    want = C.g1_msm(pts, scal)
    for _ in range(2):
        bases = MsmBases(pts, ctx=gpu_ctx)
        np.testing.assert_array_equal(bases.msm(scal), want)
        bases.close()
        gpu_ctx.trim()


def test_prod_asm_matches_column_products(gpu_ctx):
    """The whole-product asm statements of the piece sums (prod_asm.h, tools/gen_prod_asm.py) equal
    the column-block mul29 / sqr29 / mul29_sum2 bit for bit on 2^22 operands of each kind at the
    contracts' limb bounds, half of them with every limb at its maximum."""
    for seed in (1, 2, 3, 4):
        assert gpu_ctx.prod_asm_check(1 << 20, seed) == [0, 0, 0]
