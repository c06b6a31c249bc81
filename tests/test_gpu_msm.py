"""GPU parity of the BN254 G1 MSM (G1::multi_exp, bn254/src/curve.rs:158-179) against the
oracles: the reference's own MSM identities (curve.rs:598-628), the Python double-and-add
oracle, the C Pippenger restatement, and the size-independent KZG identity
sum_i s_i * (alpha^i G) = [f(alpha)] G."""

import numpy as np
import pytest

from oracle import coracle as C
from oracle import pyoracle as O
from plonky3_eon_amd.msm import MsmBases, multi_exp, srs_powers

pytestmark = pytest.mark.gpu


def fr(x):
    return np.array(O.int_to_limbs(O.to_mont(x)), dtype=np.uint64)


def pt(p):
    return np.frombuffer(O.g1_to_bytes(p), dtype=np.uint64).copy()


def as_py(a):
    return O.g1_from_bytes(np.ascontiguousarray(a, dtype=np.uint64).tobytes())


def test_reference_msm_identities(gpu_ctx):
    g = O.G1_GEN
    empty = multi_exp(np.zeros((0, 8), np.uint64), np.zeros((0, 4), np.uint64), gpu_ctx)
    assert as_py(empty) is O.INF
    assert as_py(multi_exp(pt(g)[None], fr(5)[None], gpu_ctx)) == O.g1_mul(g, 5)
    assert as_py(multi_exp(np.stack([pt(g), pt(g)]), np.stack([fr(2), fr(3)]), gpu_ctx)) == O.g1_mul(g, 5)
    p7, p11 = O.g1_mul(g, 7), O.g1_mul(g, 11)
    r = multi_exp(np.stack([pt(p7), pt(p11)]), np.stack([fr(3), fr(5)]), gpu_ctx)
    assert as_py(r) == O.g1_mul(g, 76)
    from plonky3_eon_amd import EonError
    with pytest.raises(EonError):
        multi_exp(np.stack([pt(g), pt(g)]), fr(1)[None], gpu_ctx)


@pytest.mark.parametrize("precompute", [False, True])
def test_edge_cases_vs_python(gpu_ctx, precompute):
    g = O.G1_GEN
    rng = O.SplitMix64(99)
    ks = [rng.next() % 1000 + 1 for _ in range(12)]
    P = [O.g1_mul(g, k) for k in ks]
    # duplicates (bucket doubling), a point and its negation, the identity base
    P += [P[0], P[0], O.g1_neg(P[1]), O.INF]
    scal = [O.from_mont(rng.fr_mont()) for _ in range(len(P))]
    scal[2] = 0
    scal[3] = O.P - 1
    scal[12] = scal[13] = scal[0]
    scal[14] = scal[1]
    bases = MsmBases(np.stack([pt(p) for p in P]), gpu_ctx, precompute=precompute)
    for n in (0, 1, 2, 5, len(P)):
        want = O.msm(P[:n], scal[:n])
        got = bases.msm(np.stack([fr(s) for s in scal[:n]]) if n else np.zeros((0, 4), np.uint64))
        assert as_py(got) == want, n


@pytest.mark.parametrize("log_n,precompute", [(6, True), (10, False), (12, True), (12, False), (14, True)])
def test_vs_c_pippenger(gpu_ctx, log_n, precompute):
    n = 1 << log_n
    k = C.random_fr(log_n, n)
    g = C.g1_generator()
    pts = np.stack([C.g1_mul(g, k[i]) for i in range(n)]) if n <= 4096 else C.g1_srs(n, C.fr_from_u64(12345))
    s = C.random_fr(100 + log_n, n)
    want = C.g1_msm(pts, s)
    got = MsmBases(pts, gpu_ctx, precompute=precompute).msm(s)
    np.testing.assert_array_equal(got, want)
    assert C.g1_on_curve(got)


def test_srs_powers(gpu_ctx):
    n = 300
    np.testing.assert_array_equal(srs_powers(n, 12345, gpu_ctx), C.g1_srs(n, C.fr_from_u64(12345)))


def test_structured_scalars(gpu_ctx):
    """All-small (< 2^64, as kzg/benches) and all-equal scalars skew the buckets."""
    n = 4096
    pts = C.g1_srs(n, C.fr_from_u64(12345))
    small = np.stack([C.fr_from_u64(int(x)) for x in np.random.default_rng(1).integers(0, 2**63, n)])
    same = np.repeat(C.fr_from_u64(7)[None], n, axis=0)
    for s in (small, same):
        for pre in (True, False):
            np.testing.assert_array_equal(MsmBases(pts, gpu_ctx, precompute=pre).msm(s), C.g1_msm(pts, s))


@pytest.mark.parametrize("bits", [8, 12, 16, 24, 48, 64])
def test_active_window_truncation_edges(gpu_ctx, bits):
    """A single MSM digitises only the windows its largest scalar reaches (k_scalar_or); the signed
    recoding can carry one window past that scalar's top bit.  Largest scalar exactly 2^b - 1, 2^b
    and 2^b + 2^(b-1) for b on and off the window boundaries of both layouts (c = 12 fixed-base,
    c = 8 plain at n = 4096), the rest below 2^(b-1); plus scalars over the full u64 range
    (kzg/benches/kzg_benches.rs:19, Fr::new(rng.random::<u64>()))."""
    n = 4096
    pts = C.g1_srs(n, C.fr_from_u64(12345))
    rng = np.random.default_rng(bits)
    base = [int(x) for x in rng.integers(0, 2 ** (bits - 1), n, dtype=np.uint64)]
    for top in ((1 << bits) - 1, 1 << bits, (1 << bits) + (1 << (bits - 1))):
        vals = list(base)
        vals[rng.integers(0, n)] = top
        s = np.array([O.int_to_limbs(O.to_mont(v)) for v in vals], dtype=np.uint64)
        want = C.g1_msm(pts, s)
        for pre in (True, False):
            np.testing.assert_array_equal(MsmBases(pts, gpu_ctx, precompute=pre).msm(s), want, err_msg=f"top={top:#x}")
    full = np.stack([C.fr_from_u64(int(v)) for v in rng.integers(0, 2**64, n, dtype=np.uint64)])
    for pre in (True, False):
        np.testing.assert_array_equal(MsmBases(pts, gpu_ctx, precompute=pre).msm(full), C.g1_msm(pts, full))


def test_all_equal_scalars_multi_level(gpu_ctx):
    """2^16 equal scalars: every window's digit hits one bucket, 2^16 entries -> 3 combine
    levels; the value is [s * sum(alpha^i)] G."""
    n = 1 << 16
    alpha = C.fr_from_u64(12345)
    pts = srs_powers(n, 12345, gpu_ctx)
    s7 = C.fr_from_u64(7)
    ones = np.repeat(C.fr_from_u64(1)[None], n, axis=0)
    total = C.eval_poly_col(ones.reshape(n, 1, 4), 0, alpha)  # sum_i alpha^i
    want = C.g1_mul(C.g1_generator(), C.fr_mul(total, s7))
    same = np.repeat(s7[None], n, axis=0)
    for pre in (True, False):
        np.testing.assert_array_equal(MsmBases(pts, gpu_ctx, precompute=pre).msm(same), want)


@pytest.mark.slow
def test_kzg_identity_full_size(gpu_ctx):
    """configs[2] size: sum_i s_i * alpha^i G == [f(alpha)] G for the SRS of init_srs_unsafe
    (kzg/src/params.rs:123-139), f(alpha) by Horner (eval_poly, kzg/src/util.rs:63-68)."""
    import torch

    n = 1 << 20
    alpha = C.fr_from_u64(12345)
    pts = srs_powers(n, 12345, gpu_ctx)
    for i in (0, 1, 2, 777, n - 1):  # device SRS vs the oracle's alpha^i * G
        np.testing.assert_array_equal(pts[i], C.g1_mul(C.g1_generator(), C.fr_pow(alpha, i)))
    s = C.random_fr(2021, n)
    f_alpha = C.eval_poly_col(s.reshape(n, 1, 4), 0, alpha)
    want = C.g1_mul(C.g1_generator(), f_alpha)
    bases = MsmBases(pts, gpu_ctx, precompute=True)
    st = torch.from_numpy(s.view(np.int64)).to("cuda:0")
    np.testing.assert_array_equal(bases.msm(st), want)
    np.testing.assert_array_equal(MsmBases(pts, gpu_ctx, precompute=False).msm(s), want)


@pytest.mark.slow
def test_msm_full_size_vs_c_pippenger(gpu_ctx):
    """configs[2] at its full size, bit for bit: the 2^20-point MSM over the alpha = 12345 SRS
    (fixed-base tables, and the plain bases) equals the C signed-window Pippenger restatement's
    affine result (G1::multi_exp, bn254/src/curve.rs:158-179; the sum is unique, so the bytes are
    the reference's), for uniform scalars and for scalars below 2^64 (kzg/benches/kzg_benches.rs)."""
    import torch

    n = 1 << 20
    pts = srs_powers(n, 12345, gpu_ctx)
    bases = MsmBases(pts, gpu_ctx, precompute=True)
    plain = MsmBases(pts, gpu_ctx, precompute=False)
    for seed, small in ((2022, False), (2023, True)):
        s = C.random_fr(seed, n)
        if small:
            s = np.stack([C.fr_from_u64(int(v)) for v in
                          np.random.default_rng(seed).integers(0, 2**63, size=n, dtype=np.int64)])
        want = C.g1_msm(pts, s)
        st = torch.from_numpy(s.view(np.int64)).to("cuda:0")
        np.testing.assert_array_equal(bases.msm(st), want)
        np.testing.assert_array_equal(plain.msm(s), want)


@pytest.mark.parametrize("precompute", [True, False])
def test_msm_columns_vs_c(gpu_ctx, precompute):
    """KzgPcs::commit's per-column commit_column loop (kzg/src/pcs.rs:244-251) as one batched call."""
    rows, width = 200, 7
    pts = srs_powers(256, 12345, gpu_ctx)
    mat = C.random_fr(31, rows * width).reshape(rows, width, 4)
    mat[:, 3] = 0  # an all-zero column commits to the identity
    got = MsmBases(pts, gpu_ctx, precompute=precompute).msm_columns(mat)
    for j in range(width):
        np.testing.assert_array_equal(got[j], C.g1_msm(pts[:rows], mat[:, j]))
    assert not got[3].any()


@pytest.mark.parametrize("rows", [4096, 4100])
def test_fused_digit_sort_columns_vs_c(gpu_ctx, monkeypatch, rows):
    """The digit sort's first pass fused with the digit extraction (k_digit_sort_pass: fixed-base
    tables with c = 16, 16 windows, rows a multiple of 1024 -- the headline prove's shape, forced
    here at 4096 rows by EON_MSM_FORCE_C); 4100 rows take the unfused route at the same c.  Several
    columns per batch check that every (digit, column) bucket stays one run."""
    monkeypatch.setenv("EON_MSM_FORCE_C", "16")
    width = 5
    pts = srs_powers(rows, 777, gpu_ctx)
    mat = C.random_fr(41, rows * width).reshape(rows, width, 4)
    mat[:, 1] = 0  # an all-zero column
    mat[: rows // 2, 2] = mat[0, 2]  # half the rows one scalar: long runs in few buckets
    r_minus_1 = np.array(O.int_to_limbs(O.to_mont(O.P - 1)), dtype=np.uint64)
    mat[::3, 4] = r_minus_1  # top-heavy digits, every window negative
    bases = MsmBases(pts, gpu_ctx, precompute=True)
    gpu_ctx.profile(True)
    try:
        got = bases.msm_columns(mat)
        kernels = gpu_ctx.profile_report()
    finally:
        gpu_ctx.profile(False)
    assert ("k_digit_sort_pass" in kernels) == (rows % 1024 == 0), sorted(kernels)
    for j in range(width):
        np.testing.assert_array_equal(got[j], C.g1_msm(pts, mat[:, j]), err_msg=f"column {j}")
    assert not got[1].any()
    np.testing.assert_array_equal(bases.msm(mat[:, 0]), C.g1_msm(pts, mat[:, 0]))


@pytest.mark.slow
def test_msm_columns_batched_kzg_identity(gpu_ctx):
    """300 columns x 2^16 rows (split into 2 internal batches), device-resident: every column
    satisfies sum_i m[i][j] alpha^i G = [f_j(alpha)] G."""
    import torch

    rows, width = 1 << 16, 300
    alpha = C.fr_from_u64(12345)
    pts = srs_powers(rows, 12345, gpu_ctx)
    mat = C.random_fr(32, rows * width).reshape(rows, width, 4)
    bases = MsmBases(pts, gpu_ctx, precompute=True)
    got = bases.msm_columns(torch.from_numpy(mat.view(np.int64)).to("cuda:0"))
    g = C.g1_generator()
    for j in list(range(0, width, 13)) + [width - 1]:
        f_alpha = C.eval_poly_col(mat, j, alpha)
        np.testing.assert_array_equal(got[j], C.g1_mul(g, f_alpha), err_msg=f"column {j}")


def test_columns_fused_reduce_edge_cases(gpu_ctx):
    """>= 64 columns of fixed-base MSMs take the fused radix-2^29 bucket reduction
    (k_bucket_reduce29): equal piece partials (doubling) and opposite ones (identity) inside one
    bucket, zero and small-scalar columns, against the Python double-and-add oracle."""
    g = O.G1_GEN
    P = O.g1_mul(g, 1234567)
    rows, width = 300, 66
    pts = np.stack([pt(P)] * 150 + [pt(O.g1_neg(P))] * 150)
    bases = MsmBases(pts, gpu_ctx, precompute=True)
    rng = O.SplitMix64(5)
    cols, want = [], []
    for j in range(width):
        if j == 0:
            s = [0] * rows
        elif j % 3 == 1:  # equal scalars: every bucket holds equal pieces of one sign
            v = O.from_mont(rng.fr_mont())
            s = [v] * rows
        elif j % 3 == 2:  # small scalars
            s = [rng.next() % 1000 for _ in range(rows)]
        else:
            s = [O.from_mont(rng.fr_mont()) for _ in range(rows)]
        cols.append(s)
        k = (sum(s[:150]) - sum(s[150:])) % O.P
        want.append(O.g1_mul(P, k) if k else O.INF)
    mat = np.stack([np.stack([fr(cols[j][i]) for j in range(width)]) for i in range(rows)])
    got = bases.msm_columns(mat)
    for j in range(width):
        assert as_py(got[j]) == want[j], j
    # the same with all bases equal: pieces of one bucket are equal (the doubling case)
    bases2 = MsmBases(np.stack([pt(P)] * rows), gpu_ctx, precompute=True)
    got2 = bases2.msm_columns(mat)
    for j in range(width):
        k = sum(cols[j]) % O.P
        assert as_py(got2[j]) == (O.g1_mul(P, k) if k else O.INF), j


@pytest.mark.parametrize("rows", [24, 32, 48])
@pytest.mark.parametrize("cancel", [False, True])
def test_columns_piece_merge(gpu_ctx, rows, cancel):
    """Buckets straddling piece-sum chunk boundaries (k_piece_sum29's in-wave merge and
    k_piece_merge29 between waves, msm.hip): 64 columns of `rows` equal scalars over bases all P
    (or P then -P), so every bucket is a run of `rows` sorted pairs laid end to end and the
    16-pair chunks cut them -- 24 rows: two unequal pieces, a run across the chunk-64 wave
    boundary; 32: two equal pieces (the merge doubles); 48: three pieces (no merge); with -P
    the pieces cancel (the merge's identity)."""
    g = O.G1_GEN
    P = O.g1_mul(g, 987654321)
    width = 64
    bases_pts = [P] * rows if not cancel else [P] * (rows // 2) + [O.g1_neg(P)] * (rows - rows // 2)
    bases = MsmBases(np.stack([pt(p) for p in bases_pts]), gpu_ctx, precompute=True)
    rng = O.SplitMix64(rows * 2 + cancel)
    scal = [O.from_mont(rng.fr_mont()) for _ in range(width)]
    mat = np.stack([np.stack([fr(scal[j]) for j in range(width)]) for _ in range(rows)])
    got = bases.msm_columns(mat)
    mult = rows if not cancel else (rows // 2) - (rows - rows // 2)
    for j in range(width):
        k = scal[j] * mult % O.P
        assert as_py(got[j]) == (O.g1_mul(P, k) if k else O.INF), j


def test_all_windows_knob_same_result():
    """EON_MSM_ALL_WINDOWS=1 (digitise every window, not only those the largest scalar reaches)
    gives the same MSMs: window-boundary scalars and full-range ones, in a fresh process (the knob
    is read once)."""
    import subprocess
    import sys
    from pathlib import Path

    code = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[2])
from oracle import coracle as C
from oracle import pyoracle as O
from plonky3_eon_amd import Context
from plonky3_eon_amd.msm import MsmBases
ctx = Context(0)
n = 2048
pts = C.g1_srs(n, C.fr_from_u64(777))
out = []
for top in (1 << 16, (1 << 24) - 1, (1 << 32) + (1 << 31), O.P - 1):
    vals = [int(x) for x in np.random.default_rng(top % 1000).integers(0, 2**15, n)]
    vals[5] = top
    s = np.array([O.int_to_limbs(O.to_mont(v)) for v in vals], dtype=np.uint64)
    for pre in (True, False):
        out.append(MsmBases(pts, ctx, precompute=pre).msm(s))
np.save(sys.argv[1], np.stack(out))
'''
    import os
    import tempfile

    root = str(Path(__file__).resolve().parents[1])
    res = []
    with tempfile.TemporaryDirectory() as d:
        for knob in (None, "1"):
            env = dict(os.environ)
            env.pop("EON_MSM_ALL_WINDOWS", None)
            if knob:
                env["EON_MSM_ALL_WINDOWS"] = knob
            f = os.path.join(d, f"r{knob}.npy")
            subprocess.run([sys.executable, "-c", code, f, root], check=True, env=env, timeout=240)
            res.append(np.load(f))
    np.testing.assert_array_equal(res[0], res[1])
