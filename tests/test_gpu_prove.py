"""End-to-end GPU prove of the (vectorized) Poseidon2-AIR with the KZG PCS against the CPU
restatement (oracle/prove_oracle.py, which uses the reference's Horner
get_evaluations_on_domain and per-column quotient_and_eval), every output bit-exact."""

import numpy as np
import pytest

from oracle import coracle as C
from oracle import prove_oracle
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu
HF, PR = 4, 56


def lim(x):
    return np.array(O.int_to_limbs(O.to_mont(x)), dtype=np.uint64)


@pytest.fixture(scope="module")
def consts():
    py = O.p2_constants(2024, HF, PR)
    return C.P2Constants([[lim(x) for x in r] for r in py[0]], [lim(x) for x in py[1]],
                         [[lim(x) for x in r] for r in py[2]])


@pytest.mark.parametrize("prepared", [False, True])
def test_open_kernel_vs_oracle(gpu_ctx, prepared):
    """KzgPcs::open both ways: the reference's quotients (prepared digits absent) and the MSM of
    the committed coefficients against the opening bases."""
    import torch

    from mirror_kzg import GpuKzgPcs, MatrixProverData, Domain

    pcs = GpuKzgPcs(600, 12345, gpu_ctx)
    for rows, w in [(1, 2), (2, 3), (257, 5), (600, 3)]:
        cf = C.random_fr(rows + w, rows * w).reshape(rows, w, 4)
        dev = torch.from_numpy(cf.view(np.int64)).to("cuda:0")
        prep = pcs.bases.prepare_columns(dev, want_commitments=False)[1] if prepared else None
        data = [MatrixProverData(Domain(1, 0), None, dev, prep)]
        z = 0xABCDEF123456789
        r = pcs.open([(data, [[z, 0]])])[0]
        for pi, pt in enumerate((z, 0)):
            for j in range(w):
                q, v = C.quotient_and_eval(cf[:, j], lim(pt))
                np.testing.assert_array_equal(r.values[0][pi][j], v)
                want = C.g1_msm(C.g1_srs(rows - 1, C.fr_from_u64(12345)), q) if rows > 1 else np.zeros(8, np.uint64)
                np.testing.assert_array_equal(r.witnesses[0][pi][j], want)


@pytest.mark.parametrize("log_n,vl", [(3, 1), (4, 2), (5, 8)])
def test_prove_vs_oracle(gpu_ctx, consts, log_n, vl):
    import torch

    from plonky3_eon_amd.air import Poseidon2Air
    from mirror_kzg import GpuKzgPcs
    from mirror_prover import prove

    n = 1 << log_n
    alpha_srs = 12345
    pcs = GpuKzgPcs(n, alpha_srs, gpu_ctx)
    air = Poseidon2Air(consts.begin, consts.partial, consts.end, vl, gpu_ctx)
    inputs = C.random_fr(log_n * 3 + vl, n * vl * 3).reshape(n * vl, 3, 4)
    trace = air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to("cuda:0"))
    alpha, zeta = 0x1234567890ABCDEF1234, 0xFEDCBA0987654321
    proof = prove(air, pcs, trace, alpha, zeta)

    srs = C.g1_srs(n + 1, C.fr_from_u64(alpha_srs))
    want = prove_oracle.prove(C.p2_generate_trace(inputs, vl, consts), srs, consts, vl, alpha, zeta)
    np.testing.assert_array_equal(proof.trace_commit[0], want["trace_commit"])
    np.testing.assert_array_equal(np.stack([c[0] for c in proof.quotient_commit]), want["quotient_commit"])
    tr = proof.opened[0]
    for p in range(2):
        np.testing.assert_array_equal(tr.values[0][p], want["trace_open"][0][p])
        np.testing.assert_array_equal(tr.witnesses[0][p], want["trace_open"][1][p])
    qo = proof.opened[1]
    for c in range(2):
        np.testing.assert_array_equal(qo.values[c][0], want["quotient_open"][c][0][0])
        np.testing.assert_array_equal(qo.witnesses[c][0], want["quotient_open"][c][1][0])


def test_open_routes_agree_full_height(gpu_ctx, consts):
    """At the headline height (2^17 rows, VECTOR_LEN 1: 164 columns, two MSM batches) the prove
    through the opening bases equals the prove through the reference's per-column quotients --
    the oracle cannot run this size, the two GPU routes check each other."""
    import torch

    from plonky3_eon_amd.air import Poseidon2Air
    from mirror_kzg import GpuKzgPcs
    from mirror_prover import prove

    log_n, vl = 17, 1
    n = 1 << log_n
    pcs = GpuKzgPcs(n, 12345, gpu_ctx)
    air = Poseidon2Air(consts.begin, consts.partial, consts.end, vl, gpu_ctx)
    inputs = C.random_fr(91, n * vl * 3).reshape(n * vl, 3, 4)
    trace = air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to("cuda:0"))
    alpha, zeta = 0x1234567890ABCDEF1234, 0xFEDCBA0987654321
    a = prove(air, pcs, trace, alpha, zeta)
    pcs.keep_digits = False
    b = prove(air, pcs, trace, alpha, zeta)
    np.testing.assert_array_equal(a.trace_commit[0], b.trace_commit[0])
    for r in range(2):
        for m in range(len(a.opened[r].values)):
            for p in range(len(a.opened[r].values[m])):
                np.testing.assert_array_equal(a.opened[r].values[m][p], b.opened[r].values[m][p])
                np.testing.assert_array_equal(a.opened[r].witnesses[m][p], b.opened[r].witnesses[m][p])


@pytest.mark.parametrize("log_n,vl", [(3, 1), (5, 8)])
def test_native_prove_vs_oracle(gpu_ctx, consts, log_n, vl):
    """The C++ prove driver (libeonprove.so, include/eon_prove.h) against the same restatement."""
    import torch

    from plonky3_eon_amd.air import Poseidon2Air
    from plonky3_eon_amd.native import NativeKzgPcs, prove_native

    n = 1 << log_n
    alpha_srs = 12345
    pcs = NativeKzgPcs(n, alpha_srs, gpu_ctx)
    air = Poseidon2Air(consts.begin, consts.partial, consts.end, vl, gpu_ctx)
    inputs = C.random_fr(log_n * 3 + vl, n * vl * 3).reshape(n * vl, 3, 4)
    trace = air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to("cuda:0"))
    alpha, zeta = 0x1234567890ABCDEF1234, 0xFEDCBA0987654321
    proof = prove_native(air, pcs, trace, alpha, zeta)
    assert proof.degree_bits == log_n

    srs = C.g1_srs(n + 1, C.fr_from_u64(alpha_srs))
    want = prove_oracle.prove(C.p2_generate_trace(inputs, vl, consts), srs, consts, vl, alpha, zeta)
    np.testing.assert_array_equal(proof.trace_commit[0], want["trace_commit"])
    np.testing.assert_array_equal(np.stack([c[0] for c in proof.quotient_commit]), want["quotient_commit"])
    tr = proof.opened[0]
    for p in range(2):
        np.testing.assert_array_equal(tr.values[0][p], want["trace_open"][0][p])
        np.testing.assert_array_equal(tr.witnesses[0][p], want["trace_open"][1][p])
    qo = proof.opened[1]
    for c in range(2):
        np.testing.assert_array_equal(qo.values[c][0], want["quotient_open"][c][0][0])
        np.testing.assert_array_equal(qo.witnesses[c][0], want["quotient_open"][c][1][0])


@pytest.mark.parametrize("log_n,vl", [(3, 1), (4, 2)])
def test_native_prove_fiat_shamir_vs_oracle(gpu_ctx, consts, log_n, vl):
    """eon_prove_p2air_fs: alpha and zeta sampled from the DuplexChallenger transcript
    (prover.rs:196-208, 300, 373, 416) -- challenges and proof equal the oracle's."""
    import torch

    from plonky3_eon_amd.air import Poseidon2Air
    from plonky3_eon_amd.native import Challenger, NativeKzgPcs, Poseidon2Constants, prove_native

    n = 1 << log_n
    pcs = NativeKzgPcs(n, 12345, gpu_ctx)
    air = Poseidon2Air(consts.begin, consts.partial, consts.end, vl, gpu_ctx)
    inputs = C.random_fr(log_n * 5 + vl, n * vl * 3).reshape(n * vl, 3, 4)
    trace = air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to("cuda:0"))
    pyc = O.p2_constants(99, 2, 22)  # the challenger's own permutation, as new_from_rng(4, 22)
    ch = Challenger(Poseidon2Constants([[lim(x) for x in r] for r in pyc[0]], [lim(x) for x in pyc[1]],
                                       [[lim(x) for x in r] for r in pyc[2]]))
    proof = prove_native(air, pcs, trace, None, None, challenger=ch)

    ref = O.DuplexChallenger(pyc)
    srs = C.g1_srs(n + 1, C.fr_from_u64(12345))
    want = prove_oracle.prove(C.p2_generate_trace(inputs, vl, consts), srs, consts, vl, None, None,
                              challenger=ref)
    assert (proof.alpha, proof.zeta) == (want["alpha"], want["zeta"])
    np.testing.assert_array_equal(ch.state(), np.stack([lim(x) for x in ref.state]))
    # the Python mirror (prover.py) with its own challenger samples the same challenges
    from mirror_kzg import GpuKzgPcs
    from mirror_prover import prove

    ch2 = Challenger(Poseidon2Constants([[lim(x) for x in r] for r in pyc[0]], [lim(x) for x in pyc[1]],
                                        [[lim(x) for x in r] for r in pyc[2]]))
    pp = prove(air, GpuKzgPcs(n, 12345, gpu_ctx), trace, None, None, challenger=ch2)
    assert (pp.alpha, pp.zeta) == (want["alpha"], want["zeta"])
    np.testing.assert_array_equal(pp.opened[0].witnesses[0][1], want["trace_open"][1][1])
    np.testing.assert_array_equal(proof.trace_commit[0], want["trace_commit"])
    np.testing.assert_array_equal(np.stack([c[0] for c in proof.quotient_commit]), want["quotient_commit"])
    tr = proof.opened[0]
    for p in range(2):
        np.testing.assert_array_equal(tr.values[0][p], want["trace_open"][0][p])
        np.testing.assert_array_equal(tr.witnesses[0][p], want["trace_open"][1][p])
    qo = proof.opened[1]
    for c in range(2):
        np.testing.assert_array_equal(qo.values[c][0], want["quotient_open"][c][0][0])
        np.testing.assert_array_equal(qo.witnesses[c][0], want["quotient_open"][c][1][0])


def test_native_errors(gpu_ctx, consts):
    """Reference panics -> EonError: degree above the SRS (KzgError::DegreeTooLarge), a
    non-power-of-two height."""
    import torch

    from plonky3_eon_amd import _lib
    from plonky3_eon_amd.air import Poseidon2Air
    from plonky3_eon_amd.native import NativeKzgPcs, prove_native

    air = Poseidon2Air(consts.begin, consts.partial, consts.end, 1, gpu_ctx)
    inputs = C.random_fr(3, 16 * 3).reshape(16, 3, 4)
    trace = air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to("cuda:0"))
    small = NativeKzgPcs(8, 12345, gpu_ctx)
    with pytest.raises(_lib.EonError) as e:
        prove_native(air, small, trace, 3, 5)
    assert e.value.code == _lib.EON_E_DEGREE_TOO_LARGE
    pcs = NativeKzgPcs(16, 12345, gpu_ctx)
    with pytest.raises(_lib.EonError) as e:
        prove_native(air, pcs, trace[:12], 3, 5)
    assert e.value.code == _lib.EON_E_SHAPE


def test_native_rccl_collective_single_rank(gpu_ctx):
    """The driver's RCCL eon_collective (used at N > 1 GPUs) initialises and all-gathers on device
    with one rank (RCCL allows one rank per GPU, so this is all one box can run)."""
    import ctypes

    import torch

    from plonky3_eon_amd.native import RcclCollective

    coll = RcclCollective(0, 1)
    src = torch.arange(1000, dtype=torch.uint8, device="cuda:0")
    dst = torch.zeros_like(src)
    stream = torch.cuda.current_stream().cuda_stream
    rc = coll.c.all_gather(None if coll.c.user is None else coll.c.user, ctypes.c_void_p(src.data_ptr()),
                           ctypes.c_void_p(dst.data_ptr()), 1000, ctypes.c_void_p(stream))
    torch.cuda.synchronize()
    assert rc == 0
    assert torch.equal(src, dst)
    coll.close()
