"""The generic quotient path (eon_air_program / eon_quotient_values_dev, eon_prove_air*) on the GPU:

* quotient_values of FibonacciAir (eon-uni-stark/tests/fib_air.rs) and of an AIR exercising every
  node kind, against the oracle's quotient_values_fn with constraints written out directly;
* the Poseidon2-AIR compiled from its symbolic eval equals the fused kernel and the C oracle;
* the reference's end-to-end Fibonacci tests (fib_air.rs:112-135: n = 1 and n = 8, publics
  (0, 1, F_n), KzgPcs max_degree 1024 with alpha = 12345, Fiat-Shamir) prove on the GPU bit-exact
  against the CPU restatement and verify; the incorrect-public-value case does not verify;
* MulAir (uni-stark/tests/mul_air.rs: degree 3, 60 columns, boundary + transition constraints,
  two quotient chunks) likewise, and its invalid trace (c doubled) does not verify.

Parity note: the Fibonacci tests' challenger permutation is the reference's own
`Perm::new_from_rng(4, 22, SmallRng::seed_from_u64(1))` (fib_air.rs:113-115) through the restated
rand 0.9 SmallRng (oracle/smallrng.py, Xoshiro256++ pinned by its published vector); the
compressed-G1 transcript bytes stay unpinned."""

import numpy as np
import pytest

from airs import FibonacciAir, MixedAir, MockAir, MulAir
from oracle import coracle as C
from oracle import prove_oracle
from oracle import pyoracle as O
from oracle import verify_oracle as V
from oracle.smallrng import SmallRng, poseidon2_new_from_rng

pytestmark = pytest.mark.gpu
P = O.P


def lim(x):
    return np.array(O.int_to_limbs(O.to_mont(x % P)), dtype=np.uint64)


def ints(a):
    return [O.from_mont(O.limbs_to_int([int(v) for v in e])) for e in np.asarray(a, dtype=np.uint64).reshape(-1, 4)]


def mixed_constraints(loc, nxt, sels, pub):
    first, last, trans = sels
    s = (loc[0] + 3 * loc[1]) % P
    return [(s * s - nxt[2]) % P, first * (loc[3] - pub[0]) % P, last * ((-loc[4] + pub[1]) - 1) % P,
            trans * (nxt[0] - (pow(s, 5, P) - pow(loc[2], 7, P))) % P, (1 - loc[1]) * loc[1] % P,
            (loc[2] - 7) * loc[3] * nxt[4] % P, (loc[2] - 7) * (-(nxt[1] - 11)) % P, s, loc[4]]


@pytest.mark.parametrize("air_cls,fn,log_n,log_qd", [
    (FibonacciAir, O.fib_constraints, 0, 0), (FibonacciAir, O.fib_constraints, 3, 0),
    (FibonacciAir, O.fib_constraints, 4, 1), (FibonacciAir, O.fib_constraints, 2, 2),
    (MixedAir, mixed_constraints, 3, 3), (MixedAir, mixed_constraints, 5, 3)])
def test_quotient_values_vs_oracle(gpu_ctx, air_cls, fn, log_n, log_qd):
    import torch

    from plonky3_eon_amd.air import AirProgram

    air = air_cls()
    prog = AirProgram(air, gpu_ctx)
    if air_cls is MixedAir:
        assert prog.max_constraint_degree == 7 and prog.log_quotient_degree() == 3
    q = 1 << (log_n + log_qd)
    lde = C.random_fr(log_n * 7 + log_qd, q * prog.width).reshape(q, prog.width, 4)
    pub = [int(x) for x in ints(C.random_fr(99 + log_n, prog.n_public))]
    alpha = 0x1234567890ABCDEF1234567
    got = prog.quotient_values(torch.from_numpy(lde.view(np.int64)).to("cuda:0"), log_n, log_qd, alpha, pub)
    got = ints(got.cpu().numpy().view(np.uint64))
    want = O.quotient_values_fn([ints(r) for r in lde], log_n, log_qd, fn, alpha, pub)
    assert got == want


@pytest.mark.parametrize("specs", [[(0, 1)], [(0, 0), (1, 2)], [(1, 0), (0, 2), (0, 1)],
                                   [(0, 0), (0, 1), (1, 1), (0, 2)]])
def test_constraint_pairing_edges(gpu_ctx, specs):
    """The device folds constraints in pairs (acc alpha^2 + C_k alpha + C_k+1, one reduction); an
    odd count opens the chain with a lone constraint.  1-4 constraints (MockAir leaves) against the
    oracle's one-at-a-time Horner fold."""
    import torch

    from plonky3_eon_amd.air import AirProgram

    air = MockAir(specs, 3)
    prog = AirProgram(air, gpu_ctx)
    assert prog.num_constraints == len(specs)
    log_n, log_qd = 3, 1
    q = 1 << (log_n + log_qd)
    lde = C.random_fr(40 + len(specs), q * prog.width).reshape(q, prog.width, 4)
    alpha = 0x2F1E0D0C0B0A09080706050403020100
    got = prog.quotient_values(torch.from_numpy(lde.view(np.int64)).to("cuda:0"), log_n, log_qd, alpha, [])
    got = ints(got.cpu().numpy().view(np.uint64))

    def fn(loc, nxt, sels, pub):
        return [(loc if o == 0 else nxt)[i] for o, i in specs]

    want = O.quotient_values_fn([ints(r) for r in lde], log_n, log_qd, fn, alpha, [])
    assert got == want


def test_register_file_modes(gpu_ctx):
    """The two register files of k_air_quotient -- LDS (the default) and global memory
    (EON_AIR_REGS=global) -- give the same values (run in child processes: the knob is read once
    per process); the default run is checked against the oracle by test_quotient_values_vs_oracle."""
    import os
    import subprocess
    import sys

    code = ("import numpy as np, torch, sys; sys.path[:0] = ['tests', '.'];"
            "from airs import MixedAir; from plonky3_eon_amd import Context; from plonky3_eon_amd.air import AirProgram;"
            "from oracle import coracle as C;"
            "ctx = Context(0); prog = AirProgram(MixedAir(), ctx);"
            "lde = C.random_fr(5, 64 * 5).reshape(64, 5, 4);"
            "out = prog.quotient_values(torch.from_numpy(lde.view(np.int64)).to('cuda:0'), 3, 3, 77, [5, 6]);"
            "np.save(sys.argv[1], out.cpu().numpy())")
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        outs = []
        for mode in ("lds", "global"):
            f = os.path.join(d, mode + ".npy")
            env = dict(os.environ, EON_AIR_REGS=mode)
            subprocess.run([sys.executable, "-c", code, f], check=True, env=env, timeout=300)
            outs.append(np.load(f))
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("vl,log_n", [(1, 3), (2, 4)])
def test_poseidon2_generic_equals_fused(gpu_ctx, vl, log_n):
    import torch

    from plonky3_eon_amd.air import AirProgram, Poseidon2Air

    py = O.p2_constants(2024, 4, 56)
    k = C.P2Constants([[lim(v) for v in r] for r in py[0]], [lim(v) for v in py[1]],
                      [[lim(v) for v in r] for r in py[2]])
    air = Poseidon2Air(k.begin, k.partial, k.end, vl, gpu_ctx)
    prog = AirProgram(air, gpu_ctx)
    assert prog.num_constraints == 160 * vl and prog.max_constraint_degree == 3
    # CSE: shared round-constant sums and external-layer sums evaluated once
    assert prog.stats["num_instructions"] < 8 * 160 * vl, prog.stats
    log_qd = 1
    q = 1 << (log_n + log_qd)
    lde = C.random_fr(vl + log_n, q * air.width).reshape(q, air.width, 4)
    dev = torch.from_numpy(lde.view(np.int64)).to("cuda:0")
    alpha = 0xABCDEF0123456789
    generic = prog.quotient_values(dev, log_n, log_qd, alpha).cpu().numpy()
    fused = air.quotient_values(dev, log_n, log_qd, alpha).cpu().numpy()
    np.testing.assert_array_equal(generic, fused)
    want = C.p2_quotient_values(lde, log_n, log_qd, vl, k, lim(alpha))
    np.testing.assert_array_equal(generic.view(np.uint64), want)


def test_poseidon2_vl8_generic_equals_fused_2_12(gpu_ctx):
    """The headline AIR (VECTOR_LEN 8: 1312 columns, 1280 constraints) through the generic program
    equals the fused kernel on a 2^12-row trace (2^13 quotient rows)."""
    import torch

    from plonky3_eon_amd.air import AirProgram, Poseidon2Air

    py = O.p2_constants(2024, 4, 56)
    k = C.P2Constants([[lim(v) for v in r] for r in py[0]], [lim(v) for v in py[1]],
                      [[lim(v) for v in r] for r in py[2]])
    air = Poseidon2Air(k.begin, k.partial, k.end, 8, gpu_ctx)
    prog = AirProgram(air, gpu_ctx)
    assert prog.num_constraints == 1280 and air.width == 1312
    log_n, log_qd = 12, 1
    q = 1 << (log_n + log_qd)
    # full-range canonical residues (the top limb unmasked: values up to p - 1, so the interpreter's
    # 12p reduce threshold and the fused kernel's bounds see their worst operands)
    host_lde = C.random_fr(1212, q * air.width).reshape(q, air.width, 4)
    host_lde[::7, ::5] = np.array(O.int_to_limbs(P - 1), dtype=np.uint64)
    lde = torch.from_numpy(host_lde.view(np.int64)).to("cuda:0")
    alpha = O.from_mont(P - 1)  # stored residue p - 1
    generic = prog.quotient_values(lde, log_n, log_qd, alpha)
    fused = air.quotient_values(lde, log_n, log_qd, alpha)
    assert torch.equal(generic, fused)  # the fused kernel is oracle-checked at VECTOR_LEN 1/2/8


def test_program_rejects_bad_input(gpu_ctx):
    import ctypes

    import torch

    from plonky3_eon_amd import _lib
    from plonky3_eon_amd.air import AirProgram

    lib = gpu_ctx.lib
    h = ctypes.c_void_p()
    consts = np.zeros((1, 4), np.uint64)
    roots = np.array([0], np.uint32)

    def create(nodes, width=2, npub=0):
        arr = (_lib.eon_sym_node * len(nodes))(*[_lib.eon_sym_node(*n) for n in nodes])
        return lib.eon_air_program_create(gpu_ctx.handle, arr, len(nodes), consts.ctypes.data_as(ctypes.c_void_p), 1,
                                          roots.ctypes.data_as(ctypes.c_void_p), 1, width, npub, ctypes.byref(h))

    assert create([(10, 0, 0)]) == _lib.EON_E_ARG  # preprocessed: not supported
    assert create([(11, 0, 0)]) == _lib.EON_E_ARG  # permutation (LogUp)
    assert create([(6, 0, 0)]) == _lib.EON_E_ARG  # operand does not precede its user
    assert create([(1, 5, 0)]) == _lib.EON_E_ARG  # column out of range
    assert create([(2, 0, 0)]) == _lib.EON_E_ARG  # public index out of range (no publics)
    # operand indices are 28 bits (bit 28 is the raw flag): wider widths / slot counts are shape errors
    assert create([(1, 0, 0)], width=1 << 28) == _lib.EON_E_SHAPE
    assert create([(1, 0, 0)], width=2, npub=(1 << 28) - 1) == _lib.EON_E_SHAPE
    prog = AirProgram(FibonacciAir(), gpu_ctx)
    lde = torch.zeros((8, 2, 4), dtype=torch.int64, device="cuda:0")
    with pytest.raises(_lib.EonError) as e:
        prog.quotient_values(lde, 3, 0, 5, [0, 1])  # 2 publics for a 3-public program
    assert e.value.code == _lib.EON_E_SHAPE


@pytest.fixture(scope="module")
def ch_consts():
    # the reference's own challenger permutation: Perm::new_from_rng(4, 22, SmallRng(1))
    # (fib_air.rs:113-115), through the restated rand 0.9 SmallRng (oracle/smallrng.py)
    py = poseidon2_new_from_rng(SmallRng.seed_from_u64(1), 4, 22)
    return py, ([[lim(v) for v in r] for r in py[0]], [lim(v) for v in py[1]], [[lim(v) for v in r] for r in py[2]])


@pytest.mark.parametrize("n,x", [(1, 1), (8, 21)])
def test_fibonacci_prove_vs_oracle_and_verify(gpu_ctx, ch_consts, n, x):
    """fib_air.rs:112-135 test_one_row_trace / test_public_value."""
    import torch

    from plonky3_eon_amd.air import AirProgram
    from plonky3_eon_amd.native import Challenger, NativeKzgPcs, Poseidon2Constants, prove_native

    py, limbs = ch_consts
    pis = [0, 1, x]
    trace_rows = O.fib_trace(0, 1, n)
    trace = np.stack([np.stack([lim(v) for v in r]) for r in trace_rows])
    prog = AirProgram(FibonacciAir(), gpu_ctx)
    pcs = NativeKzgPcs(1024, 12345, gpu_ctx)
    proof = prove_native(prog, pcs, torch.from_numpy(trace.view(np.int64)).to("cuda:0"), None, None,
                         challenger=Challenger(Poseidon2Constants(*limbs)), public_values=pis)
    pcs.close()
    assert proof.degree_bits == n.bit_length() - 1

    srs = C.g1_srs(1025, C.fr_from_u64(12345))
    want = prove_oracle.prove(trace, srs, None, None, None, None, log_qd=0, challenger=O.DuplexChallenger(py),
                              constraint_fn=O.fib_constraints, publics=pis)
    assert (proof.alpha, proof.zeta) == (want["alpha"], want["zeta"])
    np.testing.assert_array_equal(proof.trace_commit[0], want["trace_commit"])
    np.testing.assert_array_equal(np.stack([c[0] for c in proof.quotient_commit]), want["quotient_commit"])
    for p in range(2):
        np.testing.assert_array_equal(proof.opened[0].values[0][p], want["trace_open"][0][p])
        np.testing.assert_array_equal(proof.opened[0].witnesses[0][p], want["trace_open"][1][p])
    np.testing.assert_array_equal(proof.opened[1].values[0][0], want["quotient_open"][0][0][0])
    np.testing.assert_array_equal(proof.opened[1].witnesses[0][0], want["quotient_open"][0][1][0])
    res = V.verify_kzg_proof(proof, V.fib_constraint_fn(pis), n.bit_length() - 1, 0, 12345,
                             challenger=O.DuplexChallenger(py), trace=trace, publics=pis, pairing=True)
    assert res == {"transcript": True, "ood": True, "opened_vs_trace": True, "kzg": True,
                   "kzg_pairing": True}, res


def test_fibonacci_incorrect_public_value_does_not_verify(gpu_ctx, ch_consts):
    """fib_air.rs:138-155: x = 123123 is not F_8.  The reference panics in its debug-only
    check_constraints; here the proof is produced and the verifier's OOD identity fails."""
    import torch

    from plonky3_eon_amd.air import AirProgram
    from plonky3_eon_amd.native import Challenger, NativeKzgPcs, Poseidon2Constants, prove_native

    py, limbs = ch_consts
    pis = [0, 1, 123123]
    trace = np.stack([np.stack([lim(v) for v in r]) for r in O.fib_trace(0, 1, 8)])
    prog = AirProgram(FibonacciAir(), gpu_ctx)
    pcs = NativeKzgPcs(1024, 12345, gpu_ctx)
    proof = prove_native(prog, pcs, torch.from_numpy(trace.view(np.int64)).to("cuda:0"), None, None,
                         challenger=Challenger(Poseidon2Constants(*limbs)), public_values=pis)
    pcs.close()
    res = V.verify_kzg_proof(proof, V.fib_constraint_fn(pis), 3, 0, 12345, challenger=O.DuplexChallenger(py),
                             publics=pis)
    assert res["transcript"] and res["kzg"] and not res["ood"]


def test_poseidon2_generic_prove_equals_fused_prove(gpu_ctx):
    """The whole proof of the Poseidon2-AIR through the generic program equals the fused one."""
    import torch

    from plonky3_eon_amd.air import AirProgram, Poseidon2Air
    from plonky3_eon_amd.native import NativeKzgPcs, prove_native

    py = O.p2_constants(2024, 4, 56)
    k = C.P2Constants([[lim(v) for v in r] for r in py[0]], [lim(v) for v in py[1]],
                      [[lim(v) for v in r] for r in py[2]])
    air = Poseidon2Air(k.begin, k.partial, k.end, 2, gpu_ctx)
    n = 1 << 5
    inputs = C.random_fr(31, n * 2 * 3).reshape(n * 2, 3, 4)
    trace = air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to("cuda:0"))
    pcs = NativeKzgPcs(n, 12345, gpu_ctx)
    a, z = 0x1111, 0x2222
    fused = prove_native(air, pcs, trace, a, z)
    generic = prove_native(AirProgram(air, gpu_ctx), pcs, trace, a, z)
    pcs.close()
    np.testing.assert_array_equal(fused.trace_commit[0], generic.trace_commit[0])
    for c in range(2):
        np.testing.assert_array_equal(fused.quotient_commit[c], generic.quotient_commit[c])
        np.testing.assert_array_equal(fused.opened[1].witnesses[c][0], generic.opened[1].witnesses[c][0])


def mul_constraints(loc, nxt, sels, pub):
    """MulAir (uni-stark/tests/mul_air.rs:96-118) written out directly, in eval order."""
    first, _, trans = sels
    out = []
    for i in range(MulAir.REPETITIONS):
        a, b, c = loc[3 * i], loc[3 * i + 1], loc[3 * i + 2]
        out += [(a * a * b - c) % P, first * (a * a + 1 - b) % P, trans * (a + MulAir.REPETITIONS - nxt[3 * i]) % P]
    return out


def mul_trace(rows: int, valid: bool = True):
    """random_valid_trace (mul_air.rs:55-81) with degree 3 and both constraint kinds: a = the
    triple's index, b = a^2 + 1 on the first row and random elsewhere, c = a^2 b (doubled when
    invalid); randomness from the in-repo PRNG."""
    rng = O.SplitMix64(7)
    reps = MulAir.REPETITIONS
    t = []
    for i in range(rows * reps):
        a = i % P
        b = (a * a + 1) % P if i // reps == 0 else rng.fr_mont() % P
        c = a * a * b % P
        t.append([a, b, c * (2 if not valid else 1) % P])
    return [sum(t[r * reps:(r + 1) * reps], []) for r in range(rows)]


@pytest.mark.parametrize("log_n,valid", [(3, True), (5, True), (3, False)])
def test_mul_air_prove_vs_oracle_and_verify(gpu_ctx, ch_consts, log_n, valid):
    import torch

    from plonky3_eon_amd.air import AirProgram
    from plonky3_eon_amd.native import Challenger, NativeKzgPcs, Poseidon2Constants, prove_native

    py, limbs = ch_consts
    n = 1 << log_n
    rows = mul_trace(n, valid)
    trace = np.stack([np.stack([lim(v) for v in r]) for r in rows])
    prog = AirProgram(MulAir(), gpu_ctx)
    assert prog.max_constraint_degree == 3 and prog.log_quotient_degree() == 1
    assert prog.num_constraints == 3 * MulAir.REPETITIONS
    pcs = NativeKzgPcs(1024, 12345, gpu_ctx)
    proof = prove_native(prog, pcs, torch.from_numpy(trace.view(np.int64)).to("cuda:0"), None, None,
                         challenger=Challenger(Poseidon2Constants(*limbs)))
    pcs.close()
    res = V.verify_kzg_proof(proof, lambda loc, nxt, sels: mul_constraints(loc, nxt, sels[:3], ()), log_n, 1, 12345,
                             challenger=O.DuplexChallenger(py), trace=trace)
    if not valid:
        assert res["transcript"] and res["kzg"] and not res["ood"], res
        return
    assert res == {"transcript": True, "ood": True, "opened_vs_trace": True, "kzg": True}, res
    srs = C.g1_srs(1025, C.fr_from_u64(12345))
    want = prove_oracle.prove(trace, srs, None, None, None, None, log_qd=1, challenger=O.DuplexChallenger(py),
                              constraint_fn=mul_constraints, publics=[])
    assert (proof.alpha, proof.zeta) == (want["alpha"], want["zeta"])
    np.testing.assert_array_equal(proof.trace_commit[0], want["trace_commit"])
    np.testing.assert_array_equal(np.stack([c[0] for c in proof.quotient_commit]), want["quotient_commit"])
    for p in range(2):
        np.testing.assert_array_equal(proof.opened[0].values[0][p], want["trace_open"][0][p])
        np.testing.assert_array_equal(proof.opened[0].witnesses[0][p], want["trace_open"][1][p])


PM1 = np.array(O.int_to_limbs(P - 1), dtype=np.uint64)


def extreme_lde(kind, rows, width, seed):
    out = np.zeros((rows, width, 4), dtype=np.uint64)
    if kind == "pm1":
        out[:] = PM1
    elif kind == "alt":
        out[(np.add.outer(np.arange(rows), np.arange(width)) % 2) == 0] = PM1
    elif kind == "alt_rows":
        out[::2] = PM1
    else:
        out[:] = C.random_fr(seed, rows * width).reshape(rows, width, 4)
        out[np.random.default_rng(seed).random((rows, width)) < 0.25] = PM1
    return out


@pytest.mark.parametrize("kind", ["pm1", "alt", "alt_rows", "rand_pm1"])
def test_generic_quotient_extreme_mixed(gpu_ctx, kind):
    """k_air_quotient's bound tracking (reduce above 12p, raw leaves of bound 32, K p offsets of the
    differences) at its worst operands: every LDE cell, public value and alpha stored as p - 1, or
    p - 1 next to 0, against the oracle's fully reduced fold (MixedAir: every node kind, degree 7)."""
    import torch

    from plonky3_eon_amd.air import AirProgram

    prog = AirProgram(MixedAir(), gpu_ctx)
    for log_n, log_qd in ((3, 3), (2, 1)):
        q = 1 << (log_n + log_qd)
        lde = extreme_lde(kind, q, prog.width, 5 + log_n)
        for pub, alpha in (([P - 1, P - 1], P - 1), ([0, P - 1], 0x1234567890ABCDEF1234567)):
            # public values and alpha are canonical ints given in the Montgomery domain by the
            # binding; P - 1 as a residue is from_mont(P - 1)
            pub_i = [O.from_mont(v) for v in pub]
            alpha_i = O.from_mont(alpha) if alpha == P - 1 else alpha
            got = prog.quotient_values(torch.from_numpy(lde.view(np.int64)).to("cuda:0"), log_n, log_qd, alpha_i, pub_i)
            got = ints(got.cpu().numpy().view(np.uint64))
            want = O.quotient_values_fn([ints(r) for r in lde], log_n, log_qd, mixed_constraints, alpha_i, pub_i)
            assert got == want, (kind, log_n, pub, hex(alpha))


@pytest.mark.parametrize("vl", [1, 8])
@pytest.mark.parametrize("kind", ["pm1", "alt", "rand_pm1"])
def test_generic_quotient_extreme_poseidon2(gpu_ctx, vl, kind):
    """The Poseidon2-AIR through the generic program at worst-case LDE values, with every round
    constant stored as p - 1, against the C oracle (VECTOR_LEN 1 and 8)."""
    import torch

    from plonky3_eon_amd.air import AirProgram, Poseidon2Air

    hf, pr = 4, 56
    k = C.P2Constants([[PM1.copy() for _ in range(3)] for _ in range(hf)], [PM1.copy() for _ in range(pr)],
                      [[PM1.copy() for _ in range(3)] for _ in range(hf)])
    air = Poseidon2Air(k.begin, k.partial, k.end, vl, gpu_ctx)
    prog = AirProgram(air, gpu_ctx)
    log_n, log_qd = 3, 1
    q = 1 << (log_n + log_qd)
    lde = extreme_lde(kind, q, air.width, 70 + vl)
    dev = torch.from_numpy(lde.view(np.int64)).to("cuda:0")
    alpha_i = O.from_mont(P - 1)
    generic = prog.quotient_values(dev, log_n, log_qd, alpha_i).cpu().numpy().view(np.uint64)
    want = C.p2_quotient_values(lde, log_n, log_qd, vl, k, PM1)
    np.testing.assert_array_equal(generic, want)
    fused = air.quotient_values(dev, log_n, log_qd, alpha_i).cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(fused, want)
