"""CPU: the verifier restatement (oracle/verify_oracle.py) accepts the CPU restatement's own
proofs (oracle/prove_oracle.py: the reference's algorithms) and rejects tampered ones -- so it
can be trusted as the validity check of the full-size GPU proof (tests/test_gpu_prove_full.py)."""

import copy

import numpy as np
import pytest

from oracle import coracle as C
from oracle import prove_oracle
from oracle import pyoracle as O
from oracle import verify_oracle as V
from oracle.smallrng import SmallRng, poseidon2_new_from_rng

HF, PR = 4, 56


def lim(x):
    return np.array(O.int_to_limbs(O.to_mont(x)), dtype=np.uint64)


@pytest.fixture(scope="module")
def setup():
    py = O.p2_constants(2024, HF, PR)
    consts = C.P2Constants([[lim(x) for x in r] for r in py[0]], [lim(x) for x in py[1]],
                           [[lim(x) for x in r] for r in py[2]])
    log_n, vl = 4, 2
    n = 1 << log_n
    inputs = C.random_fr(17, n * vl * 3).reshape(n * vl, 3, 4)
    trace = C.p2_generate_trace(inputs, vl, consts)
    srs = C.g1_srs(n + 1, C.fr_from_u64(12345))
    chc = O.p2_constants(99, 2, 22)
    d = prove_oracle.prove(trace, srs, consts, vl, None, None, challenger=O.DuplexChallenger(chc))
    return py, chc, log_n, vl, trace, V.proof_from_oracle(d)


def _verify(setup, proof, with_trace=True):
    py, chc, log_n, vl, trace, _ = setup
    return V.verify_kzg_proof(proof, V.p2air_constraint_fn(py, vl), log_n, 1, 12345,
                              challenger=O.DuplexChallenger(chc), trace=trace if with_trace else None)


def test_accepts_oracle_proof(setup):
    res = _verify(setup, setup[5])
    assert res == {"transcript": True, "ood": True, "opened_vs_trace": True, "kzg": True}


def test_selectors_at_point_match_coset_selectors():
    """selectors_at_point (domain.rs:237-246) at the points of the quotient coset equal
    selectors_on_coset (domain.rs:252-292) there."""
    log_n, log_q = 3, 4
    sel = O.selectors_on_coset(log_n, log_q, O.GENERATOR)
    gq = O.two_adic_generator(log_q)
    for i in (0, 5, 15):
        x = O.GENERATOR * pow(gq, i, O.P) % O.P
        assert V.selectors_at_point(log_n, x) == tuple(s[i] for s in sel)


@pytest.mark.parametrize("what", ["trace_value", "next_value", "quotient_value", "witness", "commit",
                                  "quotient_commit"])
def test_rejects_tampered(setup, what):
    p = copy.deepcopy(setup[5])
    one = lim(1)
    if what == "trace_value":
        v = p.opened[0].values[0][0]
        v[3] = C.fr_mul(v[3], C.fr_from_u64(2)) if np.any(v[3]) else one
    elif what == "next_value":
        v = p.opened[0].values[0][1]
        v[0] = C.fr_mul(v[0], C.fr_from_u64(3)) if np.any(v[0]) else one
    elif what == "quotient_value":
        v = p.opened[1].values[1][0]
        v[0] = C.fr_mul(v[0], C.fr_from_u64(3)) if np.any(v[0]) else one
    elif what == "witness":
        w = p.opened[0].witnesses[0][0]
        w[2] = C.g1_add(w[2], C.g1_generator())
    elif what == "commit":
        p.trace_commit[0][1] = C.g1_add(p.trace_commit[0][1], C.g1_generator())
    else:
        p.quotient_commit[0] = C.g1_add(np.asarray(p.quotient_commit[0]).reshape(8), C.g1_generator())
    res = _verify(setup, p)
    assert not all(res.values()), res


@pytest.mark.parametrize("n,x,ok", [(1, 1, True), (8, 21, True), (8, 123123, False)])
def test_fibonacci_oracle_prove_verifies(n, x, ok):
    """fib_air.rs:112-155 on the CPU restatement: prove + verify for n = 1 and 8 with publics
    (0, 1, F_n); the incorrect public value yields a proof whose OOD identity fails."""
    chc = poseidon2_new_from_rng(SmallRng.seed_from_u64(1), 4, 22)  # fib_air.rs:113-115
    pis = [0, 1, x]
    trace = np.stack([np.stack([lim(v) for v in r]) for r in O.fib_trace(0, 1, n)])
    srs = C.g1_srs(1025, C.fr_from_u64(12345))
    d = prove_oracle.prove(trace, srs, None, None, None, None, log_qd=0, challenger=O.DuplexChallenger(chc),
                           constraint_fn=O.fib_constraints, publics=pis)
    res = V.verify_kzg_proof(V.proof_from_oracle(d), V.fib_constraint_fn(pis), n.bit_length() - 1, 0, 12345,
                             challenger=O.DuplexChallenger(chc), trace=trace, publics=pis, pairing=True)
    assert res["transcript"] and res["kzg"] and res["opened_vs_trace"]
    assert res["kzg_pairing"]  # KzgPcs::verify's verify_batch with the pairing restatement
    assert res["ood"] == ok
