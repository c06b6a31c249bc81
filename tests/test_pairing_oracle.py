"""The BN254 pairing restatement (oracle/pairing.py) that stands in for halo2curves'
multi_miller_loop + final_exponentiation (bn254/src/curve.rs:429-452), pinned by the group laws and
by the reference's own KZG tests restated (kzg/src/tests.rs:20-47 pcs_roundtrip, :73-136
test_batch_verification) through verify_single / verify_batch (kzg/src/util.rs:150-168, 245-292)."""

import pytest

from oracle import pairing as E
from oracle import pyoracle as O


def test_generators_and_torsion():
    assert O.g1_is_on_curve(E.G1_GEN) and E.g2_on_curve(E.G2_GEN)
    assert E.g2_add(E.g2_mul(E.G2_GEN, E.R - 1), E.G2_GEN) is None  # r G2 = O
    assert O.g1_add(O.g1_mul(E.G1_GEN, E.R - 1), E.G1_GEN) is None  # r G1 = O


def test_bilinear_and_nondegenerate():
    e = E.pairing(E.G1_GEN, E.G2_GEN)
    assert e != E.f12_one() and E.f12_pow(e, E.R) == E.f12_one()
    a, b = 12345, 678
    lhs = E.pairing(E.g1_mul(E.G1_GEN, a), E.g2_mul(E.G2_GEN, b))
    assert lhs == E.f12_pow(e, a * b)
    assert E.pairing(None, E.G2_GEN) == E.f12_one() and E.pairing(E.G1_GEN, None) == E.f12_one()
    # e(P, Q) e(-P, Q) = 1 through one final exponentiation (multi_pairing)
    assert E.multi_pairing([(E.G1_GEN, E.G2_GEN), (E.g1_neg(E.G1_GEN), E.G2_GEN)]) == E.f12_one()


def _commit(srs, coeffs):
    return O.commit_column(srs, coeffs)


def _quotient(coeffs, z):
    """quotient_and_eval (kzg/src/util.rs:100-111) over ints."""
    n = len(coeffs)
    q = [0] * (n - 1)
    carry = coeffs[-1]
    for i in range(n - 2, -1, -1):
        q[i] = carry
        carry = (coeffs[i] + carry * z) % O.P
    return q, carry


def test_reference_batch_verification():
    """kzg/src/tests.rs:73-136: alpha 42, SRS 16, two polynomials opened at 2 and 3."""
    alpha = 42
    srs = O.init_srs_g1(16, alpha)
    g2a = E.g2_alpha(alpha)
    p1, p2 = [1, 2, 3], [5, 7, 11]
    c1, c2 = _commit(srs, p1), _commit(srs, p2)
    z1, z2 = 2, 3
    v1 = 1 + 2 * z1 + 3 * z1 * z1  # 17
    v2 = 5 + 7 * z2 + 11 * z2 * z2  # 125
    w1 = _commit(srs, [2 + 3 * z1, 3])
    w2 = _commit(srs, [7 + 11 * z2, 11])
    assert (v1, v2) == (17, 125)
    assert E.verify_batch([(c1, w1, v1, z1), (c2, w2, v2, z2)], g2a)
    assert not E.verify_batch([(c1, w1, v1 + 1, z1), (c2, w2, v2, z2)], g2a)
    assert E.verify_batch([], g2a)


def test_reference_pcs_roundtrip():
    """kzg/src/tests.rs:20-47: alpha 7, SRS max degree 8, the 2^3 subgroup, evaluations x + 1
    (coefficients (1, 1, 0, ...)), opened at 2: value 3, and the opening verifies."""
    alpha = 7
    srs = O.init_srs_g1(8, alpha)
    g2a = E.g2_alpha(alpha)
    w = O.two_adic_generator(3)
    evals = [(pow(w, i, O.P) + 1) % O.P for i in range(8)]
    coeffs = [r[0] for r in O.idft([[e] for e in evals])]  # coset_idft_batch, shift 1 (pcs.rs:242)
    assert coeffs[:2] == [1, 1] and not any(coeffs[2:])
    c = _commit(srs, coeffs)
    q, v = _quotient(coeffs, 2)
    assert v == 3
    wit = _commit(srs, q)
    assert E.verify_single(c, wit, v, 2, g2a)
    assert E.verify_batch([(c, wit, v, 2)], g2a)
    assert not E.verify_single(c, wit, v, 5, g2a)
