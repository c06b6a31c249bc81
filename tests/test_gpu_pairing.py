"""N4 on the GPU: G2 scalar multiplication, multi_pairing and verify_batch (include/eon.h,
csrc/pairing.hip) against the pairing restatement oracle/pairing.py (itself pinned by the group laws
and the reference's KZG tests, tests/test_pairing_oracle.py):

* g2_mul == g2_alpha (init_srs_unsafe, kzg/src/params.rs:123-139);
* multi_pairing (bn254/src/curve.rs:439-452) == the oracle's Gt element, bit for bit, for single
  pairings, products, identity inputs, and bilinearity;
* verify_batch / verify_single (kzg/src/util.rs:150-168, 245-292): the reference's
  kzg/src/tests.rs:20-47 (pcs_roundtrip) and :73-136 (test_batch_verification) cases, a tampered
  value / witness / point, and openings that share points (the merged-pair path).
"""

import numpy as np
import pytest

from oracle import pairing as E
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


def g1_limbs(p):
    if p is None:
        return np.zeros(8, dtype=np.uint64)
    return np.array(O.int_to_limbs(O.fq_to_mont(p[0])) + O.int_to_limbs(O.fq_to_mont(p[1])), dtype=np.uint64)


def g2_limbs(q):
    if q is None:
        return np.zeros(16, dtype=np.uint64)
    (x0, x1), (y0, y1) = q
    out = []
    for v in (x0, x1, y0, y1):
        out += O.int_to_limbs(O.fq_to_mont(v))
    return np.array(out, dtype=np.uint64)


def fr_limbs(x):
    return np.array(O.int_to_limbs(O.to_mont(x % O.P)), dtype=np.uint64)


def gt_limbs(f):
    """oracle Fq12 (w-basis, w^12 = 18 w^6 - 82) -> the tower layout of eon_fq12: the coefficient
    of w^k (k = 2j + i) is a + b u with u = w^6 - 9, i.e. flat[k] = a - 9 b, flat[k + 6] = b."""
    out = np.zeros((12, 4), dtype=np.uint64)
    for i in range(2):
        for j in range(3):
            k = 2 * j + i
            b = f[k + 6] % O.Q
            a = (f[k] + 9 * b) % O.Q
            m = 3 * i + j
            out[2 * m] = O.int_to_limbs(O.fq_to_mont(a))
            out[2 * m + 1] = O.int_to_limbs(O.fq_to_mont(b))
    return out


def test_g2_mul_matches_oracle(gpu_ctx):
    from plonky3_eon_amd import verify as V

    for k in (1, 2, 42, 12345, O.P - 1, 0x1234567890ABCDEF1234567890ABCDEF):
        np.testing.assert_array_equal(V.g2_mul(k, ctx=gpu_ctx), g2_limbs(E.g2_mul(E.G2_GEN, k)), err_msg=f"k={k}")
    assert not V.g2_mul(0, ctx=gpu_ctx).any()  # identity
    base = g2_limbs(E.g2_mul(E.G2_GEN, 7))
    np.testing.assert_array_equal(V.g2_mul(3, base=base, ctx=gpu_ctx), g2_limbs(E.g2_mul(E.G2_GEN, 21)))


def test_pairing_matches_oracle(gpu_ctx):
    from plonky3_eon_amd import verify as V

    p, q = O.g1_mul(E.G1_GEN, 5), E.g2_mul(E.G2_GEN, 11)
    got = V.pairing(g1_limbs(p), g2_limbs(q), ctx=gpu_ctx)
    np.testing.assert_array_equal(got, gt_limbs(E.pairing(p, q)))
    # the generator pairing and bilinearity e(aP, bQ) = e(abP, Q)
    np.testing.assert_array_equal(V.pairing(g1_limbs(E.G1_GEN), g2_limbs(E.G2_GEN), ctx=gpu_ctx),
                                  gt_limbs(E.pairing(E.G1_GEN, E.G2_GEN)))
    np.testing.assert_array_equal(V.pairing(g1_limbs(O.g1_mul(E.G1_GEN, 55)), g2_limbs(E.G2_GEN), ctx=gpu_ctx), got)


def test_multi_pairing_matches_oracle(gpu_ctx):
    from plonky3_eon_amd import verify as V

    pairs = [(O.g1_mul(E.G1_GEN, 3), E.g2_mul(E.G2_GEN, 5)), (O.g1_mul(E.G1_GEN, 7), E.G2_GEN),
             (None, E.G2_GEN), (E.G1_GEN, None), (O.g1_mul(E.G1_GEN, 0xABCDEF), E.g2_mul(E.G2_GEN, 0x1357))]
    got = V.multi_pairing(np.stack([g1_limbs(p) for p, _ in pairs]), np.stack([g2_limbs(q) for _, q in pairs]),
                          ctx=gpu_ctx)
    np.testing.assert_array_equal(got, gt_limbs(E.multi_pairing(pairs)))
    # e(P, Q) e(-P, Q) = 1; the empty product is 1
    one = gt_limbs(E.f12_one())
    cancel = V.multi_pairing(np.stack([g1_limbs(E.G1_GEN), g1_limbs(E.g1_neg(E.G1_GEN))]),
                             np.stack([g2_limbs(E.G2_GEN)] * 2), ctx=gpu_ctx)
    np.testing.assert_array_equal(cancel, one)
    np.testing.assert_array_equal(V.multi_pairing(np.zeros((0, 8), np.uint64), np.zeros((0, 16), np.uint64),
                                                  ctx=gpu_ctx), one)


def test_rejects_points_off_the_curve(gpu_ctx):
    from plonky3_eon_amd import _lib
    from plonky3_eon_amd import verify as V

    bad = g2_limbs(E.G2_GEN)
    bad[0] ^= 1
    with pytest.raises(_lib.EonError) as e:
        V.pairing(g1_limbs(E.G1_GEN), bad, ctx=gpu_ctx)
    assert e.value.code == _lib.EON_E_ARG
    bad1 = g1_limbs(E.G1_GEN)
    bad1[4] ^= 1
    with pytest.raises(_lib.EonError):
        V.pairing(bad1, g2_limbs(E.G2_GEN), ctx=gpu_ctx)


def _commit(srs, coeffs):
    return O.commit_column(srs, coeffs)


def test_reference_batch_verification(gpu_ctx):
    """kzg/src/tests.rs:73-136: alpha 42, two polynomials opened at 2 and 3."""
    from plonky3_eon_amd import verify as V

    alpha = 42
    srs = O.init_srs_g1(16, alpha)
    g2a = V.g2_mul(alpha, ctx=gpu_ctx)
    np.testing.assert_array_equal(g2a, g2_limbs(E.g2_alpha(alpha)))
    p1, p2 = [1, 2, 3], [5, 7, 11]
    c = [_commit(srs, p1), _commit(srs, p2)]
    z = [2, 3]
    v = [17, 125]
    w = [_commit(srs, [2 + 3 * z[0], 3]), _commit(srs, [7 + 11 * z[1], 11])]

    def run(cs, ws, vs, zs):
        return V.verify_batch(np.stack([g1_limbs(x) for x in cs]), np.stack([g1_limbs(x) for x in ws]),
                              np.stack([fr_limbs(x) for x in vs]), np.stack([fr_limbs(x) for x in zs]), g2a,
                              ctx=gpu_ctx)

    assert run(c, w, v, z) is True
    assert run(c, w, [v[0] + 1, v[1]], z) is False  # wrong value
    assert run(c, [w[1], w[0]], v, z) is False  # swapped witnesses
    assert run(c, w, v, [z[0], 4]) is False  # wrong point
    assert V.verify_batch(np.zeros((0, 8)), np.zeros((0, 8)), np.zeros((0, 4)), np.zeros((0, 4)), g2a, ctx=gpu_ctx)
    # the oracle agrees on each case
    assert E.verify_batch([(c[0], w[0], v[0], z[0]), (c[1], w[1], v[1], z[1])], E.g2_alpha(alpha))


def test_reference_pcs_roundtrip_verify_single(gpu_ctx):
    """kzg/src/tests.rs:20-47: alpha 7, evaluations x + 1 on the 2^3 subgroup, opened at 2."""
    from plonky3_eon_amd import verify as V

    alpha = 7
    srs = O.init_srs_g1(8, alpha)
    g2a = V.g2_mul(alpha, ctx=gpu_ctx)
    coeffs = [1, 1, 0, 0, 0, 0, 0, 0]
    c = _commit(srs, coeffs)
    q = [1, 0, 0, 0, 0, 0, 0]  # (x + 1 - 3) / (x - 2) = 1
    wit = _commit(srs, q)

    def one(val, pt, wt=wit):
        return V.verify_batch(g1_limbs(c)[None], g1_limbs(wt)[None], fr_limbs(val)[None], fr_limbs(pt)[None], g2a,
                              ctx=gpu_ctx)

    assert one(3, 2) is True and E.verify_single(c, wit, 3, 2, E.g2_alpha(alpha))
    assert one(3, 5) is False and not E.verify_single(c, wit, 3, 5, E.g2_alpha(alpha))
    assert one(4, 2) is False
    assert one(3, 2, wt=O.g1_mul(wit, 2)) is False


def test_many_openings_sharing_points(gpu_ctx):
    """The merged-pair path: 40 openings of random polynomials at three points (as a proof's
    zeta / zeta h / quotient openings), one tampered witness makes the batch fail."""
    from plonky3_eon_amd import verify as V

    alpha = 0xC0FFEE
    srs = O.init_srs_g1(9, alpha)
    g2a = V.g2_mul(alpha, ctx=gpu_ctx)
    rng = np.random.default_rng(5)
    pts = [0x1234567, 0x89ABCDEF, O.P - 3]
    cs, ws, vs, zs = [], [], [], []
    for i in range(40):
        coeffs = [int(x) for x in rng.integers(0, 2**62, 8)]
        z = pts[i % 3]
        qq, val = _quotient(coeffs, z)
        cs.append(_commit(srs, coeffs))
        ws.append(_commit(srs, qq))
        vs.append(val)
        zs.append(z)
    args = [np.stack([g1_limbs(x) for x in cs]), np.stack([g1_limbs(x) for x in ws]),
            np.stack([fr_limbs(x) for x in vs]), np.stack([fr_limbs(x) for x in zs])]
    assert V.verify_batch(*args, g2a, ctx=gpu_ctx) is True
    args[1][17] = g1_limbs(O.g1_add(ws[17], E.G1_GEN))
    assert V.verify_batch(*args, g2a, ctx=gpu_ctx) is False


def _quotient(coeffs, z):
    """quotient_and_eval (kzg/src/util.rs:100-111) over ints."""
    n = len(coeffs)
    q = [0] * (n - 1)
    carry = coeffs[-1]
    for i in range(n - 2, -1, -1):
        q[i] = carry
        carry = (coeffs[i] + carry * z) % O.P
    return q, carry
