"""BN254 optimal-ate pairing restatement (TEST INFRASTRUCTURE ONLY).

The reference verifies KZG openings with halo2curves' `Bn256::multi_miller_loop` +
`final_exponentiation` (bn254/src/curve.rs:429-452) in verify_single / verify_batch
(kzg/src/util.rs:150-168, 245-292): e(C - [v]G1, G2) == e(W, [s]G2 - [z]G2).  halo2curves is not in
the container, so the pairing is restated here from its published definition:

* Fq12 = Fq[w] / (w^12 - 18 w^6 + 82) (the tower Fq2 = Fq[u]/(u^2 + 1), Fq6 = Fq2[v]/(v^3 - (9 + u)),
  Fq12 = Fq6[w]/(w^2 - v) flattened, u = w^6 - 9);
* G2 on the sextic twist y^2 = x^3 + 3 / (9 + u) over Fq2, mapped into E(Fq12) by
  (x, y) -> (x w^2, y w^3);
* Miller loop over 6x + 2 (x = 4965661367192848881) with affine line functions, then the two
  Frobenius-twisted additions of the optimal ate pairing, and the final exponentiation
  f^((q^12 - 1) / r).

Pure Python big integers: ~1 s per pairing, for small test instances only.  Pinned by the group
laws (bilinearity, non-degeneracy, r-torsion of the generators) in tests/test_pairing_oracle.py,
and by the reference's own KZG tests (kzg/src/tests.rs:20-47, 73-136) restated there.
"""

from __future__ import annotations

from . import pyoracle as O

Q = O.Q  # base field modulus
R = O.P  # group order (Fr modulus)
ATE_LOOP_COUNT = 29793968203157093288  # 6x + 2, x = 4965661367192848881
X_BN = 4965661367192848881

# ---- Fq2 = Fq[u] / (u^2 + 1) as (a0, a1) ----------------------------------------------------------


def f2(a0, a1=0):
    return (a0 % Q, a1 % Q)


def f2_add(a, b):
    return ((a[0] + b[0]) % Q, (a[1] + b[1]) % Q)


def f2_sub(a, b):
    return ((a[0] - b[0]) % Q, (a[1] - b[1]) % Q)


def f2_neg(a):
    return ((-a[0]) % Q, (-a[1]) % Q)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % Q, (a[0] * b[1] + a[1] * b[0]) % Q)


def f2_inv(a):
    d = pow(a[0] * a[0] + a[1] * a[1], Q - 2, Q)
    return (a[0] * d % Q, (-a[1]) * d % Q)


F2_ZERO = (0, 0)
F2_ONE = (1, 0)
XI = (9, 1)  # 9 + u
B2 = f2_mul((3, 0), f2_inv(XI))  # the twist's b = 3 / (9 + u)

# The standard BN254 G2 generator (the one halo2curves' G2::generator returns; EIP-197)
G2_GEN = (
    (10857046999023057135944570762232829481370756359578518086990519993285655852781,
     11559732032986387107991004021392285783925812861821192530917403151452391805634),
    (8495653923123431417604973247489272438418190587263600148770280649306958101930,
     4082367875863433681332203403145435568316851327593401208105741076214120093531),
)
G1_GEN = (1, 2)

# ---- G2 (affine over Fq2, None = infinity) -----------------------------------------------------------


def g2_on_curve(p) -> bool:
    if p is None:
        return True
    x, y = p
    return f2_sub(f2_mul(y, y), f2_add(f2_mul(f2_mul(x, x), x), B2)) == F2_ZERO


def g2_add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    (x1, y1), (x2, y2) = p, q
    if x1 == x2:
        if y1 == y2:
            return g2_double(p)
        return None
    lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_mul(lam, lam), x1), x2)
    return (x3, f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1))


def g2_double(p):
    if p is None:
        return None
    x, y = p
    if y == F2_ZERO:
        return None
    lam = f2_mul(f2_mul((3, 0), f2_mul(x, x)), f2_inv(f2_add(y, y)))
    x3 = f2_sub(f2_mul(lam, lam), f2_add(x, x))
    return (x3, f2_sub(f2_mul(lam, f2_sub(x, x3)), y))


def g2_neg(p):
    return None if p is None else (p[0], f2_neg(p[1]))


def g2_mul(p, k: int):
    k %= R
    acc = None
    for bit in bin(k)[2:] if k else "":
        acc = g2_double(acc)
        if bit == "1":
            acc = g2_add(acc, p)
    return acc


# ---- G1 (affine canonical ints, None = infinity), via pyoracle ---------------------------------------


def g1_add(p, q):
    return O.g1_add(p, q)


def g1_mul(p, k: int):
    return O.g1_mul(p, k % R)


def g1_neg(p):
    return O.g1_neg(p)


# ---- Fq12 = Fq[w] / (w^12 - 18 w^6 + 82) as 12-tuples -----------------------------------------------
# (w^6 = 9 + u, so u = w^6 - 9 and u^2 = -1 give the modulus)

_MOD = {6: 18, 0: -82}  # w^12 = 18 w^6 - 82


def f12_mul(a, b):
    t = [0] * 23
    for i, ai in enumerate(a):
        if ai:
            for j, bj in enumerate(b):
                if bj:
                    t[i + j] += ai * bj
    for k in range(22, 11, -1):
        c = t[k]
        if c:
            t[k - 6] += 18 * c
            t[k - 12] -= 82 * c
    return tuple(x % Q for x in t[:12])


def f12_one():
    return (1,) + (0,) * 11


def f12_sub(a, b):
    return tuple((x - y) % Q for x, y in zip(a, b))


def f12_pow(a, e: int):
    r = f12_one()
    for bit in bin(e)[2:]:
        r = f12_mul(r, r)
        if bit == "1":
            r = f12_mul(r, a)
    return r


def _poly_deg(p):
    d = len(p) - 1
    while d >= 0 and p[d] % Q == 0:
        d -= 1
    return d


def f12_inv(a):
    """Inverse by the extended Euclidean algorithm over Fq[w] modulo w^12 - 18 w^6 + 82."""
    lm, hm = [1] + [0] * 12, [0] * 13
    low, high = list(a) + [0], [82, 0, 0, 0, 0, 0, (-18) % Q, 0, 0, 0, 0, 0, 1]
    while _poly_deg(low):
        # r = high // low (polynomial division)
        dl, dh = _poly_deg(low), _poly_deg(high)
        r = [0] * 13
        rem = list(high)
        inv_lead = pow(low[dl], Q - 2, Q)
        for i in range(dh - dl, -1, -1):
            c = rem[dl + i] * inv_lead % Q
            r[i] = c
            for j in range(dl + 1):
                rem[i + j] = (rem[i + j] - c * low[j]) % Q
        nm = list(hm)
        new = list(high)
        for i in range(13):
            for j in range(13 - i):
                nm[i + j] = (nm[i + j] - lm[i] * r[j]) % Q
                new[i + j] = (new[i + j] - low[i] * r[j]) % Q
        lm, low, hm, high = nm, new, lm, low
    inv0 = pow(low[0], Q - 2, Q)
    return tuple(x * inv0 % Q for x in lm[:12])


def f12_from_f2(a):
    """a0 + a1 u with u = w^6 - 9."""
    t = [0] * 12
    t[0] = (a[0] - 9 * a[1]) % Q
    t[6] = a[1] % Q
    return tuple(t)


def f12_scalar(c):
    return (c % Q,) + (0,) * 11


def _w_pow(k):
    t = [0] * 12
    t[k] = 1
    return tuple(t)


W2, W3 = _w_pow(2), _w_pow(3)


def twist(p):
    """G2 point on the twist -> E(Fq12): (x w^2, y w^3)."""
    if p is None:
        return None
    return (f12_mul(f12_from_f2(p[0]), W2), f12_mul(f12_from_f2(p[1]), W3))


def cast_g1(p):
    return None if p is None else (f12_scalar(p[0]), f12_scalar(p[1]))


# ---- E(Fq12) arithmetic for the Miller loop ----------------------------------------------------------


def e12_double(p):
    x, y = p
    lam = f12_mul(f12_mul(f12_scalar(3), f12_mul(x, x)), f12_inv(f12_mul(f12_scalar(2), y)))
    x3 = f12_sub(f12_mul(lam, lam), f12_mul(f12_scalar(2), x))
    return (x3, f12_sub(f12_mul(lam, f12_sub(x, x3)), y))


def e12_add(p, q):
    (x1, y1), (x2, y2) = p, q
    if x1 == x2:
        return e12_double(p) if y1 == y2 else None
    lam = f12_mul(f12_sub(y2, y1), f12_inv(f12_sub(x2, x1)))
    x3 = f12_sub(f12_sub(f12_mul(lam, lam), x1), x2)
    return (x3, f12_sub(f12_mul(lam, f12_sub(x1, x3)), y1))


def _line(p1, p2, t):
    """The line through p1 and p2 (tangent if equal) evaluated at t."""
    (x1, y1), (x2, y2), (xt, yt) = p1, p2, t
    if x1 != x2:
        m = f12_mul(f12_sub(y2, y1), f12_inv(f12_sub(x2, x1)))
        return f12_sub(f12_mul(m, f12_sub(xt, x1)), f12_sub(yt, y1))
    if y1 == y2:
        m = f12_mul(f12_mul(f12_scalar(3), f12_mul(x1, x1)), f12_inv(f12_mul(f12_scalar(2), y1)))
        return f12_sub(f12_mul(m, f12_sub(xt, x1)), f12_sub(yt, y1))
    return f12_sub(xt, x1)


def _frob(p):
    """The q-power Frobenius on coordinates."""
    return (f12_pow(p[0], Q), f12_pow(p[1], Q))


def miller_loop(q_fq12, p_fq12):
    """f_{6x+2, Q}(P) times the two optimal-ate correction lines; no final exponentiation."""
    if q_fq12 is None or p_fq12 is None:
        return f12_one()
    rr = q_fq12
    f = f12_one()
    for bit in bin(ATE_LOOP_COUNT)[3:]:
        f = f12_mul(f12_mul(f, f), _line(rr, rr, p_fq12))
        rr = e12_double(rr)
        if bit == "1":
            f = f12_mul(f, _line(rr, q_fq12, p_fq12))
            rr = e12_add(rr, q_fq12)
    q1 = _frob(q_fq12)
    nq2 = _frob(q1)
    nq2 = (nq2[0], f12_sub(f12_scalar(0), nq2[1]))
    f = f12_mul(f, _line(rr, q1, p_fq12))
    rr = e12_add(rr, q1)
    f = f12_mul(f, _line(rr, nq2, p_fq12))
    return f


FINAL_EXP = (Q ** 12 - 1) // R


def final_exponentiation(f):
    return f12_pow(f, FINAL_EXP)


def pairing(p_g1, q_g2):
    """e(P, Q) for P in G1 (canonical-int affine, None = O) and Q in G2 (Fq2 affine)."""
    return final_exponentiation(miller_loop(twist(q_g2), cast_g1(p_g1)))


def multi_pairing(pairs):
    """prod_i e(P_i, Q_i) with one final exponentiation (multi_pairing, bn254/src/curve.rs:439-452)."""
    f = f12_one()
    for p, q in pairs:
        f = f12_mul(f, miller_loop(twist(q), cast_g1(p)))
    return final_exponentiation(f)


# ---- KZG verification as the reference states it (kzg/src/util.rs) -------------------------------


def g2_alpha(alpha: int):
    """KzgParams.g2_alpha = [alpha] G2 (init_srs_unsafe, kzg/src/params.rs:123-139)."""
    return g2_mul(G2_GEN, alpha)


def verify_single(commitment, witness, value: int, point: int, g2a) -> bool:
    """kzg/src/util.rs:150-168: e(C - [v]G1, G2) == e(W, [alpha]G2 - [z]G2)."""
    left = pairing(g1_add(commitment, g1_neg(g1_mul(G1_GEN, value))), G2_GEN)
    right = pairing(witness, g2_add(g2a, g2_neg(g2_mul(G2_GEN, point))))
    return left == right


def verify_batch(openings, g2a) -> bool:
    """kzg/src/util.rs:245-292: prod_i e(C_i - v_i G1, G2) e(-W_i, [alpha]G2 - z_i G2) == 1.
    openings: [(commitment, witness, value, point)] with points as canonical-int affine G1."""
    if not openings:
        return True
    if len(openings) == 1:
        return verify_single(*openings[0], g2a)
    pairs = []
    for c, w, v, z in openings:
        pairs.append((g1_add(c, g1_neg(g1_mul(G1_GEN, v))), G2_GEN))
        pairs.append((g1_neg(w), g2_add(g2a, g2_neg(g2_mul(G2_GEN, z)))))
    return multi_pairing(pairs) == f12_one()
