#!/usr/bin/env python3
"""GLV constants of BN254 G1 for the KZG opening bases (csrc/opening.hip, namespace glv).

phi(x, y) = (beta x, y) is the curve endomorphism with beta a primitive cube root of unity in Fq;
on the prime-order group it acts as multiplication by lambda, a cube root of unity mod r.  Of the
two (beta, lambda) pairs, the one with phi(G) = lambda G for the generator G = (1, 2) is taken.
The scalar decomposition k = k1 + k2 lambda (mod r) uses the short basis (a1, b1), (a2, b2) of the
lattice {(a, b) : a + b lambda = 0 mod r} from the extended Euclidean algorithm on (r, lambda)
(Gallant-Lambert-Vanstone 2001, section 4): c1 = floor(k g1 / 2^256), c2 = floor(k g2 / 2^256)
with g1 = round(b2 2^256 / r), g2 = round(-b1 2^256 / r); k1 = k - c1 a1 - c2 a2,
k2 = -c1 b1 - c2 b2, both below 2^127 in absolute value.

usage: python tools/glv_consts.py   (prints the C++ limb arrays)
"""
from __future__ import annotations

import math

Q = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001


def cube_roots(p: int) -> list[int]:
    for g in range(2, 100):
        w = pow(g, (p - 1) // 3, p)
        if w != 1:
            return [w, w * w % p]
    raise ValueError("no cube root of unity")


def g1_mul(pt, k: int):
    """Affine double-and-add on y^2 = x^3 + 3 over Fq (None = identity)."""
    def add(a, b):
        if a is None:
            return b
        if b is None:
            return a
        if a[0] == b[0]:
            if (a[1] + b[1]) % Q == 0:
                return None
            lam = 3 * a[0] * a[0] * pow(2 * a[1], -1, Q) % Q
        else:
            lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, Q) % Q
        x = (lam * lam - a[0] - b[0]) % Q
        return (x, (lam * (a[0] - x) - a[1]) % Q)

    acc = None
    for bit in bin(k)[2:]:
        acc = add(acc, acc)
        if bit == "1":
            acc = add(acc, pt)
    return acc


def endomorphism():
    """(beta, lambda) with phi(G) = lambda G."""
    g = (1, 2)
    for lam in cube_roots(R):
        p = g1_mul(g, lam)
        for beta in cube_roots(Q):
            if p == (beta % Q, 2):
                return beta, lam
    raise ValueError("no matching pair")


def lattice_basis(lam: int):
    """Short vectors (a1, b1), (a2, b2) with a + b lambda = 0 mod r (GLV section 4)."""
    s0, t0, r0, s1, t1, r1 = 1, 0, R, 0, 1, lam
    rows = [(r0, s0, t0), (r1, s1, t1)]
    while r1:
        q = r0 // r1
        r0, r1 = r1, r0 - q * r1
        s0, s1 = s1, s0 - q * s1
        t0, t1 = t1, t0 - q * t1
        rows.append((r1, s1, t1))
    root = math.isqrt(R)
    idx = max(i for i, (ri, _, _) in enumerate(rows) if ri >= root)
    (rl, _, tl), (rl1, _, tl1), (rl2, _, tl2) = rows[idx], rows[idx + 1], rows[idx + 2]
    v1 = (rl1, -tl1)
    v2 = min([(rl, -tl), (rl2, -tl2)], key=lambda v: v[0] ** 2 + v[1] ** 2)
    return v1, v2


def constants() -> dict:
    beta, lam = endomorphism()
    (a1, b1), (a2, b2) = lattice_basis(lam)
    g1 = ((b2 << 256) + R // 2) // R
    g2 = ((-b1 << 256) + R // 2) // R
    return {"beta": beta, "lambda": lam, "a1": a1, "b1": b1, "a2": a2, "b2": b2, "g1": g1, "g2": g2}


def decompose(k: int, c: dict) -> tuple[int, int]:
    """The device's decomposition (opening.hip glv_split) in integers."""
    c1 = (k * c["g1"]) >> 256
    c2 = (k * c["g2"]) >> 256
    return k - c1 * c["a1"] - c2 * c["a2"], -c1 * c["b1"] - c2 * c["b2"]


def limbs32(x: int, n: int) -> list[int]:
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def limbs29(x: int) -> list[int]:
    return [(x >> (29 * i)) & ((1 << 29) - 1) for i in range(9)]


def device_arrays(c: dict) -> dict:
    """The arrays csrc/opening.hip's namespace glv holds."""
    return {"G1": limbs32(c["g1"], 3), "G2": limbs32(c["g2"], 5), "A1": limbs32(c["a1"], 2),
            "A2": limbs32(c["a2"], 4), "NB1": limbs32(-c["b1"], 4),
            "BETA29": limbs29((c["beta"] << 261) % Q)}


if __name__ == "__main__":
    c = constants()
    for k, v in device_arrays(c).items():
        print(f"constexpr uint32_t {k}[{len(v)}] = {{" + ", ".join(f"0x{x:x}u" for x in v) + "};")
