// BN254 extension-field tower and optimal-ate pairing pieces for the KZG verifier (pairing.hip).
//
// Replaces halo2curves' Bn256::multi_miller_loop + final_exponentiation behind the reference's
// pairing / multi_pairing (bn254/src/curve.rs:429-452), used by verify_single / verify_batch
// (kzg/src/util.rs:150-168, 245-292).  The tower is the standard one (halo2curves' layout):
//   Fq2  = Fq[u] / (u^2 + 1)
//   Fq6  = Fq2[v] / (v^3 - xi),  xi = 9 + u
//   Fq12 = Fq6[w] / (w^2 - v)    (so w^6 = xi, and c_i.c_j is the coefficient of w^(2j + i))
// G2 lives on the sextic twist y^2 = x^3 + 3/xi over Fq2, untwisted by (x, y) -> (x w^2, y w^3).
// Elements are Montgomery residues in 8 x 32-bit limbs (field.h), every value canonical.
//
// Verification is not on the prove path: one thread per pair, plain formulas -- a projective
// Miller loop whose lines differ from the affine ones by factors in Fq2 (removed by the easy part),
// and the exact final exponent (q^12 - 1) / r = (q^6 - 1)(q^2 + 1) * (q^4 - q^2 + 1) / r, the hard
// part from its base-q decomposition in x with cyclotomic squarings -- so that the value of every
// pairing equals the definition's, bit for bit (tests/test_gpu_pairing.py).
#pragma once
#include "ec.h"
#include "pairing_consts.h"

// the tower products are real calls (a force-inlined Miller loop / final exponentiation is
// minutes of compile time and no faster: verification is latency-, not throughput-bound)
#define EON_NI __host__ __device__ __attribute__((noinline))

namespace eon {

EON_HD Fq fq_c(const uint32_t (&c)[8]) {
    Fq r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = c[i];
    return r;
}

// ---- Fq2 ----------------------------------------------------------------------------------------

struct Fq2 {
    Fq c0, c1;
};

EON_HD Fq2 f2_zero() { return {Fq::zero(), Fq::zero()}; }
EON_HD Fq2 f2_one() { return {Fq::one(), Fq::zero()}; }
EON_HD Fq2 f2_c(const uint32_t (&c)[2][8]) { return {fq_c(c[0]), fq_c(c[1])}; }
EON_HD bool f2_is_zero(const Fq2& a) { return a.c0.is_zero() && a.c1.is_zero(); }
EON_HD bool f2_eq(const Fq2& a, const Fq2& b) { return a.c0 == b.c0 && a.c1 == b.c1; }
EON_HD Fq2 f2_add(const Fq2& a, const Fq2& b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
EON_HD Fq2 f2_sub(const Fq2& a, const Fq2& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
EON_HD Fq2 f2_neg(const Fq2& a) { return {neg(a.c0), neg(a.c1)}; }
EON_HD Fq2 f2_dbl(const Fq2& a) { return {dbl(a.c0), dbl(a.c1)}; }
EON_HD Fq2 f2_conj(const Fq2& a) { return {a.c0, neg(a.c1)}; }
EON_HD Fq2 f2_mul_fq(const Fq2& a, const Fq& b) { return {mul(a.c0, b), mul(a.c1, b)}; }

// (a0 + a1 u)(b0 + b1 u), u^2 = -1 (Karatsuba: 3 products).  f2_mul_inl is the inlined body for
// the latency-bound team kernels (pairing_team.h): a call passes its Fq2 operands through scratch
// (the calling convention takes at most 16 registers of aggregate arguments).
EON_HD Fq2 f2_mul_inl(const Fq2& a, const Fq2& b) {
    const Fq t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1);
    const Fq t2 = mul(add(a.c0, a.c1), add(b.c0, b.c1));
    return {sub(t0, t1), sub(sub(t2, t0), t1)};
}

EON_NI Fq2 f2_mul(const Fq2& a, const Fq2& b) { return f2_mul_inl(a, b); }

EON_NI Fq2 f2_sqr(const Fq2& a) {
    const Fq t = mul(a.c0, a.c1);
    return {mul(add(a.c0, a.c1), sub(a.c0, a.c1)), dbl(t)};
}

// a * xi = (9 a0 - a1) + (a0 + 9 a1) u
EON_HD Fq2 f2_mul_xi(const Fq2& a) {
    const Fq a0x8 = dbl(dbl(dbl(a.c0))), a1x8 = dbl(dbl(dbl(a.c1)));
    return {sub(add(a0x8, a.c0), a.c1), add(add(a1x8, a.c1), a.c0)};
}

EON_NI Fq2 f2_inv(const Fq2& a) {
    const Fq inv_norm = inverse(add(sqr(a.c0), sqr(a.c1)));
    return {mul(a.c0, inv_norm), neg(mul(a.c1, inv_norm))};
}

// ---- Fq6 ----------------------------------------------------------------------------------------

struct Fq6 {
    Fq2 c0, c1, c2;
};

EON_HD Fq6 f6_zero() { return {f2_zero(), f2_zero(), f2_zero()}; }
EON_HD Fq6 f6_add(const Fq6& a, const Fq6& b) { return {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; }
EON_HD Fq6 f6_sub(const Fq6& a, const Fq6& b) { return {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; }
EON_HD Fq6 f6_neg(const Fq6& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
// a * v = (xi a2, a0, a1)
EON_HD Fq6 f6_mul_v(const Fq6& a) { return {f2_mul_xi(a.c2), a.c0, a.c1}; }

EON_NI Fq6 f6_mul(const Fq6& a, const Fq6& b) {
    const Fq2 t0 = f2_mul(a.c0, b.c0), t1 = f2_mul(a.c1, b.c1), t2 = f2_mul(a.c2, b.c2);
    const Fq2 s12 = f2_sub(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), t1), t2);
    const Fq2 s01 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), t0), t1);
    const Fq2 s02 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), t0), t2);
    return {f2_add(f2_mul_xi(s12), t0), f2_add(s01, f2_mul_xi(t2)), f2_add(s02, t1)};
}

EON_NI Fq6 f6_inv(const Fq6& a) {
    const Fq2 A = f2_sub(f2_sqr(a.c0), f2_mul_xi(f2_mul(a.c1, a.c2)));
    const Fq2 B = f2_sub(f2_mul_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
    const Fq2 C = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
    const Fq2 F = f2_add(f2_mul(a.c0, A), f2_mul_xi(f2_add(f2_mul(a.c2, B), f2_mul(a.c1, C))));
    const Fq2 fi = f2_inv(F);
    return {f2_mul(A, fi), f2_mul(B, fi), f2_mul(C, fi)};
}

// ---- Fq12 ---------------------------------------------------------------------------------------

struct Fq12 {
    Fq6 c0, c1;
};

EON_HD Fq12 f12_one() { return {{f2_one(), f2_zero(), f2_zero()}, f6_zero()}; }

EON_HD bool f12_is_one(const Fq12& a) {
    const Fq12 o = f12_one();
    const Fq2* x = &a.c0.c0;
    const Fq2* y = &o.c0.c0;
    bool eq = true;
    for (int i = 0; i < 6; i++) eq = eq && f2_eq(x[i], y[i]);
    return eq;
}

EON_NI Fq12 f12_mul(const Fq12& a, const Fq12& b) {
    const Fq6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
    const Fq6 s = f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1));
    return {f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(s, t0), t1)};
}

// (a0 + a1 w)^2 = (a0 + a1)(a0 + v a1) - t - v t + 2 t w, t = a0 a1
EON_NI Fq12 f12_sqr(const Fq12& a) {
    const Fq6 t = f6_mul(a.c0, a.c1);
    const Fq6 s = f6_mul(f6_add(a.c0, a.c1), f6_add(a.c0, f6_mul_v(a.c1)));
    return {f6_sub(f6_sub(s, t), f6_mul_v(t)), f6_add(t, t)};
}

// Granger-Scott squaring, valid on the cyclotomic subgroup (a^(q^6 + 1) = 1: the values after the
// easy part of the final exponentiation).  Fq12 viewed as Fq4^3 with Fq4 = Fq2[y]/(y^2 - xi):
// (z0 + z1 y), (z2 + z3 y), (z4 + z5 y) with z0 = c0.c0, z1 = c1.c1, z2 = c1.c0, z3 = c0.c2,
// z4 = c0.c1, z5 = c1.c2; three Fq4 squarings (6 Fq2 products) instead of f12_sqr's 12.
// (x + y Y)^2 = (x^2 + xi y^2) + 2 x y Y in Fq4 = Fq2[Y]/(Y^2 - xi), as (x + y)(x + xi y) - t - xi t
// with t = x y
EON_HD void fq4_sqr(const Fq2& x, const Fq2& y, Fq2& s0, Fq2& s1) {
    const Fq2 t = f2_mul(x, y);
    s0 = f2_sub(f2_sub(f2_mul(f2_add(x, y), f2_add(x, f2_mul_xi(y))), t), f2_mul_xi(t));
    s1 = f2_dbl(t);
}

EON_NI Fq12 f12_cyc_sqr(const Fq12& a) {
    const Fq2 &z0 = a.c0.c0, &z4 = a.c0.c1, &z3 = a.c0.c2, &z2 = a.c1.c0, &z1 = a.c1.c1, &z5 = a.c1.c2;
    Fq2 t0, t1, t2, t3, t4, t5;
    fq4_sqr(z0, z1, t0, t1);
    fq4_sqr(z2, z3, t2, t3);
    fq4_sqr(z4, z5, t4, t5);
    Fq12 r;
    r.c0.c0 = f2_add(f2_dbl(f2_sub(t0, z0)), t0);  // 3 t0 - 2 z0
    r.c1.c1 = f2_add(f2_dbl(f2_add(t1, z1)), t1);  // 3 t1 + 2 z1
    const Fq2 x5 = f2_mul_xi(t5);
    r.c1.c0 = f2_add(f2_dbl(f2_add(x5, z2)), x5);  // 3 xi t5 + 2 z2
    r.c0.c2 = f2_add(f2_dbl(f2_sub(t4, z3)), t4);  // 3 t4 - 2 z3
    r.c0.c1 = f2_add(f2_dbl(f2_sub(t2, z4)), t2);  // 3 t2 - 2 z4
    r.c1.c2 = f2_add(f2_dbl(f2_add(t3, z5)), t3);  // 3 t3 + 2 z5
    return r;
}

// a (b0 + b1 v) (the sparse Fq6 factor of a line): 5 Fq2 products
EON_NI Fq6 f6_mul_01(const Fq6& a, const Fq2& b0, const Fq2& b1) {
    const Fq2 t0 = f2_mul(a.c0, b0), t1 = f2_mul(a.c1, b1);
    return {f2_add(f2_mul_xi(f2_mul(a.c2, b1)), t0), f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b0, b1)), t0), t1),
            f2_add(f2_sub(f2_mul(f2_add(a.c0, a.c2), b0), t0), t1)};
}

// f * l for a line l = l0 + l1 w + l3 w^3 (l.c0 = (l0, 0, 0), l.c1 = (l1, l3, 0)): 13 Fq2 products
EON_NI Fq12 f12_mul_line(const Fq12& f, const Fq2& l0, const Fq2& l1, const Fq2& l3) {
    const Fq6 t0 = {f2_mul(f.c0.c0, l0), f2_mul(f.c0.c1, l0), f2_mul(f.c0.c2, l0)};
    const Fq6 t1 = f6_mul_01(f.c1, l1, l3);
    const Fq6 s = f6_mul_01(f6_add(f.c0, f.c1), f2_add(l0, l1), l3);
    return {f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(s, t0), t1)};
}

// a^(q^6): w -> -w
EON_HD Fq12 f12_conj(const Fq12& a) { return {a.c0, f6_neg(a.c1)}; }

EON_NI Fq12 f12_inv(const Fq12& a) {
    // 1 / (a0 + a1 w) = (a0 - a1 w) / (a0^2 - v a1^2)
    const Fq6 d = f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1)));
    const Fq6 di = f6_inv(d);
    return {f6_mul(a.c0, di), f6_neg(f6_mul(a.c1, di))};
}

// a^(q^j), j = 1, 2, 3: the coefficient of w^k becomes frob_j(a_k) xi^(k (q^j - 1) / 6)
template <int J>
EON_NI Fq12 f12_frob(const Fq12& a) {
    const Fq2* x = &a.c0.c0;  // c0.c0 c0.c1 c0.c2 c1.c0 c1.c1 c1.c2
    Fq12 r;
    Fq2* y = &r.c0.c0;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int k = 2 * j + i;
            const Fq2 c = (J & 1) ? f2_conj(x[3 * i + j]) : x[3 * i + j];
            const Fq2 g = J == 1 ? f2_c(pc::FROB1[k]) : J == 2 ? f2_c(pc::FROB2[k]) : f2_c(pc::FROB3[k]);
            y[3 * i + j] = f2_mul(c, g);
        }
    return r;
}

// ---- G2 on the twist ----------------------------------------------------------------------------

struct G2Affine {
    Fq2 x, y;  // (0, 0) = identity (not on the curve)
};

EON_HD bool g2_is_inf(const G2Affine& p) { return f2_is_zero(p.x) && f2_is_zero(p.y); }

EON_HD G2Affine g2_generator() {
    // the standard BN254 G2 generator (halo2curves' G2::generator, EIP-197), Montgomery form
    G2Affine g;
    g.x = {fq_c(pc::G2_GEN_X[0]), fq_c(pc::G2_GEN_X[1])};
    g.y = {fq_c(pc::G2_GEN_Y[0]), fq_c(pc::G2_GEN_Y[1])};
    return g;
}

EON_HD bool g2_on_curve(const G2Affine& p) {
    if (g2_is_inf(p)) return true;
    const Fq2 lhs = f2_sqr(p.y);
    const Fq2 rhs = f2_add(f2_mul(f2_sqr(p.x), p.x), f2_c(pc::TWIST_B));
    return f2_eq(lhs, rhs);
}

struct G2Jac {
    Fq2 X, Y, Z;  // (X / Z^2, Y / Z^3); Z = 0 is the identity
};

EON_HD G2Jac g2j_from_affine(const G2Affine& a) {
    if (g2_is_inf(a)) return {f2_one(), f2_one(), f2_zero()};
    return {a.x, a.y, f2_one()};
}

// 2P, dbl-2009-l (a = 0)
EON_NI G2Jac g2j_dbl(const G2Jac& p) {
    if (f2_is_zero(p.Z)) return p;
    const Fq2 A = f2_sqr(p.X), B = f2_sqr(p.Y), C = f2_sqr(B);
    const Fq2 D = f2_dbl(f2_sub(f2_sub(f2_sqr(f2_add(p.X, B)), A), C));
    const Fq2 E = f2_add(f2_dbl(A), A), F = f2_sqr(E);
    G2Jac r;
    r.X = f2_sub(F, f2_dbl(D));
    r.Y = f2_sub(f2_mul(E, f2_sub(D, r.X)), f2_dbl(f2_dbl(f2_dbl(C))));
    r.Z = f2_dbl(f2_mul(p.Y, p.Z));
    return r;
}

// P + A (A affine), madd-2007-bl with the doubling / inverse cases
EON_NI G2Jac g2j_add_affine(const G2Jac& p, const G2Affine& a) {
    if (g2_is_inf(a)) return p;
    if (f2_is_zero(p.Z)) return g2j_from_affine(a);
    const Fq2 Z1Z1 = f2_sqr(p.Z);
    const Fq2 U2 = f2_mul(a.x, Z1Z1), S2 = f2_mul(f2_mul(a.y, p.Z), Z1Z1);
    const Fq2 H = f2_sub(U2, p.X), rr = f2_dbl(f2_sub(S2, p.Y));
    if (f2_is_zero(H)) {
        if (f2_is_zero(rr)) return g2j_dbl(g2j_from_affine(a));
        return {f2_one(), f2_one(), f2_zero()};
    }
    const Fq2 HH = f2_sqr(H), I = f2_dbl(f2_dbl(HH)), J = f2_mul(H, I), V = f2_mul(p.X, I);
    G2Jac r;
    r.X = f2_sub(f2_sub(f2_sqr(rr), J), f2_dbl(V));
    r.Y = f2_sub(f2_mul(rr, f2_sub(V, r.X)), f2_dbl(f2_mul(p.Y, J)));
    r.Z = f2_sub(f2_sub(f2_sqr(f2_add(p.Z, H)), Z1Z1), HH);
    return r;
}

// P + Q (both Jacobian), add-2007-bl with the doubling / inverse / identity cases
EON_NI G2Jac g2j_add(const G2Jac& p, const G2Jac& q) {
    if (f2_is_zero(p.Z)) return q;
    if (f2_is_zero(q.Z)) return p;
    const Fq2 Z1Z1 = f2_sqr(p.Z), Z2Z2 = f2_sqr(q.Z);
    const Fq2 U1 = f2_mul(p.X, Z2Z2), U2 = f2_mul(q.X, Z1Z1);
    const Fq2 S1 = f2_mul(f2_mul(p.Y, q.Z), Z2Z2), S2 = f2_mul(f2_mul(q.Y, p.Z), Z1Z1);
    const Fq2 H = f2_sub(U2, U1), rr = f2_dbl(f2_sub(S2, S1));
    if (f2_is_zero(H)) {
        if (f2_is_zero(rr)) return g2j_dbl(p);
        return {f2_one(), f2_one(), f2_zero()};
    }
    const Fq2 I = f2_sqr(f2_dbl(H)), J = f2_mul(H, I), V = f2_mul(U1, I);
    G2Jac r;
    r.X = f2_sub(f2_sub(f2_sqr(rr), J), f2_dbl(V));
    r.Y = f2_sub(f2_mul(rr, f2_sub(V, r.X)), f2_dbl(f2_mul(S1, J)));
    r.Z = f2_mul(f2_sub(f2_sub(f2_sqr(f2_add(p.Z, q.Z)), Z1Z1), Z2Z2), H);
    return r;
}

EON_NI G2Affine g2j_to_affine(const G2Jac& p) {
    if (f2_is_zero(p.Z)) return {f2_zero(), f2_zero()};
    const Fq2 zi = f2_inv(p.Z), zi2 = f2_sqr(zi);
    return {f2_mul(p.X, zi2), f2_mul(p.Y, f2_mul(zi2, zi))};
}

// k P for a canonical 256-bit integer k (8 LE 32-bit words), double-and-add MSB first
EON_NI G2Jac g2_mul_words(const G2Affine& p, const uint32_t (&k)[8]) {
    G2Jac acc = {f2_one(), f2_one(), f2_zero()};
    for (int w = 7; w >= 0; w--)
        for (int b = 31; b >= 0; b--) {
            acc = g2j_dbl(acc);
            if ((k[w] >> b) & 1) acc = g2j_add_affine(acc, p);
        }
    return acc;
}

}  // namespace eon
