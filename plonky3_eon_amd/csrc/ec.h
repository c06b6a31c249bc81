// BN254 G1 (y^2 = x^3 + 3 over Fq) point arithmetic for the MSM kernels.
//
// Accumulators are XYZZ coordinates (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2), the cheapest form for
// mixed additions with affine bases: madd 8M+2S, add 12M+2S, dbl 6M+3S (EFD "xyzz" formulas
// madd-2008-s / add-2008-s / dbl-2008-s-1 for a = 0).  The point at infinity is ZZ = ZZZ = 0;
// the affine ABI encodes it as (0, 0), which is not on the curve.
//
// The reference delegates this arithmetic to halo2curves 0.9 (bn254/src/curve.rs:59-66,177); all
// representations denote the same group element, so results are compared in affine form.
#pragma once
#include "field.h"

namespace eon {

struct G1Affine {
    Fq x, y;
};

struct G1Xyzz {
    Fq X, Y, ZZ, ZZZ;
};

EON_HD bool is_inf(const G1Xyzz& p) { return p.ZZ.is_zero(); }
EON_HD bool is_inf(const G1Affine& p) { return p.x.is_zero() && p.y.is_zero(); }

EON_HD G1Xyzz xyzz_inf() {
    G1Xyzz r;
    r.X = Fq::one();
    r.Y = Fq::one();
    r.ZZ = Fq::zero();
    r.ZZZ = Fq::zero();
    return r;
}

EON_HD G1Xyzz xyzz_from_affine(const G1Affine& a) {
    if (is_inf(a)) return xyzz_inf();
    G1Xyzz r;
    r.X = a.x;
    r.Y = a.y;
    r.ZZ = Fq::one();
    r.ZZZ = Fq::one();
    return r;
}

EON_HD G1Affine affine_neg(const G1Affine& a) {
    G1Affine r = a;
    if (!is_inf(a)) r.y = neg(a.y);
    return r;
}

// 2P, dbl-2008-s-1 (a = 0)
EON_HD G1Xyzz xyzz_dbl(const G1Xyzz& p) {
    if (is_inf(p)) return p;
    const Fq U = dbl(p.Y);
    const Fq V = sqr(U);
    const Fq W = mul(U, V);
    const Fq S = mul(p.X, V);
    const Fq X2 = sqr(p.X);
    const Fq M = add(dbl(X2), X2);
    G1Xyzz r;
    r.X = sub(sqr(M), dbl(S));
    r.Y = sub(mul(M, sub(S, r.X)), mul(W, p.Y));
    r.ZZ = mul(V, p.ZZ);
    r.ZZZ = mul(W, p.ZZZ);
    return r;
}

// 2A for affine A, mdbl-2008-s-1
EON_HD G1Xyzz xyzz_dbl_affine(const G1Affine& a) {
    const Fq U = dbl(a.y);
    const Fq V = sqr(U);
    const Fq W = mul(U, V);
    const Fq S = mul(a.x, V);
    const Fq X2 = sqr(a.x);
    const Fq M = add(dbl(X2), X2);
    G1Xyzz r;
    r.X = sub(sqr(M), dbl(S));
    r.Y = sub(mul(M, sub(S, r.X)), mul(W, a.y));
    r.ZZ = V;
    r.ZZZ = W;
    return r;
}

// P + A (A affine, possibly the (0,0) identity), madd-2008-s with the doubling/inverse cases
EON_HD G1Xyzz xyzz_add_affine(const G1Xyzz& p, const G1Affine& a) {
    if (is_inf(a)) return p;
    if (is_inf(p)) return xyzz_from_affine(a);
    const Fq U2 = mul(a.x, p.ZZ);
    const Fq S2 = mul(a.y, p.ZZZ);
    const Fq P = sub(U2, p.X);
    const Fq R = sub(S2, p.Y);
    if (P.is_zero()) {
        if (R.is_zero()) return xyzz_dbl_affine(a);
        return xyzz_inf();
    }
    const Fq PP = sqr(P);
    const Fq PPP = mul(P, PP);
    const Fq Q = mul(p.X, PP);
    G1Xyzz r;
    r.X = sub(sub(sqr(R), PPP), dbl(Q));
    r.Y = sub(mul(R, sub(Q, r.X)), mul(p.Y, PPP));
    r.ZZ = mul(p.ZZ, PP);
    r.ZZZ = mul(p.ZZZ, PPP);
    return r;
}

// P + Q, add-2008-s with the doubling/inverse cases
EON_HD G1Xyzz xyzz_add(const G1Xyzz& p, const G1Xyzz& q) {
    if (is_inf(q)) return p;
    if (is_inf(p)) return q;
    const Fq U1 = mul(p.X, q.ZZ);
    const Fq U2 = mul(q.X, p.ZZ);
    const Fq S1 = mul(p.Y, q.ZZZ);
    const Fq S2 = mul(q.Y, p.ZZZ);
    const Fq P = sub(U2, U1);
    const Fq R = sub(S2, S1);
    if (P.is_zero()) {
        if (R.is_zero()) return xyzz_dbl(p);
        return xyzz_inf();
    }
    const Fq PP = sqr(P);
    const Fq PPP = mul(P, PP);
    const Fq Q = mul(U1, PP);
    G1Xyzz r;
    r.X = sub(sub(sqr(R), PPP), dbl(Q));
    r.Y = sub(mul(R, sub(Q, r.X)), mul(S1, PPP));
    r.ZZ = mul(mul(p.ZZ, q.ZZ), PP);
    r.ZZZ = mul(mul(p.ZZZ, q.ZZZ), PPP);
    return r;
}

// k * P for a small non-negative integer k (double-and-add, MSB first)
EON_HD G1Xyzz xyzz_mul_small(const G1Xyzz& p, uint32_t k) {
    G1Xyzz r = xyzz_inf();
    if (k == 0 || is_inf(p)) return r;
    const int top = 31 - __builtin_clz(k);
    r = p;
    for (int b = top - 1; b >= 0; b--) {
        r = xyzz_dbl(r);
        if ((k >> b) & 1) r = xyzz_add(r, p);
    }
    return r;
}

// XYZZ -> affine with a given 1/ZZZ (batch-inversion friendly): 1/z = ZZ/ZZZ, 1/ZZ = (1/z)^2
EON_HD G1Affine xyzz_to_affine_with_inv(const G1Xyzz& p, const Fq& inv_zzz) {
    G1Affine r;
    if (is_inf(p)) {
        r.x = Fq::zero();
        r.y = Fq::zero();
        return r;
    }
    const Fq inv_z = mul(p.ZZ, inv_zzz);
    r.x = mul(p.X, sqr(inv_z));
    r.y = mul(p.Y, inv_zzz);
    return r;
}

EON_HD G1Affine xyzz_to_affine(const G1Xyzz& p) {
    if (is_inf(p)) return xyzz_to_affine_with_inv(p, Fq::zero());
    return xyzz_to_affine_with_inv(p, inverse(p.ZZZ));
}

// Pinned point loads / vector stores (see ld_pinned in field.h)
__device__ __forceinline__ void pin(G1Xyzz& a) {
    pin(a.X);
    pin(a.Y);
    pin(a.ZZ);
    pin(a.ZZZ);
}

__device__ __forceinline__ G1Xyzz ld_xyzz(const G1Xyzz* p) {
    G1Xyzz r;
    r.X = ld_pinned(&p->X);
    r.Y = ld_pinned(&p->Y);
    r.ZZ = ld_pinned(&p->ZZ);
    r.ZZZ = ld_pinned(&p->ZZZ);
    return r;
}

__device__ __forceinline__ void st_xyzz(G1Xyzz* p, const G1Xyzz& a) {
    st_vec(&p->X, a.X);
    st_vec(&p->Y, a.Y);
    st_vec(&p->ZZ, a.ZZ);
    st_vec(&p->ZZZ, a.ZZZ);
}

// all four 16-byte loads issued before any pin: pinning x first (two ld_pinned calls) made the
// y loads wait for x's, two memory round trips per point instead of one
__device__ __forceinline__ G1Affine ld_affine(const G1Affine* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    G1Affine r;
    r.x.v[0] = a.x; r.x.v[1] = a.y; r.x.v[2] = a.z; r.x.v[3] = a.w;
    r.x.v[4] = b.x; r.x.v[5] = b.y; r.x.v[6] = b.z; r.x.v[7] = b.w;
    r.y.v[0] = c.x; r.y.v[1] = c.y; r.y.v[2] = c.z; r.y.v[3] = c.w;
    r.y.v[4] = d.x; r.y.v[5] = d.y; r.y.v[6] = d.z; r.y.v[7] = d.w;
    pin(r.x);
    pin(r.y);
    return r;
}

__device__ __forceinline__ void st_affine(G1Affine* p, const G1Affine& a) {
    st_vec(&p->x, a.x);
    st_vec(&p->y, a.y);
}

}  // namespace eon

