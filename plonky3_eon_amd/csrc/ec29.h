// BN254 G1 XYZZ accumulation in radix-2^29 arithmetic (field29.h) for the MSM bucket sums.
//
// Same formulas as ec.h (madd-2008-s, mdbl-2008-s-1, a = 0) with lazy reduction: no conditional
// subtraction anywhere, each coordinate carries a bound in multiples of p instead:
//   X < 8p, Y < 4p, ZZ < 2p, ZZZ < 3p        (invariant of an accumulator between additions;
//                                           ZZZ may have lazy limbs < 2^30: it only feeds mul29)
// and every product input stays below 13p (mul29's limit, field29.h).  Affine bases are read in
// 29-Montgomery form (x 2^261 mod p, canonical, as a 256-bit integer in the 64-byte G1Affine
// slot; see k_table_to29 in msm.hip), so a load is a bit re-split with no product.
#pragma once
#include "ec.h"
#include "field29.h"

namespace eon {

struct G1X29 {
    F29 X, Y, ZZ, ZZZ;
};

// The raw accumulator as stored by k_piece_sum: 36 words (X, Y, ZZ, ZZZ limbs), 144 bytes;
// ZZ = 0 marks the identity.
struct alignas(16) G1Raw29 {
    uint32_t w[36];
};


// 2A for an affine A (29-Montgomery, canonical coordinates): mdbl-2008-s-1
__device__ __forceinline__ G1X29 dbl29_affine(const F29& x, const F29& y) {
    const F29 U = add29_norm(y, y);                   // < 2p
    const F29 V = sqr29<FqP>(U);                       // < 2p
    const F29 W = mul29<FqP>(U, V);                   // < 2p
    const F29 S = mul29<FqP>(x, V);                   // < 2p
    const F29 X2 = sqr29<FqP>(x);                      // < 2p
    const F29 M = add29_norm(add29_norm(X2, X2), X2);  // < 6p
    G1X29 r;
    r.X = sub29<FqP, 4>(sqr29<FqP>(M), add29_lazy(S, S));                        // < 6p
    r.Y = sub29<FqP, 2>(mul29<FqP>(M, sub29<FqP, 6>(S, r.X)), mul29<FqP>(W, y));     // < 4p
    r.ZZ = V;
    r.ZZZ = W;
    return r;
}

// acc += (ax, ay) for a non-identity accumulator and a non-identity affine base.  Returns false in
// the exceptional case x(acc) == x(A) (then acc is left unchanged and the caller resolves it:
// doubling or the identity).
//
// CHECK = false (madd29_unchecked) skips that test: in the exceptional case PP = 0 mod p, so ZZ
// becomes 0 mod p and stays 0 under every later unchecked addition (ZZ' = ZZ PP), while a genuine
// sum never has ZZ = 0 (a product of nonzero PPs).  A caller summing a run of bases tests ZZ once
// at the end of the run and re-sums it with the checked form when it is 0.
template <bool CHECK = true>
__device__ __forceinline__ bool madd29(G1X29& acc, const F29& ax, const F29& ay) {
    const F29 U2 = mul29<FqP>(ax, acc.ZZ);            // < 2p
    const F29 P = sub29<FqP, 8>(U2, acc.X);           // < 10p
    const F29 PP = sqr29<FqP>(P);                      // < 2p
    if (CHECK && is_zero_mod29<FqP>(PP)) return false;  // P == 0 mod p
    const F29 PPP = mul29<FqP>(P, PP);                // < 2p
    const F29 Q = mul29<FqP>(acc.X, PP);              // < 2p
    const F29 S2 = mul29<FqP>(ay, acc.ZZZ);           // < 2p
    const F29 R = sub29<FqP, 4>(S2, acc.Y);           // < 6p
    acc.ZZ = mul29<FqP>(acc.ZZ, PP);                  // < 2p
    acc.ZZZ = mul29<FqP>(acc.ZZZ, PPP);               // < 2p
    // X3 = R^2 - (2Q + PPP) + 6p: one normalising subtraction of the lazy sum (limbs < 3 2^29)
    const F29 X3 = sub29<FqP, 6>(sqr29<FqP>(R), add29_lazy(add29_lazy(Q, Q), PPP));  // < 8p
    // Y3 = R (Q - X3) - Y PPP = R (Q - X3 + 9p) + Y (2p - PPP): one shared reduction, < 2p
    // (6p 11p + 4p 2p < p 2^261); Q - X3 + 9p unnormalised (X3 < 8p)
    acc.Y = mul29_sum2<FqP>(R, sub29_lazy<FqP, 9>(Q, X3), acc.Y, sub29<FqP, 2>(F29{}, PPP));
    acc.X = X3;
    return true;
}

__device__ __forceinline__ void madd29_unchecked(G1X29& acc, const F29& ax, const F29& ay) {
    madd29<false>(acc, ax, ay);
}

// madd29_unchecked computed with Pn = X - U2 instead of P = U2 - X, so that PPPn = Pn PP = -PPP
// comes out of the product directly: Y3 = R (Q - X3) - Y PPP = R (Q - X3 + 9p) + Y PPPn needs no
// normalising negation (madd29's 2p - PPP), and X3 = R^2 + PPPn - 2Q + 4p.  The one place PPP's
// sign shows is ZZZ3 = ZZZ PPP: this returns ZZZ PPPn = -ZZZ3, i.e. (X3, Y3, ZZ3, -ZZZ3) -- the
// tuple of the NEGATED sum -(acc + A).  The piece loop (k_piece_sum29) carries that sign as one
// bit per lane: it adds the next base with the opposite sign when the bit is set (the conditional
// base negation it needs anyway for negative digits), and fixes the sign at the run's flush
// (neg_zzz29_lazy).  Same bounds as madd29: X3 < 8p, Y3 < 2p, ZZ3, ZZZ3 < 2p normalised; ay may be
// a lazy negation (limbs < 2^30, value < 2p: it only feeds mul29).
__device__ __forceinline__ void madd29_negsum(G1X29& acc, const F29& ax, const F29& ay) {
    F29 U2 = ax;
    mul29_ip<FqP>(U2, acc.ZZ);                         // < 2p
    F29 Pn = sub29<FqP, 2>(acc.X, U2);                // X - U2 + 2p < 10p
    const F29 PP = sqr29_x<FqP>(Pn);                   // < 2p
    F29 Q = acc.X;
    mul29_ip<FqP>(Q, PP);                              // < 2p
    F29 S2 = ay;
    mul29_ip<FqP>(S2, acc.ZZZ);                        // < 2p
    const F29 R = sub29<FqP, 4>(S2, acc.Y);           // < 6p
    mul29_ip<FqP>(acc.ZZ, PP);                         // < 2p
    mul29_ip<FqP>(Pn, PP);                             // PPPn = -PPP, < 2p
    const F29 PPPn = Pn;
    mul29_ip<FqP>(acc.ZZZ, PPPn);                      // -ZZZ3, < 2p
    // X3 = R^2 + PPPn - 2Q + 4p (2Q < 4p, lazy limbs < 2^30): < 8p
    const F29 X3 = sub29<FqP, 4>(add29_lazy(sqr29_x<FqP>(R), PPPn), add29_lazy(Q, Q));
    // Y3 = R (Q - X3 + 9p) + Y PPPn, one shared reduction (6p 11p + 4p 2p < p 2^261), < 2p
    mul29_sum2_ip<FqP>(R, sub29_lazy<FqP, 9>(Q, X3), acc.Y, PPPn);
    acc.X = X3;
}

// -a as K p - a limb by limb, no carries (a normalised, a < (K - 1) p): limbs < 2^30, value < K p.
// Only for values that feed nothing but mul29 / sqr29 (a base's y, an accumulator's ZZZ).
template <uint32_t K>
__device__ __forceinline__ F29 neg29_lazy(const F29& a) {
    constexpr KPB29<FqP, K> kp{};
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = kp.l[i] - a.l[i];
    return r;
}

// exceptional case of madd29: x(acc) == x(A); returns the sum (doubling when y(acc) == y(A))
// and whether it is the identity.  Rare (duplicate bases, P + (-P)): one extra product.
__device__ __forceinline__ bool madd29_exceptional(G1X29& acc, const F29& ax, const F29& ay) {
    const F29 S2 = mul29<FqP>(ay, acc.ZZZ);
    const F29 R = sub29<FqP, 4>(S2, acc.Y);
    // R mod p: times the plain integer 2^261 mod p (29-Montgomery one) -> value < 2p
    const F29 Rr = mul29<FqP>(R, const29<FqP>(R29<FqP>::ONE));
    if (is_zero_mod29<FqP>(Rr)) {
        acc = dbl29_affine(ax, ay);
        return false;
    }
    return true;  // A = -acc: the sum is the identity
}

// 2P for an accumulator under the invariant bounds: dbl-2008-s-1 (a = 0), lazy
__device__ __forceinline__ void dbl29(G1X29& p) {
    const F29 U = add29_norm(p.Y, p.Y);                // < 8p
    const F29 V = sqr29<FqP>(U);                       // < 2p
    const F29 W = mul29<FqP>(U, V);                    // < 2p
    const F29 S = mul29<FqP>(p.X, V);                  // < 2p
    const F29 X2 = sqr29<FqP>(p.X);                    // < 2p
    const F29 M = add29_norm(add29_norm(X2, X2), X2);  // < 6p
    const F29 X3 = sub29<FqP, 4>(sqr29<FqP>(M), add29_lazy(S, S));  // < 6p
    // Y3 = M (S - X3) - W Y = M (S - X3 + 7p) + W (4p - Y), one shared reduction, < 2p
    // (6p 9p + 2p 4p < p 2^261); S - X3 + 7p unnormalised (X3 < 6p)
    const F29 Y3 = mul29_sum2<FqP>(M, sub29_lazy<FqP, 7>(S, X3), W, sub29<FqP, 4>(F29{}, p.Y));
    p.ZZ = mul29<FqP>(V, p.ZZ);
    p.ZZZ = mul29<FqP>(W, p.ZZZ);
    p.X = X3;
    p.Y = Y3;
}

// p += q for two non-identity accumulators under the invariant bounds: add-2008-s, lazy
// (12M + 2S).  Returns 0, or in the exceptional case x(p) == x(q) (p unchanged) 1 when p == q
// (the caller doubles) and 2 when p == -q (the sum is the identity).
__device__ __forceinline__ int add29(G1X29& p, const G1X29& q) {
    const F29 U1 = mul29<FqP>(p.X, q.ZZ);    // < 2p
    const F29 U2 = mul29<FqP>(q.X, p.ZZ);    // < 2p
    const F29 S1 = mul29<FqP>(p.Y, q.ZZZ);   // < 2p
    const F29 S2 = mul29<FqP>(q.Y, p.ZZZ);   // < 2p
    const F29 P = sub29<FqP, 2>(U2, U1);     // < 4p
    const F29 R = sub29<FqP, 2>(S2, S1);     // < 4p
    const F29 PP = sqr29<FqP>(P);            // < 2p
    if (is_zero_mod29<FqP>(PP)) {
        const F29 Rr = mul29<FqP>(R, const29<FqP>(R29<FqP>::ONE));  // R mod p, < 2p
        return is_zero_mod29<FqP>(Rr) ? 1 : 2;
    }
    const F29 PPP = mul29<FqP>(P, PP);       // < 2p
    const F29 Q = mul29<FqP>(U1, PP);        // < 2p
    const F29 X3 = sub29<FqP, 6>(sqr29<FqP>(R), add29_lazy(add29_lazy(Q, Q), PPP));  // < 8p
    // Y3 = R (Q - X3) - S1 PPP = R (Q - X3 + 9p) + S1 (2p - PPP), < 2p (4p 11p + 2p 2p < p 2^261)
    p.Y = mul29_sum2<FqP>(R, sub29_lazy<FqP, 9>(Q, X3), S1, sub29<FqP, 2>(F29{}, PPP));
    p.ZZ = mul29<FqP>(mul29<FqP>(p.ZZ, q.ZZ), PP);
    p.ZZZ = mul29<FqP>(mul29<FqP>(p.ZZZ, q.ZZZ), PPP);
    p.X = X3;
    return 0;
}

// add29 / dbl29 with their independent products issued together (mul29_n): 5 / 4 dependent
// product steps instead of 14 / 10, for latency-bound callers (a wave alone on its SIMD).  Same
// group element, same bounds on the result (X < 8p, Y < 4p, ZZ, ZZZ < 2p), same return codes.
__device__ __forceinline__ int add29_ilp(G1X29& p, const G1X29& q) {
    F29 t[4];
    mul29_n<FqP, 4>({p.X, q.X, p.Y, q.Y}, {q.ZZ, p.ZZ, q.ZZZ, p.ZZZ}, t);
    const F29 U1 = t[0], S1 = t[2];
    const F29 P = sub29<FqP, 2>(t[1], U1);   // < 4p
    const F29 R = sub29<FqP, 2>(t[3], S1);   // < 4p
    F29 u[4];
    mul29_n<FqP, 4>({P, R, p.ZZ, p.ZZZ}, {P, R, q.ZZ, q.ZZZ}, u);
    const F29 PP = u[0], R2 = u[1];
    if (is_zero_mod29<FqP>(PP)) {
        const F29 Rr = mul29<FqP>(R, const29<FqP>(R29<FqP>::ONE));  // R mod p, < 2p
        return is_zero_mod29<FqP>(Rr) ? 1 : 2;
    }
    F29 v[3];
    mul29_n<FqP, 3>({P, U1, u[2]}, {PP, PP, PP}, v);
    const F29 PPP = v[0], Q = v[1];
    const F29 X3 = sub29<FqP, 6>(R2, add29_lazy(add29_lazy(Q, Q), PPP));  // < 8p
    // Y3 = R (Q - X3 + 9p) + S1 (2p - PPP): two products < 2p each, their sum < 4p
    F29 w[3];
    mul29_n<FqP, 3>({R, S1, u[3]}, {sub29_lazy<FqP, 9>(Q, X3), sub29<FqP, 2>(F29{}, PPP), PPP}, w);
    p.Y = add29_norm(w[0], w[1]);
    p.ZZ = v[2];
    p.ZZZ = w[2];
    p.X = X3;
    return 0;
}

__device__ __forceinline__ void dbl29_ilp(G1X29& p) {
    const F29 U = add29_norm(p.Y, p.Y);                // < 8p
    F29 a[2];
    mul29_n<FqP, 2>({U, p.X}, {U, p.X}, a);
    const F29 V = a[0], X2 = a[1];                     // < 2p
    const F29 M = add29_norm(add29_norm(X2, X2), X2);  // < 6p
    F29 b[4];
    mul29_n<FqP, 4>({U, p.X, M, V}, {V, V, M, p.ZZ}, b);
    const F29 W = b[0], S = b[1];
    const F29 X3 = sub29<FqP, 4>(b[2], add29_lazy(S, S));  // < 6p
    // Y3 = M (S - X3 + 7p) + W (4p - Y): two products < 2p each, their sum < 4p
    F29 c[3];
    mul29_n<FqP, 3>({M, W, W}, {sub29_lazy<FqP, 7>(S, X3), sub29<FqP, 4>(F29{}, p.Y), p.ZZZ}, c);
    p.Y = add29_norm(c[0], c[1]);
    p.ZZ = b[3];
    p.ZZZ = c[2];
    p.X = X3;
}

__device__ __forceinline__ void acc29_ilp(G1X29& p, bool& p_inf, const G1X29& q, bool q_inf) {
    if (q_inf) return;
    if (p_inf) {
        p = q;
        p_inf = false;
        return;
    }
    const int e = add29_ilp(p, q);
    if (e == 1) dbl29_ilp(p);
    if (e == 2) p_inf = true;
}

// p += q with identity flags
__device__ __forceinline__ void acc29(G1X29& p, bool& p_inf, const G1X29& q, bool q_inf) {
    if (q_inf) return;
    if (p_inf) {
        p = q;
        p_inf = false;
        return;
    }
    const int e = add29(p, q);
    if (e == 1) dbl29(p);
    if (e == 2) p_inf = true;
}

// a raw accumulator (k_piece_sum29's partial); returns whether it is the identity
__device__ __forceinline__ bool ld_raw29(const G1Raw29* p, G1X29& a) {
    const uint4* q = reinterpret_cast<const uint4*>(p->w);
    uint32_t w[36];
#pragma unroll
    for (int k = 0; k < 9; k++) {
        const uint4 v = q[k];
        w[4 * k] = v.x;
        w[4 * k + 1] = v.y;
        w[4 * k + 2] = v.z;
        w[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
        a.X.l[i] = w[i];
        a.Y.l[i] = w[9 + i];
        a.ZZ.l[i] = w[18 + i];
        a.ZZZ.l[i] = w[27 + i];
    }
    pin29(a.X);
    pin29(a.Y);
    pin29(a.ZZ);
    pin29(a.ZZZ);
    return is_zero29_raw(a.ZZ);
}

// 29-Montgomery coordinate (any bound < 13p) -> canonical radix-2^32 Montgomery Fq
__device__ __forceinline__ Fq to_fq256(const F29& a) {
    return pack29<FqP>(canon29<FqP>(mul29<FqP>(a, const29<FqP>(R29<FqP>::TO256))));
}

// canonical radix-2^32 Fq -> 29-Montgomery, canonical (x 2^256 -> x 2^261)
__device__ __forceinline__ Fq to_fq261(const Fq& a) {
    return pack29<FqP>(canon29<FqP>(mul29<FqP>(unpack29(a), const29<FqP>(R29<FqP>::TO261))));
}

__device__ __forceinline__ void st_raw29(G1Raw29* p, const G1X29& a) {
    uint32_t w[36];
#pragma unroll
    for (int i = 0; i < 9; i++) {
        w[i] = a.X.l[i];
        w[9 + i] = a.Y.l[i];
        w[18 + i] = a.ZZ.l[i];
        w[27 + i] = a.ZZZ.l[i];
    }
    uint4* q = reinterpret_cast<uint4*>(p->w);
#pragma unroll
    for (int k = 0; k < 9; k++) q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

__device__ __forceinline__ void st_raw29_inf(G1Raw29* p) {
    uint4* q = reinterpret_cast<uint4*>(p->w);
#pragma unroll
    for (int k = 0; k < 9; k++) q[k] = make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ G1Xyzz x29_to_xyzz(const G1X29& a, bool inf) {
    if (inf) return xyzz_inf();
    G1Xyzz r;
    r.X = to_fq256(a.X);
    r.Y = to_fq256(a.Y);
    r.ZZ = to_fq256(a.ZZ);
    r.ZZZ = to_fq256(a.ZZZ);
    return r;
}

__device__ __forceinline__ G1Xyzz raw29_to_xyzz(const G1Raw29* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p->w);
    uint32_t w[36];
#pragma unroll
    for (int k = 0; k < 9; k++) {
        const uint4 v = q[k];
        w[4 * k] = v.x;
        w[4 * k + 1] = v.y;
        w[4 * k + 2] = v.z;
        w[4 * k + 3] = v.w;
    }
    F29 c[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
#pragma unroll
        for (int i = 0; i < 9; i++) c[j].l[i] = w[9 * j + i];
        pin29(c[j]);
    }
    if (is_zero29_raw(c[2])) return xyzz_inf();
    G1Xyzz r;
    r.X = to_fq256(c[0]);
    r.Y = to_fq256(c[1]);
    r.ZZ = to_fq256(c[2]);
    r.ZZZ = to_fq256(c[3]);
    return r;
}

}  // namespace eon
