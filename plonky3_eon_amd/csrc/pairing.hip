// KZG verifier pairings on the GPU: G2 scalar multiplication (the SRS's
// g2_alpha, kzg/src/params.rs:123-139), multi_pairing (bn254/src/curve.rs:439-452) and
// verify_batch / verify_single (kzg/src/util.rs:150-168, 245-292).  Arithmetic: pairing.h.
//
// verify_batch checks prod_i e(C_i - v_i G1, G2) e(-W_i, [alpha]G2 - z_i G2) == 1.  Pairs with
// the same G2 argument are merged by bilinearity before any Miller loop -- every commitment pair
// shares G2 itself, and the witness pairs share [alpha - z]G2 per distinct opening point z (the
// headline proof's 2626 openings have three: zeta, zeta h, and zeta for the quotient chunks) --
// so the product is the same element of Gt computed from 1 + (#distinct z) pairings:
//   e(sum_i C_i - (sum_i v_i) G1, G2) * prod_z e(-sum_{i: z_i = z} W_i, [alpha]G2 - z G2).
// verify_single's e(C - vG1, G2) == e(W, [alpha]G2 - zG2) is the same product being 1.
//
//   k_vb_sums     one block per distinct point: -sum W_i over its openings; one more block for
//                 sum C_i and sum v_i (XYZZ partial sums per thread, LDS tree)
//   k_vb_pairs    the merged pairs: P_0 = sum C - (sum v) G1 with Q_0 = G2, P_z = -sum W with
//                 Q_z = [alpha]G2 - z G2 (fixed-generator multiples as sums of 2^i tables, 64
//                 lanes and an LDS tree per pair, then affine)
//   k_miller_team one 6-lane team per pair (pairing_team.h: lane k holds the coefficient of w^k):
//                 f_{6x+2,Q}(P) by the signed digits of 6x + 2 and the two Frobenius-twisted lines,
//                 T in projective coordinates (no inversions; lines scaled by Fq2 factors), the
//                 line and point formulas spread over the lanes
//   k_final_exp_team  one team: product of the Miller values, easy part f^((q^6-1)(q^2+1)), hard
//                 part f^((q^4-q^2+1)/r) from f^x, f^(x^2), f^(x^3) and Frobenius maps, and the
//                 test against 1
#include <algorithm>
#include <map>
#include <vector>

#include "context.h"
#include "pairing_team.h"

using namespace eon;

namespace {

// ---- Miller loop --------------------------------------------------------------------------------
//
// T runs in homogeneous projective coordinates on the twist (x = X / Z, y = Y / Z), so no step
// inverts.  Each line is the affine line through T and A, untwisted and evaluated at P,
//   l = -yp + (lambda xp) w + (y_T - lambda x_T) w^3,
// times a factor in Fq2 (2 Y Z for a tangent, X - x_A Z for a chord): Fq2 lies in Fq6, whose
// nonzero elements the easy part of the final exponentiation sends to 1, so the pairing -- the Gt
// value after the final exponentiation -- is the affine loop's exactly (Costello-Lange-Naehrig;
// Aranha et al. 2011, the D-type twist forms).

struct G2Proj {
    Fq2 X, Y, Z;
};

// tangent at T: T <- 2T, returns 2YZ times the affine tangent line
// (the published X3 = XY/2 (B - F), Y3 = ((B + F)/2)^2 - 3E^2, Z3 = B H, all scaled by 4: no halving)
__device__ __noinline__ Fq12 dbl_line(G2Proj& T, const Fq& xp, const Fq& yp) {
    const Fq2 A = f2_dbl(f2_mul(T.X, T.Y));              // 2 X Y
    const Fq2 B = f2_sqr(T.Y), C = f2_sqr(T.Z);
    const Fq2 E = f2_mul(f2_add(f2_dbl(C), C), f2_c(pc::TWIST_B));  // 3 b' Z^2
    const Fq2 F = f2_add(f2_dbl(E), E);
    const Fq2 G = f2_add(B, F);
    const Fq2 H = f2_sub(f2_sqr(f2_add(T.Y, T.Z)), f2_add(B, C));   // 2 Y Z
    const Fq2 J = f2_sqr(T.X);
    const Fq2 E2 = f2_sqr(E);
    Fq12 l = {f6_zero(), f6_zero()};
    l.c0.c0 = f2_mul_fq(f2_neg(H), yp);                  // -2YZ yp
    l.c1.c0 = f2_mul_fq(f2_add(f2_dbl(J), J), xp);        // 3 X^2 xp (= 2YZ lambda xp)
    l.c1.c1 = f2_sub(E, B);                               // 2YZ (y - lambda x) = 3 b' Z^2 - Y^2
    const Fq2 E2x3 = f2_add(f2_dbl(E2), E2);
    T.X = f2_mul(A, f2_sub(B, F));
    T.Y = f2_sub(f2_sqr(G), f2_dbl(f2_dbl(E2x3)));
    T.Z = f2_dbl(f2_dbl(f2_mul(B, H)));
    return l;
}

// chord through T and the affine A: T <- T + A, returns (X - x_A Z) times the affine line
// (vertical when x_T = x_A: Z (xp - x_T w^2), and T becomes the identity)
__device__ __noinline__ Fq12 add_line(G2Proj& T, const G2Affine& A, const Fq& xp, const Fq& yp) {
    const Fq2 theta = f2_sub(T.Y, f2_mul(A.y, T.Z));    // Y - y_A Z
    const Fq2 lam = f2_sub(T.X, f2_mul(A.x, T.Z));      // X - x_A Z
    Fq12 l = {f6_zero(), f6_zero()};
    if (f2_is_zero(lam)) {
        if (f2_is_zero(theta)) return dbl_line(T, xp, yp);  // T = A
        l.c0.c0 = f2_mul_fq(T.Z, xp);
        l.c0.c1 = f2_neg(T.X);
        T = {f2_one(), f2_one(), f2_zero()};
        return l;
    }
    const Fq2 C = f2_sqr(theta), D = f2_sqr(lam);
    const Fq2 E = f2_mul(lam, D), F = f2_mul(T.Z, C), G = f2_mul(T.X, D);
    const Fq2 H = f2_sub(f2_add(E, F), f2_dbl(G));
    l.c0.c0 = f2_mul_fq(f2_neg(lam), yp);                        // -lambda' yp
    l.c1.c0 = f2_mul_fq(theta, xp);                              // theta xp (= lambda' slope xp)
    l.c1.c1 = f2_sub(f2_mul(lam, A.y), f2_mul(theta, A.x));      // lambda' y_A - theta x_A
    T.X = f2_mul(lam, H);
    T.Y = f2_sub(f2_mul(theta, f2_sub(G, H)), f2_mul(E, T.Y));
    T.Z = f2_mul(T.Z, E);
    return l;
}

// ---- team-parallel Miller loop and final exponentiation (pairing_team.h) -----------------------
//
// Lane k of a team holds the coefficient of w^k of the running Fq12; lanes 6 and 7 of the 8-lane
// team compute as copies of lane 5 and publish nothing.  Every barrier sits in control flow that is
// uniform over the block (the loop bits are constants; per-team data decides only selects), and
// the blocks are one wave, so a barrier costs a few cycles next to an Fq2 product's hundreds.

constexpr uint32_t TEAM = 8;

struct TeamLane {
    int k;     // coefficient index this lane computes (0..5)
    bool pub;  // lanes 0..5 publish
};

__device__ __forceinline__ TeamLane team_lane() {
    const uint32_t l = threadIdx.x & (TEAM - 1);
    return {l < 6 ? (int)l : 5, l < 6};
}

// per team: the published Fq12 operands (v, xi v) and the doubling's exchanged products
struct MillerLds {
    Fq2 f[TEAM], fx[TEAM], d[TEAM], s[TEAM], sx[TEAM], e[TEAM];
};

// f times an add_line line (sparse l0 + l1 w + l3 w^3, or the vertical l0 + l2 w^2)
__device__ __forceinline__ Fq2 team_mul_add_line(MillerLds& L, const TeamLane& tl, const Fq2& f, const Fq12& l) {
    const bool vert = f2_is_zero(l.c1.c0) && f2_is_zero(l.c1.c1);
    if (tl.pub) {
        L.f[tl.k] = f;
        L.fx[tl.k] = f2_mul_xi(f);
    }
    __syncthreads();
    const int j[3] = {0, vert ? 2 : 1, 3};
    const Fq2 v[3] = {l.c0.c0, vert ? l.c0.c1 : l.c1.c0, vert ? f2_zero() : l.c1.c1};
    const Fq2 r = tm_sparse(L.f, L.fx, j, v, tl.k);
    __syncthreads();
    return r;
}

// chord step T <- T + A with f <- f l, add_line's formulas spread over the lanes in four exchanges:
//   1  publish f, and lane 0 y_A Z, 1 x_A Z;
//   2  theta = Y - y_A Z, lambda = X - x_A Z; lane 0 theta^2, 1 lambda^2, 2 -lambda yp,
//      3 theta xp, 4 lambda y_A, 5 theta x_A;
//   3  f l (3 products); lane 0 E = lambda D, 1 F = Z C, 2 G = X D;
//   4  H = E + F - 2G; lane 0 lambda H, 1 theta (G - H), 2 E Y, 3 Z E; then T.
// Returns whether lambda = 0 (T = +-A: add_line's doubling or vertical case, which this step
// does not compute; the caller redoes the step with add_line).
__device__ __forceinline__ bool team_add_step(MillerLds& L, const TeamLane& tl, Fq2& f, G2Proj& T, const G2Affine& A,
                                              const Fq& xp, const Fq& yp) {
    const int k = tl.k;
    {
        const Fq2 d = f2_mul_inl(k == 0 ? A.y : A.x, T.Z);
        if (tl.pub) {
            L.f[k] = f;
            L.fx[k] = f2_mul_xi(f);
            L.d[k] = d;
        }
    }
    __syncthreads();
    const Fq2 theta = f2_sub(T.Y, L.d[0]), lam = f2_sub(T.X, L.d[1]);
    {
        const Fq2 yp2 = {yp, Fq::zero()}, xp2 = {xp, Fq::zero()};
        const Fq2 u = k == 0 ? theta : k == 1 ? lam : k == 2 ? f2_neg(lam) : k == 3 ? theta : k == 4 ? lam : theta;
        const Fq2 v = k == 0 ? theta : k == 1 ? lam : k == 2 ? yp2 : k == 3 ? xp2 : k == 4 ? A.y : A.x;
        const Fq2 e = f2_mul_inl(u, v);
        if (tl.pub) L.e[k] = e;
    }
    __syncthreads();
    {
        const int j[3] = {0, 1, 3};
        const Fq2 l[3] = {L.e[2], L.e[3], f2_sub(L.e[4], L.e[5])};
        f = tm_sparse(L.f, L.fx, j, l, k);
        const Fq2 C = L.e[0], D = L.e[1];
        const Fq2 g = f2_mul_inl(k == 0 ? lam : k == 1 ? T.Z : T.X, k == 1 ? C : D);
        if (tl.pub) L.s[k] = g;
    }
    __syncthreads();
    {
        const Fq2 E = L.s[0], F = L.s[1], G = L.s[2];
        const Fq2 H = f2_sub(f2_add(E, F), f2_dbl(G));
        const Fq2 u = k == 0 ? lam : k == 1 ? theta : k == 2 ? E : T.Z;
        const Fq2 v = k == 0 ? H : k == 1 ? f2_sub(G, H) : k == 2 ? T.Y : E;
        const Fq2 e = f2_mul_inl(u, v);
        if (tl.pub) L.e[k] = e;
    }
    __syncthreads();
    T = {L.e[0], f2_sub(L.e[1], L.e[2]), L.e[3]};
    return f2_is_zero(lam);
}

// team_add_step, and add_line on every lane for the teams where it met T = +-A (a barrier-uniform
// branch: every team of the block takes it when any team needs it, and keeps its result only then)
__device__ __forceinline__ void team_add(MillerLds& L, const TeamLane& tl, Fq2& f, G2Proj& T, const G2Affine& A,
                                         const Fq& xp, const Fq& yp) {
    const Fq2 f0 = f;
    G2Proj T0 = T;
    const bool special = team_add_step(L, tl, f, T, A, xp, yp);
    if (__syncthreads_or(special)) {
        // copies made here, so that no operand of the hot path has its address taken by the call
        G2Affine a_c = A;
        Fq xp_c = xp, yp_c = yp;
        const Fq2 fs = team_mul_add_line(L, tl, f0, add_line(T0, a_c, xp_c, yp_c));
        if (special) {
            f = fs;
            T = T0;
        }
    }
}

// One pair per team, 8 teams per block; 6x + 2 by its non-adjacent form (65 doublings, 21 chord
// steps, -Q = (x, -y)).  A doubling step is two exchanges:
//   A  publish f and the tangent's first-level products (lane 0 XY, 1 Y^2, 2 Z^2, 3 X^2,
//      4 (Y + Z)^2);
//   B  f^2's coefficient (6 products), E = 3 b' Z^2, and the second level (lane 0 E^2, 1 G^2,
//      2 A (B - F), 3 B H, 4 -H yp, 5 3 J xp) -- dbl_line's formulas, spread over the lanes;
//   C  T from the second level, f^2 times the line (3 products).
// Lines and T are dbl_line's / add_line's exactly; the value after the final exponentiation is the
// definition's (the signed chain changes f only by vertical lines, which lie in Fq6).
__global__ void __launch_bounds__(64) k_miller_team(const G1Affine* __restrict__ P, const G2Affine* __restrict__ Q,
                                                    uint32_t m, Fq12* __restrict__ out) {
    __shared__ MillerLds lds[64 / TEAM];
    const TeamLane tl = team_lane();
    const int k = tl.k;
    const uint32_t pi = blockIdx.x * (64 / TEAM) + threadIdx.x / TEAM;
    MillerLds& L = lds[threadIdx.x / TEAM];
    const G1Affine p = P[min(pi, m - 1)];
    const G2Affine q = Q[min(pi, m - 1)];
    const Fq &xp = p.x, &yp = p.y;
    Fq2 f = k == 0 ? f2_one() : f2_zero();
    G2Proj T = {q.x, q.y, f2_one()};
    // b = 64 .. 0: the doubling and the digit's chord; b = -1, -2: the chords through pi(Q) and
    // -pi^2(Q).  One inlined copy of each step (calls would pass T and f through scratch).
    for (int b = 64; b >= -2; b--) {
        if (b >= 0) {
            {
                const Fq2 yz = f2_add(T.Y, T.Z);
                const Fq2 u = k == 0 ? T.X : k == 1 ? T.Y : k == 2 ? T.Z : k == 3 ? T.X : yz;
                const Fq2 v = k == 0 ? T.Y : k == 1 ? T.Y : k == 2 ? T.Z : k == 3 ? T.X : yz;
                const Fq2 d = f2_mul_inl(u, v);
                if (tl.pub) {
                    L.f[k] = f;
                    L.fx[k] = f2_mul_xi(f);
                    L.d[k] = d;
                }
            }
            __syncthreads();
            const Fq2 B = L.d[1], C = L.d[2];
            const Fq2 E = f2_mul_inl(f2_add(f2_dbl(C), C), f2_c(pc::TWIST_B));
            {
                const Fq2 fs = tm_mul(L.f, L.f, L.fx, k);
                const Fq2 A = f2_dbl(L.d[0]), J = L.d[3];
                const Fq2 H = f2_sub(L.d[4], f2_add(B, C));
                const Fq2 F = f2_add(f2_dbl(E), E), G = f2_add(B, F);
                const Fq2 yp2 = {yp, Fq::zero()}, xp2 = {xp, Fq::zero()};
                const Fq2 u = k == 0 ? E : k == 1 ? G : k == 2 ? A : k == 3 ? B : k == 4 ? f2_neg(H) : f2_add(f2_dbl(J), J);
                const Fq2 v = k == 0 ? E : k == 1 ? G : k == 2 ? f2_sub(B, F) : k == 3 ? H : k == 4 ? yp2 : xp2;
                const Fq2 e = f2_mul_inl(u, v);
                if (tl.pub) {
                    L.s[k] = fs;
                    L.sx[k] = f2_mul_xi(fs);
                    L.e[k] = e;
                }
            }
            __syncthreads();
            {
                const Fq2 E2 = L.e[0];
                T.X = L.e[2];
                T.Y = f2_sub(L.e[1], f2_dbl(f2_dbl(f2_add(f2_dbl(E2), E2))));
                T.Z = f2_dbl(f2_dbl(L.e[3]));
                const int j[3] = {0, 1, 3};
                const Fq2 v[3] = {L.e[4], L.e[5], f2_sub(E, B)};
                f = tm_sparse(L.s, L.sx, j, v, k);
            }
        }
        const bool pos = b >= 0 && b < 64 && ((pc::ATE_NAF_POS >> b) & 1);
        const bool neg = b >= 0 && b < 64 && ((pc::ATE_NAF_NEG >> b) & 1);
        if (pos || neg || b < 0) {
            // the chord's point, formed here (uniform branches) rather than kept live across the
            // loop: -Q = (x, -y), pi(Q) = (conj(x) g_x, conj(y) g_y), -pi^2(Q) = (x g2_x, y)
            G2Affine A = q;
            if (neg) {
                A.y = f2_neg(q.y);
            } else if (b == -1) {
                A = {f2_mul_inl(f2_conj(q.x), f2_c(pc::TWIST_FROB_X)), f2_mul_inl(f2_conj(q.y), f2_c(pc::TWIST_FROB_Y))};
            } else if (b == -2) {
                A.x = f2_mul_fq(q.x, fq_c(pc::TWIST_FROB2_X));
            }
            team_add(L, tl, f, T, A, xp, yp);
        }
    }
    if (is_inf(p) || g2_is_inf(q)) f = k == 0 ? f2_one() : f2_zero();
    if (pi < m && tl.pub) set_w_coef(out[pi], k, f);
}

struct ExpLds {
    Fq2 a[TEAM], b[TEAM], bx[TEAM];
    uint32_t flag[TEAM];
};

// the final exponentiation's exchange slots (one team per launch).  Namespace scope, so that the
// called helpers below address it as LDS directly; their operands go by value (registers), not by
// reference (scratch)
__shared__ ExpLds g_exp;

// The exchanges inline (publish, barrier, compute, barrier); the products of the compute half are
// one called function per kind reading the slots, so the ~20 products of the chain share a copy of
// the code and no operand passes through a call (an Fq2 pair exceeds the 16 registers the calling
// convention gives aggregate arguments, and the rest would go through scratch).
__device__ __noinline__ Fq2 team_mul_compute() { return tm_mul(g_exp.a, g_exp.b, g_exp.bx, team_lane().k); }
__device__ __noinline__ Fq2 team_cyc_sqr_compute() { return tm_cyc_sqr(g_exp.a, team_lane().k); }

// coefficient k of a b
__device__ __forceinline__ Fq2 team_mul(const Fq2& a, const Fq2& b) {
    const TeamLane tl = team_lane();
    if (tl.pub) {
        g_exp.a[tl.k] = a;
        g_exp.b[tl.k] = b;
        g_exp.bx[tl.k] = f2_mul_xi(b);
    }
    __syncthreads();
    const Fq2 r = team_mul_compute();
    __syncthreads();
    return r;
}

// coefficient k of a^2 for a unitary a
__device__ __forceinline__ Fq2 team_cyc_sqr(const Fq2& a) {
    const TeamLane tl = team_lane();
    if (tl.pub) g_exp.a[tl.k] = a;
    __syncthreads();
    const Fq2 r = team_cyc_sqr_compute();
    __syncthreads();
    return r;
}

// coefficient k of a^x (x = pc::BN_X by its non-adjacent form, a^-1 = conj(a))
__device__ __noinline__ Fq2 team_pow_x(Fq2 a) {
    const Fq2 ai = tm_conj(a, team_lane().k);
    Fq2 r = a;
    for (int b = 61; b >= 0; b--) {
        r = team_cyc_sqr(r);
        if ((pc::BN_X_NAF_POS >> b) & 1) r = team_mul(r, a);
        if ((pc::BN_X_NAF_NEG >> b) & 1) r = team_mul(r, ai);
    }
    return r;
}

// One team: the product of the m Miller values, the final exponentiation (easy part
// f^((q^6 - 1)(q^2 + 1)); hard part t^((q^4 - q^2 + 1) / r) = t^(l0 + l1 q + l2 q^2 + l3 q^3)
// exactly, the l_i polynomials in x (Scott et al. 2009; identity asserted in
// tools/pairing_consts.py): y0 = t^(q + q^2 + q^3), y1 = t^-1, y2 = t^(x^2 q^2), y3 = t^(-x q),
// y4 = t^(-x - x^2 q), y5 = t^(-x^2), y6 = t^(-x^3 - x^3 q), and y0 y1^2 y2^6 y3^12 y4^18 y5^30
// y6^36 by the addition chain), and the test against 1.  The one inversion gathers the element
// on every lane.
__global__ void __launch_bounds__(TEAM) k_final_exp_team(const Fq12* __restrict__ f, uint32_t m,
                                                         Fq12* __restrict__ out, uint32_t* __restrict__ is_one) {
    ExpLds& L = g_exp;
    const TeamLane tl = team_lane();
    const int k = tl.k;
    Fq2 acc = m ? w_coef(f[0], k) : (k == 0 ? f2_one() : f2_zero());
    for (uint32_t i = 1; i < m; i++) acc = team_mul(acc, w_coef(f[i], k));
    // easy part; t is unitary from here on (its inverse is its conjugate)
    if (tl.pub) L.a[k] = acc;
    __syncthreads();
    Fq12 whole;
    for (int j = 0; j < 6; j++) set_w_coef(whole, j, L.a[j]);
    __syncthreads();
    const Fq12 inv = f12_inv(whole);
    Fq2 t = team_mul(tm_conj(acc, k), w_coef(inv, k));
    t = team_mul(tm_frob<2>(t, k), t);
    // hard part
    const Fq2 fx = team_pow_x(t);
    const Fq2 fx2 = team_pow_x(fx);
    const Fq2 fx3 = team_pow_x(fx2);
    const Fq2 y0 = team_mul(team_mul(tm_frob<1>(t, k), tm_frob<2>(t, k)), tm_frob<3>(t, k));
    const Fq2 y1 = tm_conj(t, k);
    const Fq2 y2 = tm_frob<2>(fx2, k);
    const Fq2 y3 = tm_conj(tm_frob<1>(fx, k), k);
    const Fq2 y4 = tm_conj(team_mul(fx, tm_frob<1>(fx2, k)), k);
    const Fq2 y5 = tm_conj(fx2, k);
    const Fq2 y6 = tm_conj(team_mul(fx3, tm_frob<1>(fx3, k)), k);
    Fq2 t0 = team_mul(team_mul(team_cyc_sqr(y6), y4), y5);
    Fq2 t1 = team_mul(team_mul(y3, y5), t0);
    t0 = team_mul(t0, y2);
    t1 = team_cyc_sqr(team_mul(team_cyc_sqr(t1), t0));
    t0 = team_cyc_sqr(team_mul(t1, y1));
    t1 = team_mul(t1, y0);
    const Fq2 r = team_mul(t0, t1);
    if (tl.pub) {
        set_w_coef(*out, k, r);
        L.flag[k] = f2_eq(r, k == 0 ? f2_one() : f2_zero()) ? 1u : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t all = 1;
        for (int j = 0; j < 6; j++) all &= L.flag[j];
        *is_one = all;
    }
}

// ---- verify_batch: merged pairs -----------------------------------------------------------------

constexpr uint32_t VB_THREADS = 128;

// block g < G: -sum of the witnesses of openings ord[gs[g] .. gs[g+1]); block G: sum of every
// commitment and sum of every value
__global__ void __launch_bounds__(VB_THREADS) k_vb_sums(const G1Affine* __restrict__ com, const G1Affine* __restrict__ wit,
                                                        const Fr* __restrict__ val, const uint32_t* __restrict__ ord,
                                                        const uint32_t* __restrict__ gs, uint32_t G, uint32_t n,
                                                        G1Xyzz* __restrict__ sums, Fr* __restrict__ vsum) {
    __shared__ G1Xyzz part[VB_THREADS];
    __shared__ Fr vpart[VB_THREADS];
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    G1Xyzz acc = xyzz_inf();
    Fr vacc = Fr::zero();
    if (g < G) {
        for (uint32_t i = gs[g] + t; i < gs[g + 1]; i += VB_THREADS) acc = xyzz_add_affine(acc, wit[ord[i]]);
    } else {
        for (uint32_t i = t; i < n; i += VB_THREADS) {
            acc = xyzz_add_affine(acc, com[i]);
            vacc = add(vacc, val[i]);
        }
    }
    part[t] = acc;
    vpart[t] = vacc;
    __syncthreads();
    for (uint32_t s = VB_THREADS / 2; s > 0; s >>= 1) {
        if (t < s) {
            part[t] = xyzz_add(part[t], part[t + s]);
            vpart[t] = add(vpart[t], vpart[t + s]);
        }
        __syncthreads();
    }
    if (t == 0) {
        G1Xyzz r = part[0];
        if (g < G && !is_inf(r)) r.Y = neg(r.Y);  // -sum W
        sums[g] = r;
        if (g == G) *vsum = vpart[0];
    }
}


// One block of VBP_THREADS per merged pair.  [k] of a fixed generator is the sum of the table
// entries 2^i G of k's set bits: thread i sums the entries of bits [4i, 4i + 4), then an LDS tree
// adds the 64 partial sums -- 4 + 6 dependent additions instead of one thread's ~128.
constexpr uint32_t VBP_THREADS = 64;

__global__ void __launch_bounds__(VBP_THREADS) k_vb_pairs(const G1Xyzz* __restrict__ sums, const Fr* __restrict__ vsum,
                                                          const Fr* __restrict__ zs, uint32_t G, G2Affine g2_alpha,
                                                          G1Affine* __restrict__ P, G2Affine* __restrict__ Q) {
    __shared__ G1Xyzz p1[VBP_THREADS];
    __shared__ G2Jac p2[VBP_THREADS];
    const uint32_t t = blockIdx.x, i = threadIdx.x;
    if (t > G) return;
    const Fr k = to_canonical(t == 0 ? *vsum : zs[t - 1]);
    const uint32_t word = k.v[i >> 3], b0 = 4 * i, sh = b0 & 31;
    if (t == 0) {
        // P_0 = sum C - (sum v) G1, Q_0 = G2
        G1Xyzz acc = xyzz_inf();
        for (uint32_t b = 0; b < 4; b++)
            if ((word >> (sh + b)) & 1)
                acc = xyzz_add_affine(acc, {fq_c(pc::G1_POW2[b0 + b][0]), fq_c(pc::G1_POW2[b0 + b][1])});
        p1[i] = acc;
        __syncthreads();
        for (uint32_t s = VBP_THREADS / 2; s > 0; s >>= 1) {
            if (i < s) p1[i] = xyzz_add(p1[i], p1[i + s]);
            __syncthreads();
        }
        if (i == 0) {
            const G1Affine vg = xyzz_to_affine(p1[0]);
            P[0] = xyzz_to_affine(xyzz_add_affine(sums[G], affine_neg(vg)));
            Q[0] = g2_generator();
        }
    } else {
        // P_z = -sum W, Q_z = [alpha]G2 - z G2
        G2Jac acc = {f2_one(), f2_one(), f2_zero()};
        for (uint32_t b = 0; b < 4; b++)
            if ((word >> (sh + b)) & 1)
                acc = g2j_add_affine(acc, {f2_c(pc::G2_POW2[b0 + b][0]), f2_c(pc::G2_POW2[b0 + b][1])});
        p2[i] = acc;
        __syncthreads();
        for (uint32_t s = VBP_THREADS / 2; s > 0; s >>= 1) {
            if (i < s) p2[i] = g2j_add(p2[i], p2[i + s]);
            __syncthreads();
        }
        if (i == 0) {
            G2Jac zg = p2[0];
            if (!f2_is_zero(zg.Z)) zg.Y = f2_neg(zg.Y);
            P[t] = xyzz_to_affine(sums[t - 1]);
            Q[t] = g2j_to_affine(g2j_add_affine(zg, g2_alpha));
        }
    }
}

__global__ void k_g2_mul(G2Affine base, Fr k_mont, G2Affine* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const Fr kc = to_canonical(k_mont);
    uint32_t k[8];
    for (int i = 0; i < 8; i++) k[i] = kc.v[i];
    *out = g2j_to_affine(g2_mul_words(base, k));
}

// ---- ABI conversions ----------------------------------------------------------------------------

Fq fq_from_u64x4(const uint64_t (&l)[4]) {
    Fq r;
    for (int i = 0; i < 4; i++) {
        r.v[2 * i] = (uint32_t)l[i];
        r.v[2 * i + 1] = (uint32_t)(l[i] >> 32);
    }
    return r;
}

void fq_to_u64x4(const Fq& a, uint64_t (&l)[4]) {
    for (int i = 0; i < 4; i++) l[i] = (uint64_t)a.v[2 * i] | (uint64_t)a.v[2 * i + 1] << 32;
}

bool fq_is_canonical(const Fq& x) {
    for (int i = 7; i >= 0; i--) {
        if (x.v[i] < FqP::P[i]) return true;
        if (x.v[i] > FqP::P[i]) return false;
    }
    return false;
}

Status g2_from_abi(const eon_g2_affine& a, G2Affine& out) {
    out.x = {fq_from_u64x4(a.x[0]), fq_from_u64x4(a.x[1])};
    out.y = {fq_from_u64x4(a.y[0]), fq_from_u64x4(a.y[1])};
    for (const Fq* c : {&out.x.c0, &out.x.c1, &out.y.c0, &out.y.c1})
        if (!fq_is_canonical(*c)) return Status::err(EON_E_ARG, "G2 coordinate is not a canonical Fq");
    if (!g2_on_curve(out)) return Status::err(EON_E_ARG, "G2 point is not on the twist curve");
    return Status::ok();
}

void g2_to_abi(const G2Affine& a, eon_g2_affine& out) {
    fq_to_u64x4(a.x.c0, out.x[0]);
    fq_to_u64x4(a.x.c1, out.x[1]);
    fq_to_u64x4(a.y.c0, out.y[0]);
    fq_to_u64x4(a.y.c1, out.y[1]);
}

Status g1_from_abi(const eon_g1_affine& a, G1Affine& out) {
    out.x = fq_from_u64x4(a.x);
    out.y = fq_from_u64x4(a.y);
    if (!fq_is_canonical(out.x) || !fq_is_canonical(out.y))
        return Status::err(EON_E_ARG, "G1 coordinate is not a canonical Fq");
    if (!is_inf(out)) {
        // y^2 = x^3 + 3
        const Fq lhs = mul(out.y, out.y);
        const Fq rhs = add(mul(mul(out.x, out.x), out.x), from_u64<FqP>(3));
        if (lhs != rhs) return Status::err(EON_E_ARG, "G1 point is not on the curve");
    }
    return Status::ok();
}

void fq12_to_abi(const Fq12& a, eon_fq12& out) {
    const Fq2* x = &a.c0.c0;
    for (int i = 0; i < 6; i++) {
        fq_to_u64x4(x[i].c0, out.c[2 * i]);
        fq_to_u64x4(x[i].c1, out.c[2 * i + 1]);
    }
}

// product of the pairings of m device pairs -> Gt element and the is-one flag (host)
Status pair_product(eon_ctx* ctx, const G1Affine* P, const G2Affine* Q, uint32_t m, Fq12* gt, bool* one) {
    DevBuf f, res;
    PoolScope ps(ctx->pool, ctx->stream);
    EON_HIP(ps.take(f, (size_t)std::max<uint32_t>(m, 1) * sizeof(Fq12)));
    EON_HIP(ps.take(res, sizeof(Fq12) + 16));
    ctx->prof.begin("k_miller_team", (uint64_t)m * (64 + 128 + 384), ctx->stream);
    if (m) hipLaunchKernelGGL(k_miller_team, dim3((m + 64 / TEAM - 1) / (64 / TEAM)), dim3(64), 0, ctx->stream, P, Q, m,
                              f.as<Fq12>());
    ctx->prof.end(ctx->stream);
    ctx->prof.begin("k_final_exp_team", (uint64_t)m * 384 + 384, ctx->stream);
    hipLaunchKernelGGL(k_final_exp_team, dim3(1), dim3(TEAM), 0, ctx->stream, f.as<Fq12>(), m, res.as<Fq12>(),
                       reinterpret_cast<uint32_t*>(res.as<char>() + sizeof(Fq12)));
    ctx->prof.end(ctx->stream);
    EON_HIP(hipGetLastError());
    struct {
        Fq12 v;
        uint32_t flag;
    } host;
    EON_HIP(hipMemcpyAsync(&host.v, res.p, sizeof(Fq12), hipMemcpyDeviceToHost, ctx->stream));
    EON_HIP(hipMemcpyAsync(&host.flag, res.as<char>() + sizeof(Fq12), 4, hipMemcpyDeviceToHost, ctx->stream));
    EON_HIP(hipStreamSynchronize(ctx->stream));
    if (gt) *gt = host.v;
    if (one) *one = host.flag != 0;
    return Status::ok();
}

int finish(eon_ctx* ctx, const Status& s) {
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // namespace

extern "C" {

int eon_g2_mul(eon_ctx* ctx, const eon_g2_affine* base, const eon_fr* k, eon_g2_affine* out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!k || !out) return Status::err(EON_E_ARG, "null argument");
        G2Affine b = g2_generator();
        if (base) EON_TRY(g2_from_abi(*base, b));
        const Fr kk = fr_from_abi(k);
        if (!fr_is_canonical(kk)) return Status::err(EON_E_ARG, "scalar is not a canonical Fr");
        DevBuf d;
        PoolScope ps(ctx->pool, ctx->stream);
        EON_HIP(ps.take(d, sizeof(G2Affine)));
        hipLaunchKernelGGL(k_g2_mul, dim3(1), dim3(64), 0, ctx->stream, b, kk, d.as<G2Affine>());
        EON_HIP(hipGetLastError());
        G2Affine r;
        EON_HIP(hipMemcpyAsync(&r, d.p, sizeof(r), hipMemcpyDeviceToHost, ctx->stream));
        EON_HIP(hipStreamSynchronize(ctx->stream));
        g2_to_abi(r, *out);
        return Status::ok();
    }();
    return finish(ctx, s);
}

int eon_multi_pairing(eon_ctx* ctx, const eon_g1_affine* p, const eon_g2_affine* q, uint64_t n, eon_fq12* out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!out || (n && (!p || !q))) return Status::err(EON_E_ARG, "null argument");
        if (n > (1u << 24)) return Status::err(EON_E_SHAPE, "at most 2^24 pairs");
        std::vector<G1Affine> hp(n);
        std::vector<G2Affine> hq(n);
        for (uint64_t i = 0; i < n; i++) {
            EON_TRY(g1_from_abi(p[i], hp[i]));
            EON_TRY(g2_from_abi(q[i], hq[i]));
        }
        DevBuf dp, dq;
        PoolScope ps(ctx->pool, ctx->stream);
        EON_HIP(ps.take(dp, std::max<uint64_t>(n, 1) * sizeof(G1Affine)));
        EON_HIP(ps.take(dq, std::max<uint64_t>(n, 1) * sizeof(G2Affine)));
        if (n) {
            EON_HIP(hipMemcpyAsync(dp.p, hp.data(), n * sizeof(G1Affine), hipMemcpyHostToDevice, ctx->stream));
            EON_HIP(hipMemcpyAsync(dq.p, hq.data(), n * sizeof(G2Affine), hipMemcpyHostToDevice, ctx->stream));
        }
        Fq12 gt;
        EON_TRY(pair_product(ctx, dp.as<G1Affine>(), dq.as<G2Affine>(), (uint32_t)n, &gt, nullptr));
        fq12_to_abi(gt, *out);
        return Status::ok();
    }();
    return finish(ctx, s);
}

int eon_kzg_verify_batch(eon_ctx* ctx, const eon_g1_affine* commitments, const eon_g1_affine* witnesses,
                         const eon_fr* values, const eon_fr* points, uint64_t n, const eon_g2_affine* g2_alpha,
                         int* ok) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!ok || !g2_alpha || (n && (!commitments || !witnesses || !values || !points)))
            return Status::err(EON_E_ARG, "null argument");
        if (n > (1u << 26)) return Status::err(EON_E_SHAPE, "at most 2^26 openings");
        *ok = 0;
        if (n == 0) {  // verify_batch: no openings is Ok(())
            *ok = 1;
            return Status::ok();
        }
        G2Affine ga;
        EON_TRY(g2_from_abi(*g2_alpha, ga));
        std::vector<G1Affine> hc(n), hw(n);
        std::vector<Fr> hv(n);
        // group the openings by point (host: the points are few and small)
        std::map<std::vector<uint32_t>, uint32_t> gid;
        std::vector<Fr> zs;
        std::vector<uint32_t> grp(n);
        for (uint64_t i = 0; i < n; i++) {
            EON_TRY(g1_from_abi(commitments[i], hc[i]));
            EON_TRY(g1_from_abi(witnesses[i], hw[i]));
            hv[i] = fr_from_abi(&values[i]);
            const Fr z = fr_from_abi(&points[i]);
            if (!fr_is_canonical(hv[i]) || !fr_is_canonical(z)) return Status::err(EON_E_ARG, "value or point is not a canonical Fr");
            std::vector<uint32_t> key(z.v, z.v + 8);
            auto it = gid.find(key);
            if (it == gid.end()) {
                it = gid.emplace(key, (uint32_t)zs.size()).first;
                zs.push_back(z);
            }
            grp[i] = it->second;
        }
        const uint32_t G = (uint32_t)zs.size();
        std::vector<uint32_t> gs(G + 1, 0), ord(n);
        for (uint64_t i = 0; i < n; i++) gs[grp[i] + 1]++;
        for (uint32_t g = 0; g < G; g++) gs[g + 1] += gs[g];
        {
            std::vector<uint32_t> fill(gs.begin(), gs.end() - 1);
            for (uint64_t i = 0; i < n; i++) ord[fill[grp[i]]++] = (uint32_t)i;
        }
        DevBuf dc, dw, dv, dord, dgs, dz, dsums, dvsum, dP, dQ;
        PoolScope ps(ctx->pool, ctx->stream);
        EON_HIP(ps.take(dc, n * sizeof(G1Affine)));
        EON_HIP(ps.take(dw, n * sizeof(G1Affine)));
        EON_HIP(ps.take(dv, n * sizeof(Fr)));
        EON_HIP(ps.take(dord, n * 4));
        EON_HIP(ps.take(dgs, (G + 1) * 4));
        EON_HIP(ps.take(dz, G * sizeof(Fr)));
        EON_HIP(ps.take(dsums, (G + 1) * sizeof(G1Xyzz)));
        EON_HIP(ps.take(dvsum, sizeof(Fr)));
        EON_HIP(ps.take(dP, (G + 1) * sizeof(G1Affine)));
        EON_HIP(ps.take(dQ, (G + 1) * sizeof(G2Affine)));
        hipStream_t st = ctx->stream;
        EON_HIP(hipMemcpyAsync(dc.p, hc.data(), n * sizeof(G1Affine), hipMemcpyHostToDevice, st));
        EON_HIP(hipMemcpyAsync(dw.p, hw.data(), n * sizeof(G1Affine), hipMemcpyHostToDevice, st));
        EON_HIP(hipMemcpyAsync(dv.p, hv.data(), n * sizeof(Fr), hipMemcpyHostToDevice, st));
        EON_HIP(hipMemcpyAsync(dord.p, ord.data(), n * 4, hipMemcpyHostToDevice, st));
        EON_HIP(hipMemcpyAsync(dgs.p, gs.data(), (G + 1) * 4, hipMemcpyHostToDevice, st));
        EON_HIP(hipMemcpyAsync(dz.p, zs.data(), G * sizeof(Fr), hipMemcpyHostToDevice, st));
        // algorithmic bytes: each opening's commitment, witness, value and point read once
        ctx->prof.begin("k_vb_sums", n * (64 + 64 + 32 + 32), st);
        hipLaunchKernelGGL(k_vb_sums, dim3(G + 1), dim3(VB_THREADS), 0, st, dc.as<G1Affine>(), dw.as<G1Affine>(),
                           dv.as<Fr>(), dord.as<uint32_t>(), dgs.as<uint32_t>(), G, (uint32_t)n, dsums.as<G1Xyzz>(),
                           dvsum.as<Fr>());
        ctx->prof.end(st);
        ctx->prof.begin("k_vb_pairs", (uint64_t)(G + 1) * (96 + 192), st);
        hipLaunchKernelGGL(k_vb_pairs, dim3(G + 1), dim3(VBP_THREADS), 0, st, dsums.as<G1Xyzz>(), dvsum.as<Fr>(),
                           dz.as<Fr>(), G, ga, dP.as<G1Affine>(), dQ.as<G2Affine>());
        ctx->prof.end(st);
        EON_HIP(hipGetLastError());
        bool one = false;
        EON_TRY(pair_product(ctx, dP.as<G1Affine>(), dQ.as<G2Affine>(), G + 1, nullptr, &one));
        *ok = one ? 1 : 0;
        return Status::ok();
    }();
    return finish(ctx, s);
}

}  // extern "C"
