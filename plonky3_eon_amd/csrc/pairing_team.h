// Team-parallel Fq12 arithmetic for the verifier's latency-bound chains (pairing.hip: the Miller
// loops and the final exponentiation run on one or a few Fq12 values, so a thread per value
// leaves them as one long dependent chain of Fq2 products).
//
// A team is 6 lanes (of 8 consecutive lanes of a block; lanes 6 and 7 follow along as copies of
// lane 5 and publish nothing); lane k holds the coefficient of w^k of an Fq12 written in the
// w-basis, Fq12 = Fq2[w] / (w^6 - xi) (w^2 = v, v^3 = xi): k even is c0.c(k/2), k odd is
// c1.c((k-1)/2) of pairing.h's tower.  An operation is PUBLISH (each lane writes its coefficients,
// and xi times the right operand's, to the team's LDS slots), a barrier, then COMPUTE (each lane
// reads the slots and forms its own output coefficient).  The functions here are the COMPUTE
// halves for one lane k; they take the slots as plain arrays, so tests/team_check.cpp runs all six
// lanes in turn on the host against the tower's sequential functions.  No lane branches on k:
// which slot a term reads is an address select, so the six lanes stay converged.
//
//   tm_mul       h_k = sum_i a_i b_(k-i mod 6) (times xi when i > k): 6 Fq2 products per lane
//                against f12_mul's 18 in sequence
//   tm_sparse    a times a line's 2 or 3 nonzero coefficients (2-3 products per lane against 13)
//   tm_cyc_sqr   Granger-Scott on the cyclotomic subgroup: 2 Fq2 products per lane against 6
//   tm_frob<J>, tm_conj   coefficient-local (no exchange)
#pragma once
#include "pairing.h"

namespace eon {

EON_HD const Fq2& w_coef(const Fq12& a, int k) {
    const Fq6& h = (k & 1) ? a.c1 : a.c0;
    const int j = k >> 1;
    return j == 0 ? h.c0 : j == 1 ? h.c1 : h.c2;
}

EON_HD void set_w_coef(Fq12& a, int k, const Fq2& v) {
    Fq6& h = (k & 1) ? a.c1 : a.c0;
    const int j = k >> 1;
    if (j == 0)
        h.c0 = v;
    else if (j == 1)
        h.c1 = v;
    else
        h.c2 = v;
}

// h_k of a b: a[0..6) plain, b[0..6) plain and bx[0..6) = xi b
EON_HD Fq2 tm_mul(const Fq2* a, const Fq2* b, const Fq2* bx, int k) {
    Fq2 acc = f2_zero();
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const int j = k - i;
        const Fq2* src = j < 0 ? bx : b;
        acc = f2_add(acc, f2_mul_inl(a[i], src[j < 0 ? j + 6 : j]));
    }
    return acc;
}

// h_k of a l for a sparse l = sum_t l_t w^(j_t), t < N (the j_t the same on every lane): a[0..6)
// plain and ax[0..6) = xi a
template <int N>
EON_HD Fq2 tm_sparse(const Fq2* a, const Fq2* ax, const int (&j)[N], const Fq2 (&l)[N], int k) {
    Fq2 acc = f2_zero();
#pragma unroll
    for (int t = 0; t < N; t++) {
        const int i = k - j[t];
        const Fq2* src = i < 0 ? ax : a;
        acc = f2_add(acc, f2_mul_inl(src[i < 0 ? i + 6 : i], l[t]));
    }
    return acc;
}

// lane k of f12_cyc_sqr (pairing.h): the pairs (w^0, w^3), (w^1, w^4), (w^2, w^5) are the Fq4
// elements x + y Y whose squares give s0 (the even lanes) and s1 (the odd lanes); lane k reads the
// pair m = {0, 3} -> 0, {2, 5} -> 1, {1, 4} -> 2 and its own coefficient z:
//   k even: 3 s0 - 2 z;   k odd: 3 s1 + 2 z, with s1 times xi at k = 1
EON_HD Fq2 tm_cyc_sqr(const Fq2* a, int k) {
    const int m = (k == 0 || k == 3) ? 0 : (k == 2 || k == 5) ? 1 : 2;
    const Fq2 x = a[m], y = a[m + 3], z = a[k];
    const Fq2 t = f2_mul_inl(x, y);
    const Fq2 u = f2_mul_inl(f2_add(x, y), f2_add(x, f2_mul_xi(y)));
    const Fq2 s0 = f2_sub(f2_sub(u, t), f2_mul_xi(t));
    const Fq2 t2 = f2_dbl(t);
    const Fq2 s1 = k == 1 ? f2_mul_xi(t2) : t2;
    const bool even = (k & 1) == 0;
    const Fq2 s = even ? s0 : s1;
    const Fq2 zz = even ? f2_neg(z) : z;
    return f2_add(f2_dbl(f2_add(s, zz)), s);  // 3 s -+ 2 z
}

// coefficient k of a^(q^J): frob_J(a_k) xi^(k (q^J - 1) / 6) (pairing.h f12_frob)
template <int J>
EON_HD Fq2 tm_frob(const Fq2& a, int k) {
    const Fq2 c = (J & 1) ? f2_conj(a) : a;
    const auto& tab = J == 1 ? pc::FROB1 : J == 2 ? pc::FROB2 : pc::FROB3;
    return f2_mul_inl(c, f2_c(tab[k]));
}

// coefficient k of a^(q^6): w -> -w
EON_HD Fq2 tm_conj(const Fq2& a, int k) { return (k & 1) ? f2_neg(a) : a; }

}  // namespace eon
