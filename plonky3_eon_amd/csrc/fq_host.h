// Host-side Fq (the BN254 G1 base field) arithmetic in 4 x 64-bit limbs, Montgomery form
// x 2^256 mod q -- the same residues as the device's Fq (field.h), so bytes are interchangeable:
// msm.hip converts a call's few XYZZ results to affine on the host with it (batch inversion).
// Self-contained (no HIP headers): tests/fq_host_check.cpp compiles it with the host compiler.
#pragma once
#include <cstdint>

namespace eon {
namespace hostq {

// q and 2^512 mod q (the device's FqP::P / FqP::R2 as 64-bit limbs)
constexpr uint64_t FQ_P64[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull,
                                0x30644e72e131a029ull};
constexpr uint64_t FQ_R2_64[4] = {0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull, 0x47ab1eff0a417ff6ull,
                                  0x06d89f71cab8351full};

struct F {
    uint64_t l[4];
};

static const F& P() {
    static const F p = [] {
        F r;
        for (int i = 0; i < 4; i++) r.l[i] = FQ_P64[i];
        return r;
    }();
    return p;
}

static uint64_t inv64() {
    static const uint64_t v = [] {
        uint64_t x = 1;
        for (int i = 0; i < 6; i++) x *= 2 - P().l[0] * x;
        return ~x + 1;
    }();
    return v;
}

static bool is_zero(const F& a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0; }

// a b 2^-256 mod p, canonical (CIOS)
static F mul(const F& a, const F& b) {
    const F& p = P();
    const uint64_t inv = inv64();
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        unsigned __int128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (unsigned __int128)a.l[j] * b.l[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[4] = (uint64_t)c;
        t[5] = (uint64_t)(c >> 64);
        const uint64_t m = t[0] * inv;
        c = (unsigned __int128)m * p.l[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 4; j++) {
            c += (unsigned __int128)m * p.l[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[3] = (uint64_t)c;
        t[4] = t[5] + (uint64_t)(c >> 64);
    }
    F r{{t[0], t[1], t[2], t[3]}}, d;
    uint64_t borrow = 0;
    for (int i = 0; i < 4; i++) {
        const unsigned __int128 x = (unsigned __int128)t[i] - p.l[i] - borrow;
        d.l[i] = (uint64_t)x;
        borrow = (uint64_t)(x >> 64) & 1;
    }
    return (t[4] || !borrow) ? d : r;
}

static bool is_one(const F& a) { return a.l[0] == 1 && (a.l[1] | a.l[2] | a.l[3]) == 0; }
static bool geq(const F& a, const F& b) {
    for (int i = 3; i >= 0; i--)
        if (a.l[i] != b.l[i]) return a.l[i] > b.l[i];
    return true;
}
static void sub_in(F& a, const F& b) {  // a -= b (a >= b)
    unsigned __int128 br = 0;
    for (int i = 0; i < 4; i++) {
        const unsigned __int128 x = (unsigned __int128)a.l[i] - b.l[i] - (uint64_t)br;
        a.l[i] = (uint64_t)x;
        br = (x >> 64) & 1;
    }
}
static void add_in(F& a, const F& b) {  // a += b (no overflow: both below 2^255)
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (unsigned __int128)a.l[i] + b.l[i];
        a.l[i] = (uint64_t)c;
        c >>= 64;
    }
}
static void shr1(F& a) {
    for (int i = 0; i < 3; i++) a.l[i] = (a.l[i] >> 1) | (a.l[i + 1] << 63);
    a.l[3] >>= 1;
}
// x / 2 mod p for x < p
static void half_mod(F& x) {
    if (x.l[0] & 1) add_in(x, P());
    shr1(x);
}
// x - y mod p for x, y < p
static void sub_mod(F& x, const F& y) {
    if (!geq(x, y)) add_in(x, P());
    sub_in(x, y);
}

// the Montgomery-form inverse of a = x 2^256: the binary extended Euclid algorithm gives a^-1 mod p
// (~2 log2 p shift / subtract steps, against ~380 products for a^(p-2)), and one Montgomery product
// by 2^768 mod p brings it to x^-1 2^256.  a is first reduced below p; a = 0 mod p (no inverse)
// returns 0, as a^(p-2) did -- the loop below would never end on u = 0.
static F inverse(const F& a_in) {
    static const F r3 = [] {
        F r2;
        for (int i = 0; i < 4; i++) r2.l[i] = FQ_R2_64[i];
        return mul(r2, r2);  // 2^512 2^512 2^-256
    }();
    F a = a_in;
    while (geq(a, P())) sub_in(a, P());  // a < 2^256 < 6p: at most five subtractions
    if (is_zero(a)) return a;
    F u = a, v = P(), x1{{1, 0, 0, 0}}, x2{{0, 0, 0, 0}};
    while (!is_one(u) && !is_one(v)) {
        while (!(u.l[0] & 1)) {
            shr1(u);
            half_mod(x1);
        }
        while (!(v.l[0] & 1)) {
            shr1(v);
            half_mod(x2);
        }
        if (geq(u, v)) {
            sub_in(u, v);
            sub_mod(x1, x2);
        } else {
            sub_in(v, u);
            sub_mod(x2, x1);
        }
    }
    return mul(is_one(u) ? x1 : x2, r3);
}

}  // namespace hostq
}  // namespace eon
