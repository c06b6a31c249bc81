// Host-side BN254 Fr for the prove driver's domain bookkeeping (coset shifts, the next-row point,
// lane weights): a handful of products per proof, so plain 64-bit-limb Montgomery arithmetic.
//
// Values are eon_fr: [u64;4] little-endian Montgomery residues a*2^256 mod r, canonical -- the
// layout of p3_bn254::Fr (bn254/src/field.rs:98-105); products follow monty_mul's contract
// (bn254/src/helpers.rs:168-205): the canonical representative of a*b*2^-256.
#pragma once
#include <stdint.h>

#include "eon.h"

namespace eon_host {

struct Fr {
    uint64_t l[4];

    static constexpr uint64_t P[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull,
                                      0xb85045b68181585dull, 0x30644e72e131a029ull};
    // 2^256 mod r (Montgomery ONE) and 2^512 mod r
    static constexpr uint64_t ONE[4] = {0xac96341c4ffffffbull, 0x36fc76959f60cd29ull,
                                        0x666ea36f7879462eull, 0x0e0a77c19a07df2full};
    static constexpr uint64_t R2[4] = {0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull,
                                       0x8c49833d53bb8085ull, 0x0216d0b17f4e44a5ull};
    // TWO_ADIC_GENERATOR = 5^((r-1)/2^28), Montgomery form (bn254/src/field.rs:556-561)
    static constexpr uint64_t G28[4] = {0x636e735580d13d9cull, 0xa22bf3742445ffd6ull,
                                        0x56452ac01eb203d8ull, 0x1860ef942963f9e7ull};
    static constexpr uint32_t TWO_ADICITY = 28;

    static Fr one() { return Fr{{ONE[0], ONE[1], ONE[2], ONE[3]}}; }
    static Fr zero() { return Fr{{0, 0, 0, 0}}; }
    static Fr from_abi(const eon_fr& a) { return Fr{{a.l[0], a.l[1], a.l[2], a.l[3]}}; }
    eon_fr abi() const {
        eon_fr r;
        for (int i = 0; i < 4; i++) r.l[i] = l[i];
        return r;
    }
    bool operator==(const Fr& o) const {
        return l[0] == o.l[0] && l[1] == o.l[1] && l[2] == o.l[2] && l[3] == o.l[3];
    }
};

// -r^-1 mod 2^64 by Newton iteration on the low limb
inline uint64_t fr_inv64() {
    uint64_t x = 1;
    for (int i = 0; i < 6; i++) x *= 2 - Fr::P[0] * x;
    return ~x + 1;
}

inline Fr fr_mul(const Fr& a, const Fr& b) {
    static const uint64_t inv = fr_inv64();
    // CIOS with a 5-word accumulator (r < 2^254, so t stays below 2r before the final subtract)
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
        c = (unsigned __int128)m * Fr::P[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 4; j++) {
            c += (unsigned __int128)m * Fr::P[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[3] = (uint64_t)c;
        t[4] = t[5] + (uint64_t)(c >> 64);
    }
    Fr r{{t[0], t[1], t[2], t[3]}}, d;
    unsigned __int128 br = 0;
    uint64_t borrow = 0;
    for (int i = 0; i < 4; i++) {
        br = (unsigned __int128)t[i] - Fr::P[i] - borrow;
        d.l[i] = (uint64_t)br;
        borrow = (uint64_t)(br >> 64) & 1;
    }
    // t (with its fifth word) >= r exactly when the subtraction did not borrow past t[4]
    return (t[4] == 0 && borrow) ? r : d;
}

inline Fr fr_pow(Fr base, uint64_t e) {
    Fr r = Fr::one();
    while (e) {
        if (e & 1) r = fr_mul(r, base);
        base = fr_mul(base, base);
        e >>= 1;
    }
    return r;
}

inline Fr fr_from_u64(uint64_t x) {
    const Fr r2{{Fr::R2[0], Fr::R2[1], Fr::R2[2], Fr::R2[3]}};
    return fr_mul(Fr{{x, 0, 0, 0}}, r2);
}

// two_adic_generator(bits) (bn254/src/field.rs:563-574): G28 squared 28 - bits times
inline Fr fr_two_adic_generator(uint32_t bits) {
    Fr g{{Fr::G28[0], Fr::G28[1], Fr::G28[2], Fr::G28[3]}};
    for (uint32_t i = bits; i < Fr::TWO_ADICITY; i++) g = fr_mul(g, g);
    return g;
}

}  // namespace eon_host
