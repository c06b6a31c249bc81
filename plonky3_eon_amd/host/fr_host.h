// Host-side BN254 Fr for the prove driver: the domain bookkeeping (coset shifts, the next-row
// point, lane weights) and the Fiat-Shamir transcript's Poseidon2 permutations (transcript.cpp:
// ~2.6k permutations of ~240 products each per headline proof, on the critical path of every rank
// of the sharded prove -- so the product is a fully unrolled 4x64 CIOS with compile-time
// constants, and the permutation keeps its state in the lazily reduced range [0, 2r)).
//
// Values are eon_fr: [u64;4] little-endian Montgomery residues a*2^256 mod r, canonical -- the
// layout of p3_bn254::Fr (bn254/src/field.rs:98-105); products follow monty_mul's contract
// (bn254/src/helpers.rs:168-205): the canonical representative of a*b*2^-256.
#pragma once
#include <cpuid.h>
#include <stdint.h>
#include <stdlib.h>

#include "eon.h"

namespace eon_host {

struct Fr {
    uint64_t l[4];

    static constexpr uint64_t P[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull,
                                      0xb85045b68181585dull, 0x30644e72e131a029ull};
    // 2r (< 2^255): the bound of the lazily reduced form
    static constexpr uint64_t P2[4] = {0x87c3eb27e0000002ull, 0x5067d090f372e122ull,
                                       0x70a08b6d0302b0baull, 0x60c89ce5c2634053ull};
    // -r^-1 mod 2^64
    static constexpr uint64_t INV = 0xc2e1f593efffffffull;
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
static_assert(Fr::P[0] * Fr::INV == ~0ull, "INV = -r^-1 mod 2^64");

// -r^-1 mod 2^64 by Newton iteration on the low limb (kept for the tests' cross-check of INV)
inline uint64_t fr_inv64() {
    uint64_t x = 1;
    for (int i = 0; i < 6; i++) x *= 2 - Fr::P[0] * x;
    return ~x + 1;
}

namespace detail {
typedef unsigned __int128 u128;

// x - m when x >= m, else x (branch-free); x < 2^256, m one of P / P2
inline void cond_sub(uint64_t x[4], const uint64_t m[4]) {
    uint64_t d[4];
    u128 t = (u128)x[0] - m[0];
    d[0] = (uint64_t)t;
    t = (u128)x[1] - m[1] - (uint64_t)(t >> 127);
    d[1] = (uint64_t)t;
    t = (u128)x[2] - m[2] - (uint64_t)(t >> 127);
    d[2] = (uint64_t)t;
    t = (u128)x[3] - m[3] - (uint64_t)(t >> 127);
    d[3] = (uint64_t)t;
    uint64_t keep = 0 - (uint64_t)(t >> 127);  // all ones when x < m (the subtraction borrowed)
    // opaque to the compiler, so the select stays arithmetic: as a branch it mispredicts about
    // half the time on the transcript's chain (~20 cycles each)
    asm("" : "+r"(keep));
    for (int i = 0; i < 4; i++) x[i] = (x[i] & keep) | (d[i] & ~keep);
}

// One CIOS round: t = (t + a * bi + m r) / 2^64 with m chosen so the low word vanishes.  With
// a, b < 2r and t < 3r on entry, t stays below 3r (< 2^256) after every round, so four words
// and one carry word suffice.
#define EON_FR_CIOS_ROUND(bi)                                             \
    {                                                                     \
        u128 c = (u128)a[0] * (bi) + t0;                                  \
        const uint64_t s0 = (uint64_t)c;                                  \
        c = (u128)a[1] * (bi) + t1 + (uint64_t)(c >> 64);                 \
        const uint64_t s1 = (uint64_t)c;                                  \
        c = (u128)a[2] * (bi) + t2 + (uint64_t)(c >> 64);                 \
        const uint64_t s2 = (uint64_t)c;                                  \
        c = (u128)a[3] * (bi) + t3 + (uint64_t)(c >> 64);                 \
        const uint64_t s3 = (uint64_t)c;                                  \
        const uint64_t s4 = (uint64_t)(c >> 64);                          \
        const uint64_t m = s0 * Fr::INV;                                  \
        c = (u128)m * Fr::P[0] + s0;                                      \
        c = (u128)m * Fr::P[1] + s1 + (uint64_t)(c >> 64);                \
        t0 = (uint64_t)c;                                                 \
        c = (u128)m * Fr::P[2] + s2 + (uint64_t)(c >> 64);                \
        t1 = (uint64_t)c;                                                 \
        c = (u128)m * Fr::P[3] + s3 + (uint64_t)(c >> 64);                \
        t2 = (uint64_t)c;                                                 \
        t3 = s4 + (uint64_t)(c >> 64);                                    \
    }

// a * b * 2^-256 mod r for a, b < 2r, result < 2r (no final subtraction: (ab + mr) / 2^256 <
// 4r^2 / 2^256 + r < 2r since 4r < 2^256)
inline void mont_mul_lazy(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    EON_FR_CIOS_ROUND(b[0]);
    EON_FR_CIOS_ROUND(b[1]);
    EON_FR_CIOS_ROUND(b[2]);
    EON_FR_CIOS_ROUND(b[3]);
    out[0] = t0, out[1] = t1, out[2] = t2, out[3] = t3;
}
#undef EON_FR_CIOS_ROUND

// The same product with MULX and the two carry chains of ADCX / ADOX (BMI2 + ADX): ~2x lower
// latency than the compiler's code for the u128 form above, which matters because the sponge's
// partial rounds are one dependent chain of products.  `a` is passed in four registers (no store /
// reload on the chain), `b` word by word into rdx from memory or registers.  Register roles rotate
// over the four rounds (T0 of a round is zero after its reduction and becomes the next round's
// carry word), so no moves between rounds.  Same bounds as mont_mul_lazy; the clang and gcc
// assemblers accept these instructions without target flags, and kCpuAdx gates every use at run
// time.
#define EON_FR_ADX_ROUND(BSRC, T0, T1, T2, T3, T4) \
    "movq " BSRC ", %%rdx\n\t"                     \
    "xorl %k[lo], %k[lo]\n\t"                     \
    "mulxq %[a0], %[lo], %[hi]\n\t"               \
    "adoxq %[lo], " T0 "\n\t"                     \
    "adcxq %[hi], " T1 "\n\t"                     \
    "mulxq %[a1], %[lo], %[hi]\n\t"               \
    "adoxq %[lo], " T1 "\n\t"                     \
    "adcxq %[hi], " T2 "\n\t"                     \
    "mulxq %[a2], %[lo], %[hi]\n\t"               \
    "adoxq %[lo], " T2 "\n\t"                     \
    "adcxq %[hi], " T3 "\n\t"                     \
    "mulxq %[a3], %[lo], %[hi]\n\t"               \
    "adoxq %[lo], " T3 "\n\t"                     \
    "adcxq %[hi], " T4 "\n\t"                     \
    "movl $0, %k[lo]\n\t"                         \
    "adoxq %[lo], " T4 "\n\t"                     \
    "movq " T0 ", %%rdx\n\t"                      \
    "imulq %[inv], %%rdx\n\t"                     \
    "xorl %k[lo], %k[lo]\n\t"                     \
    "mulxq %[p0], %[lo], %[hi]\n\t"               \
    "adcxq %[lo], " T0 "\n\t"                     \
    "adoxq %[hi], " T1 "\n\t"                     \
    "mulxq %[p1], %[lo], %[hi]\n\t"               \
    "adcxq %[lo], " T1 "\n\t"                     \
    "adoxq %[hi], " T2 "\n\t"                     \
    "mulxq %[p2], %[lo], %[hi]\n\t"               \
    "adcxq %[lo], " T2 "\n\t"                     \
    "adoxq %[hi], " T3 "\n\t"                     \
    "mulxq %[p3], %[lo], %[hi]\n\t"               \
    "adcxq %[lo], " T3 "\n\t"                     \
    "adoxq %[hi], " T4 "\n\t"                     \
    "movl $0, %k[lo]\n\t"                         \
    "adcxq %[lo], " T4 "\n\t"
#define EON_FR_ADX_OUTS                                                                                 \
    [r0] "+&r"(r0), [r1] "+&r"(r1), [r2] "+&r"(r2), [r3] "+&r"(r3), [r4] "+&r"(r4), [lo] "=&r"(lo), \
        [hi] "=&r"(hi)
#define EON_FR_ADX_CONSTS                                                                         \
    [p0] "m"(Fr::P[0]), [p1] "m"(Fr::P[1]), [p2] "m"(Fr::P[2]), [p3] "m"(Fr::P[3]), [inv] "m"(Fr::INV)

inline void mont_mul_adx(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    uint64_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, lo, hi;
    asm(EON_FR_ADX_ROUND("0(%[b])", "%[r0]", "%[r1]", "%[r2]", "%[r3]", "%[r4]")
        EON_FR_ADX_ROUND("8(%[b])", "%[r1]", "%[r2]", "%[r3]", "%[r4]", "%[r0]")
        EON_FR_ADX_ROUND("16(%[b])", "%[r2]", "%[r3]", "%[r4]", "%[r0]", "%[r1]")
        EON_FR_ADX_ROUND("24(%[b])", "%[r3]", "%[r4]", "%[r0]", "%[r1]", "%[r2]")
        : EON_FR_ADX_OUTS
        : [a0] "r"(a[0]), [a1] "r"(a[1]), [a2] "r"(a[2]), [a3] "r"(a[3]), [b] "r"(b),
          "m"(*(const uint64_t(*)[4])b), EON_FR_ADX_CONSTS
        : "rdx", "cc");
    out[0] = r4, out[1] = r0, out[2] = r1, out[3] = r2;
}

// a * a: both operands in registers
inline void mont_sqr_adx(const uint64_t a[4], uint64_t out[4]) {
    uint64_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, lo, hi;
    asm(EON_FR_ADX_ROUND("%[a0]", "%[r0]", "%[r1]", "%[r2]", "%[r3]", "%[r4]")
        EON_FR_ADX_ROUND("%[a1]", "%[r1]", "%[r2]", "%[r3]", "%[r4]", "%[r0]")
        EON_FR_ADX_ROUND("%[a2]", "%[r2]", "%[r3]", "%[r4]", "%[r0]", "%[r1]")
        EON_FR_ADX_ROUND("%[a3]", "%[r3]", "%[r4]", "%[r0]", "%[r1]", "%[r2]")
        : EON_FR_ADX_OUTS
        : [a0] "r"(a[0]), [a1] "r"(a[1]), [a2] "r"(a[2]), [a3] "r"(a[3]), EON_FR_ADX_CONSTS
        : "rdx", "cc");
    out[0] = r4, out[1] = r0, out[2] = r1, out[3] = r2;
}
#undef EON_FR_ADX_ROUND
#undef EON_FR_ADX_OUTS
#undef EON_FR_ADX_CONSTS

// BMI2 (CPUID.7.0:EBX bit 8) and ADX (bit 19); EON_HOST_NO_ADX=1 forces the portable product
inline bool detect_adx() {
    const char* off = getenv("EON_HOST_NO_ADX");
    if (off && off[0] == '1') return false;
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    return (b & (1u << 8)) && (b & (1u << 19));
}
inline const bool kCpuAdx = detect_adx();

inline void mont_mul(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    if (kCpuAdx)
        mont_mul_adx(a, b, out);
    else
        mont_mul_lazy(a, b, out);
}

// a + b for a, b < 2r: < 4r < 2^256, brought below 2r
inline void add_lazy(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
#if defined(__x86_64__)
    // add / sbb chains and cmov: ~10 cycles on the transcript's dependency chain, against ~19 for
    // the compiler's masked form
    uint64_t r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], t0, t1, t2, t3;
    asm("addq %[b0], %[r0]\n\t"
        "adcq %[b1], %[r1]\n\t"
        "adcq %[b2], %[r2]\n\t"
        "adcq %[b3], %[r3]\n\t"
        "movq %[r0], %[t0]\n\t"
        "subq %[m0], %[t0]\n\t"
        "movq %[r1], %[t1]\n\t"
        "sbbq %[m1], %[t1]\n\t"
        "movq %[r2], %[t2]\n\t"
        "sbbq %[m2], %[t2]\n\t"
        "movq %[r3], %[t3]\n\t"
        "sbbq %[m3], %[t3]\n\t"
        "cmovncq %[t0], %[r0]\n\t"  // no borrow: the sum is >= 2r, keep the difference
        "cmovncq %[t1], %[r1]\n\t"
        "cmovncq %[t2], %[r2]\n\t"
        "cmovncq %[t3], %[r3]\n\t"
        : [r0] "+&r"(r0), [r1] "+&r"(r1), [r2] "+&r"(r2), [r3] "+&r"(r3), [t0] "=&r"(t0), [t1] "=&r"(t1),
          [t2] "=&r"(t2), [t3] "=&r"(t3)
        : [b0] "rm"(b[0]), [b1] "rm"(b[1]), [b2] "rm"(b[2]), [b3] "rm"(b[3]), [m0] "m"(Fr::P2[0]),
          [m1] "m"(Fr::P2[1]), [m2] "m"(Fr::P2[2]), [m3] "m"(Fr::P2[3])
        : "cc");
    out[0] = r0, out[1] = r1, out[2] = r2, out[3] = r3;
#else
    u128 c = (u128)a[0] + b[0];
    out[0] = (uint64_t)c;
    c = (u128)a[1] + b[1] + (uint64_t)(c >> 64);
    out[1] = (uint64_t)c;
    c = (u128)a[2] + b[2] + (uint64_t)(c >> 64);
    out[2] = (uint64_t)c;
    out[3] = a[3] + b[3] + (uint64_t)(c >> 64);
    cond_sub(out, Fr::P2);
#endif
}
}  // namespace detail

// Lazily reduced element: any representative below 2r (the permutation's working form)
struct FrLazy {
    uint64_t l[4];
    static FrLazy of(const Fr& a) { return FrLazy{{a.l[0], a.l[1], a.l[2], a.l[3]}}; }
    Fr canonical() const {
        Fr r{{l[0], l[1], l[2], l[3]}};
        detail::cond_sub(r.l, Fr::P);
        return r;
    }
};
// ADX selects the product at compile time (the permutation is instantiated for both and picks
// one per call by detail::kCpuAdx)
template <bool ADX = false>
inline FrLazy lz_mul(const FrLazy& a, const FrLazy& b) {
    FrLazy r;
    if (ADX)
        detail::mont_mul_adx(a.l, b.l, r.l);
    else
        detail::mont_mul_lazy(a.l, b.l, r.l);
    return r;
}
template <bool ADX = false>
inline FrLazy lz_sqr(const FrLazy& a) {
    FrLazy r;
    if (ADX)
        detail::mont_sqr_adx(a.l, r.l);
    else
        detail::mont_mul_lazy(a.l, a.l, r.l);
    return r;
}
inline FrLazy lz_add(const FrLazy& a, const FrLazy& b) {
    FrLazy r;
    detail::add_lazy(a.l, b.l, r.l);
    return r;
}

// a / 2 for a < 2r: a >> 1 when a is even, else (a + r) >> 1 (< 3r / 2)
inline FrLazy lz_half(const FrLazy& a) {
    uint64_t odd = 0 - (a.l[0] & 1);
    asm("" : "+r"(odd));  // keep the mask arithmetic (see cond_sub)
    uint64_t w[4];
    detail::u128 c = (detail::u128)a.l[0] + (Fr::P[0] & odd);
    w[0] = (uint64_t)c;
    c = (detail::u128)a.l[1] + (Fr::P[1] & odd) + (uint64_t)(c >> 64);
    w[1] = (uint64_t)c;
    c = (detail::u128)a.l[2] + (Fr::P[2] & odd) + (uint64_t)(c >> 64);
    w[2] = (uint64_t)c;
    w[3] = a.l[3] + (Fr::P[3] & odd) + (uint64_t)(c >> 64);  // a + r < 3r < 2^256
    return FrLazy{{(w[0] >> 1) | (w[1] << 63), (w[1] >> 1) | (w[2] << 63), (w[2] >> 1) | (w[3] << 63), w[3] >> 1}};
}

inline Fr fr_mul(const Fr& a, const Fr& b) {
    Fr r;
    detail::mont_mul(a.l, b.l, r.l);
    detail::cond_sub(r.l, Fr::P);
    return r;
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
