// BN254 field arithmetic in radix 2^29 (9 limbs in VGPRs, Montgomery R = 2^261) for the MSM's
// register-resident bucket accumulators.
//
// Why a second representation: in radix 2^32 (field.h) every 32x32 multiply-add into a column
// accumulator can carry out of 64 bits, so each v_mad_u64_u32 is followed by a v_addc carry
// capture -- half the issue slots of the product.  With 29-bit limbs a column holds at most 18
// products < 2^60 (both operands' limbs < 2^30), which together with the incoming carry stay below
// 2^64: the product is 162 bare multiply-adds plus a few shifts per column.
//
// Value conventions (p = the modulus, < 2^254):
//   * an element is 9 limbs l[i] with value sum l[i] 2^(29 i); "normalised" = every limb < 2^29;
//   * mul29(a, b) returns a b 2^-261 mod p, normalised, value < 2p, for any inputs whose limbs are
//     < 2^30 and whose values satisfy a b < 0.99 p 2^261 (e.g. both < 12p);
//   * add29_lazy (no carry propagation: limbs < 2^30) feeds a product only; sub29<K> returns
//     a - b + K p normalised (b < K p) -- no conditional subtraction anywhere on the hot path;
//   * canon29 brings a value < 2p to [0, p).
// An element x of the field is held as x 2^261 mod p ("29-Montgomery"); the radix-2^32 ABI form is
// x 2^256 mod p, and to256 / to261 convert with one product each.  unpack29 / pack29 only re-split
// the bits of an integer < 2^256.
#pragma once
#include <type_traits>

#include "field.h"
#include "mad_blocks.h"

namespace eon {

constexpr uint32_t M29 = (1u << 29) - 1;

struct F29 {
    uint32_t l[9];
};

template <class M>
struct R29;

template <>
struct R29<FqP> {
    static constexpr uint32_t P[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                                      0x2db40c0u,  0xa6e141u,  0xe5c2634u,  0x30644eu};
    static constexpr uint32_t INV = 0xe4866389u;  // -p^-1 mod 2^32 (only the low 29 bits are used)
    // 2^261 mod p (the 29-Montgomery one), 2^256 mod p and 2^266 mod p as plain integers
    static constexpr uint32_t ONE[9] = {0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x14c0419u, 0xaa36fb9u,
                                        0x1d4240ceu, 0x11d54c07u, 0x52ac7a8u,  0xdc836u};
    static constexpr uint32_t TO256[9] = {0x58f0d9du,  0x1aea1c6eu, 0x11c2cf74u, 0x11d651ebu, 0x1462c0a7u,
                                          0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0xe0a77u};
    static constexpr uint32_t TO261[9] = {0x13349ca1u, 0x1a5d84a8u, 0xa3e5cacu,  0x100249e0u, 0x12b951e8u,
                                          0xe92d304u,  0x14cb95b3u, 0x41b9d3du,  0x58003u};
};

template <>
struct R29<FrP> {
    static constexpr uint32_t P[9] = {0x10000001u, 0x1f0fac9fu, 0xe5c2450u, 0x7d090f3u, 0x1585d283u,
                                      0x2db40c0u,  0xa6e141u,   0xe5c2634u, 0x30644eu};
    static constexpr uint32_t INV = 0xefffffffu;
    static constexpr uint32_t ONE[9] = {0xfffff57u,  0x1ea70ab4u, 0x52c068bu, 0x17504f49u, 0xaa8075bu,
                                        0x1d4240ceu, 0x11d54c07u, 0x52ac7a8u, 0xdc836u};
    static constexpr uint32_t TO256[9] = {0xffffffbu,  0x4b1a0e2u,  0x18334a6bu, 0x18ed2b3eu, 0x1462e36fu,
                                          0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0xe0a77u};
    static constexpr uint32_t TO261[9] = {0xfffead7u, 0x1d5444f4u, 0x4438aa5u,  0x3b4d096u, 0x134c84dau,
                                          0xe92d304u, 0x14cb95b3u, 0x41b9d3du,  0x58003u};    // 2^261 - p and p^-1 mod 2^261 (Shoup products by twiddles, mul29_shoup / the twiddle tables)
    static constexpr uint32_t NEGP261[9] = {0xfffffffu, 0xf05360u,   0x11a3dbafu, 0x182f6f0cu, 0xa7a2d7cu,
                                            0x1d24bf3fu, 0x1f591ebeu, 0x11a3d9cbu, 0x1fcf9bb1u};
    static constexpr uint32_t PINV261[9] = {0x10000001u, 0x8f05360u,  0x5bb930fu,  0x12f36967u, 0x1dc6e9a7u,
                                            0x13ebb37cu, 0x19347195u, 0x1c5e4f97u, 0xd8c07d0u};
};

// K p as normalised limbs (compile-time)
template <class M, uint32_t K>
struct KP29 {
    uint32_t l[9];
    constexpr KP29() : l{} {
        uint64_t c = 0;
        for (int i = 0; i < 9; i++) {
            c += (uint64_t)R29<M>::P[i] * K;
            l[i] = (uint32_t)(c & M29);
            c >>= 29;
        }
    }
};

template <class M>
EON_HD F29 const29(const uint32_t (&c)[9]) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = c[i];
    return r;
}

// integer < 2^256 in 8 x 32-bit limbs <-> 9 x 29-bit limbs (bit re-split only)
template <class M>
EON_HD F29 unpack29(const Fe<M>& a) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        uint64_t v = a.v[w];
        if (w + 1 < 8) v |= (uint64_t)a.v[w + 1] << 32;
        r.l[i] = (uint32_t)(v >> s) & M29;
    }
    return r;
}

template <class M = FqP>
EON_HD Fe<M> pack29(const F29& a) {
    // a normalised, value < 2^256
    Fe<M> r;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        const int bit = 32 * w, i = bit / 29, s = bit % 29;
        uint64_t v = (uint64_t)a.l[i] >> s;
        if (i + 1 < 9) v |= (uint64_t)a.l[i + 1] << (29 - s);
        if (i + 2 < 9 && 58 - s < 32) v |= (uint64_t)a.l[i + 2] << (58 - s);
        r.v[w] = (uint32_t)v;
    }
    return r;
}

EON_HD bool limbs_ok29(const F29& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) o |= a.l[i];
    return (o >> 29) == 0;
}

EON_HD bool is_zero29_raw(const F29& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) o |= a.l[i];
    return o == 0;
}

// make every limb an opaque register value (no rematerialisation from memory; see field.h pin)
__device__ __forceinline__ void pin29(F29& a) {
#pragma unroll
    for (int i = 0; i < 9; i++) asm volatile("" : "+v"(a.l[i]));
}

// limb-wise a + b, no carry propagation (a, b normalised -> limbs < 2^30): a product input only
EON_HD F29 add29_lazy(const F29& a, const F29& b) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + b.l[i];
    return r;
}

// a + b with carry propagation (normalised result; value a + b < 2^261)
EON_HD F29 add29_norm(const F29& a, const F29& b) {
    F29 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const uint32_t t = a.l[i] + b.l[i] + c;
        r.l[i] = t & M29;
        c = t >> 29;
    }
    return r;
}

// a - b + K p, normalised (requires b < K p; a limbs < 2^30, b limbs < 3 2^29 -- the signed
// column sums stay inside int32)
template <class M, uint32_t K>
EON_HD F29 sub29(const F29& a, const F29& b) {
    constexpr KP29<M, K> kp{};
    F29 r;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int32_t t = (int32_t)(a.l[i] + kp.l[i]) - (int32_t)b.l[i] + c;
        r.l[i] = (uint32_t)t & M29;
        c = t >> 29;  // arithmetic: -1, 0 or 1
    }
    return r;
}

// K p in "borrowed" limbs: every limb below the top one in [2^29 - 1, 2^30), the top one
// (K p)_8 - 1 (same value), so that a - b + K p can be formed limb by limb without carries
template <class M, uint32_t K>
struct KPB29 {
    uint32_t l[9];
    constexpr KPB29() : l{} {
        constexpr KP29<M, K> kp{};
        l[0] = kp.l[0] + (1u << 29);
        for (int i = 1; i < 8; i++) l[i] = kp.l[i] + (1u << 29) - 1;
        l[8] = kp.l[8] - 1;
    }
};

// a - b + K p WITHOUT carry propagation: limbs in [0, 2^31), for a product input whose partner is
// normalised (9 terms < 2^60 per column; mul29 / mul29_sum2 stay below 2^64).  Requires a, b
// normalised and b's top limb < (K p)_8: b < (K - 1) p suffices.
template <class M, uint32_t K>
EON_HD F29 sub29_lazy(const F29& a, const F29& b) {
    constexpr KPB29<M, K> kp{};
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + kp.l[i] - b.l[i];
    return r;
}

// a - b + K p normalised, for a with limbs < 2.5 2^30 (add29_lazy / sub29_lazy outputs) and b
// normalised with b < K p: limb by limb a_i + (K p borrowed)_i - b_i + c in unsigned arithmetic
// (never negative: the borrowed limbs are >= 2^29 - 1 >= b_i, and the top limb is the nonnegative
// remainder of a - b + K p >= 0), so no signed column can overflow as in sub29
template <class M, uint32_t K>
EON_HD F29 sub29_wide(const F29& a, const F29& b) {
    constexpr KPB29<M, K> kp{};
    F29 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const uint32_t t = a.l[i] + kp.l[i] - b.l[i] + c;
        r.l[i] = t & M29;
        c = t >> 29;
    }
    return r;
}

template <class M>
EON_HD F29 mulp29(uint32_t k) {
    F29 r;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        c += (uint64_t)R29<M>::P[i] * k;
        r.l[i] = (uint32_t)(c & M29);
        c >>= 29;
    }
    return r;
}

// a - p if a >= p (a normalised, a < 2p) -> [0, p)
template <class M>
EON_HD F29 canon29(const F29& a) {
    F29 d;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int32_t t = (int32_t)a.l[i] - (int32_t)R29<M>::P[i] + c;
        d.l[i] = (uint32_t)t & M29;
        c = t >> 29;
    }
    return c < 0 ? a : d;
}

// value in {0, p} (a normalised, < 2p): "zero mod p" for a product output.  (A fast reject on
// the lowest limb measured equal: the 18 OR/XOR are cheaper than the branch they would skip.)
template <class M>
EON_HD bool is_zero_mod29(const F29& a) {
    uint32_t z = 0, e = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        z |= a.l[i];
        e |= a.l[i] ^ R29<M>::P[i];
    }
    return z == 0 || e == 0;
}

// acc += a b as ONE v_mad_u64_u32 on the running accumulator: written in asm so that the
// compiler cannot re-associate a column into a separate partial sum merged by an extra 64-bit add
// (what it does with the C++ form: one v_lshl_add_u64 per column, 17 per product).  The host
// pass of the compiler (kernel stubs, host-side users of EON_HD code) sees the plain expression.
EON_HD void mad29_vv(uint64_t& acc, uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "v"(b));
#else
    acc += (uint64_t)a * b;
#endif
}
EON_HD void mad29_vs(uint64_t& acc, uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "s"(b));
#else
    acc += (uint64_t)a * b;
#endif
}

// acc = a b: the first product of a fresh accumulator, with the inline constant 0 as the addend
// (no v_mov_b64 to clear the accumulator first)
EON_HD void mul29_vv(uint64_t& acc, uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(acc), "=s"(c) : "v"(a), "v"(b));
#else
    acc = (uint64_t)a * b;
#endif
}

EON_HD void mul29_vs(uint64_t& acc, uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(acc), "=s"(c) : "v"(a), "s"(b));
#else
    acc = (uint64_t)a * b;
#endif
}

// One column's terms: acc (= 0 when FIRST) + sum va[i] vb[i] + sum sa[i] sb[i], sb wave-uniform
// (SGPRs).  With EON_MAD_BLOCKS (default) the terms go out as one asm statement per up to 9 + 9
// of them (mad_blocks.h): the compiler puts an s_nop between any two adjacent asm statements,
// which cost 11-16 % of a chain's throughput as one statement per term
// (profiles/r05/s11/ubench_mad_nop.txt).  Without it, one statement per term (mad29_vv / _vs).
#ifndef EON_MAD_BLOCKS
#define EON_MAD_BLOCKS 1
#endif
template <int NV, int NS, bool FIRST = false>
EON_HD void madcol(uint64_t& acc, const uint32_t* va, const uint32_t* vb, const uint32_t* sa,
                   const uint32_t* sb) {
#if defined(__HIP_DEVICE_COMPILE__) && EON_MAD_BLOCKS
    if constexpr (NV > 9) {
        MadAsm<9, 0, FIRST>::run(acc, va, vb, sa, sb);
        madcol<NV - 9, NS, false>(acc, va + 9, vb + 9, sa, sb);
    } else if constexpr (NS > 9) {
        madcol<NV, 9, FIRST>(acc, va, vb, sa, sb);
        madcol<0, NS - 9, false>(acc, va, vb, sa + 9, sb + 9);
    } else if constexpr (NV + NS > 0) {
        MadAsm<NV, NS, FIRST>::run(acc, va, vb, sa, sb);
    }
#else
#pragma unroll
    for (int i = 0; i < NV; i++) {
        if (FIRST && i == 0)
            mul29_vv(acc, va[0], vb[0]);
        else
            mad29_vv(acc, va[i], vb[i]);
    }
#pragma unroll
    for (int i = 0; i < NS; i++) {
        if (FIRST && NV == 0 && i == 0)
            mul29_vs(acc, sa[0], sb[0]);
        else
            mad29_vs(acc, sa[i], sb[i]);
    }
#endif
}

// f(integral_constant<int, I>) for I = B .. E - 1: column loops whose term counts are template
// arguments of madcol
template <int B, int E, class F>
EON_HD void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}
#define EON_K(kc) decltype(kc)::value

// Montgomery product a b 2^-261 mod p (product scanning; see the header comment for the bounds)
//
// The reduction multipliers m_0..m_(U-1) are left unmasked (32 bits instead of 29: one v_and
// fewer each).  m_k only has to be -column * p^-1 modulo 2^29, so the reduction stays exact; the
// extra multiples of p sit below 2^(32 + 29 (U - 1)), i.e. below 2^235 p for U = 8, so the output
// stays < 2p whenever a b < 0.99 p 2^261 (2^261 = 169.3 p; e.g. both values < 12p -- the widest
// product of the curve formulas, P^2 < 100 p^2, is 0.59 p 2^261).  With the actual limbs of p and
// r the widest column sum is 0.88 (Fq) / 0.93 (Fr) of 2^64 for operands with limbs < 2^30
// (0.50 / 0.55 for normalised ones); U = 9 would add 8p to the output bound.
template <class M, int U = 8>
EON_HD F29 mul29(const F29& a, const F29& b) {
    uint32_t m[9];
    F29 r;
    uint64_t acc;
    static_for<0, 9>([&](auto kc) {
        constexpr int k = EON_K(kc);
        uint32_t va[k + 1], vb[k + 1], sa[k + 1], sb[k + 1];
#pragma unroll
        for (int i = 0; i <= k; i++) {
            va[i] = a.l[i];
            vb[i] = b.l[k - i];
        }
#pragma unroll
        for (int i = 0; i < k; i++) {
            sa[i] = m[i];
            sb[i] = R29<M>::P[k - i];
        }
        madcol<k + 1, k, k == 0>(acc, va, vb, sa, sb);
        m[k] = k < U ? (uint32_t)acc * R29<M>::INV : ((uint32_t)acc * R29<M>::INV) & M29;
        mad29_vs(acc, m[k], R29<M>::P[0]);
        acc >>= 29;
    });
    static_for<9, 17>([&](auto kc) {
        constexpr int k = EON_K(kc), n = 17 - k;
        uint32_t va[n], vb[n], sa[n], sb[n];
#pragma unroll
        for (int i = k - 8; i < 9; i++) {
            va[i - (k - 8)] = a.l[i];
            vb[i - (k - 8)] = b.l[k - i];
            sa[i - (k - 8)] = m[i];
            sb[i - (k - 8)] = R29<M>::P[k - i];
        }
        madcol<n, n>(acc, va, vb, sa, sb);
        r.l[k - 9] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    r.l[8] = (uint32_t)acc;
    return r;
}

// N independent Montgomery products r[c] = a[c] b[c] 2^-261 (mul29's contract each), their
// multiply-add chains interleaved column by column: for latency-bound code (a wave alone on its
// SIMD: the few-group MSM reduction's segment sums and trees), where one product's dependent
// chain leaves the issue slots of the others free.  Same results as N calls of mul29.
template <class M, int N>
EON_HD void mul29_n(const F29 (&a)[N], const F29 (&b)[N], F29 (&r)[N]) {
    uint32_t m[N][9];
    uint64_t acc[N];
    static_for<0, 9>([&](auto kc) {
        constexpr int k = EON_K(kc);
#pragma unroll
        for (int c = 0; c < N; c++) {
            uint32_t va[k + 1], vb[k + 1], sa[k + 1], sb[k + 1];
#pragma unroll
            for (int i = 0; i <= k; i++) {
                va[i] = a[c].l[i];
                vb[i] = b[c].l[k - i];
            }
#pragma unroll
            for (int i = 0; i < k; i++) {
                sa[i] = m[c][i];
                sb[i] = R29<M>::P[k - i];
            }
            madcol<k + 1, k, k == 0>(acc[c], va, vb, sa, sb);
        }
#pragma unroll
        for (int c = 0; c < N; c++) {
            m[c][k] = k < 8 ? (uint32_t)acc[c] * R29<M>::INV : ((uint32_t)acc[c] * R29<M>::INV) & M29;
            mad29_vs(acc[c], m[c][k], R29<M>::P[0]);
            acc[c] >>= 29;
        }
    });
    static_for<9, 17>([&](auto kc) {
        constexpr int k = EON_K(kc), n = 17 - k;
#pragma unroll
        for (int c = 0; c < N; c++) {
            uint32_t va[n], vb[n], sa[n], sb[n];
#pragma unroll
            for (int i = k - 8; i < 9; i++) {
                va[i - (k - 8)] = a[c].l[i];
                vb[i - (k - 8)] = b[c].l[k - i];
                sa[i - (k - 8)] = m[c][i];
                sb[i - (k - 8)] = R29<M>::P[k - i];
            }
            madcol<n, n>(acc[c], va, vb, sa, sb);
        }
#pragma unroll
        for (int c = 0; c < N; c++) {
            r[c].l[k - 9] = (uint32_t)acc[c] & M29;
            acc[c] >>= 29;
        }
    });
#pragma unroll
    for (int c = 0; c < N; c++) r[c].l[8] = (uint32_t)acc[c];
}

// y w mod p for a constant w < p with its Shoup quotient wq = floor(w 2^261 / p), both as
// normalised 29-bit limbs (the NTT's twiddles): q = floor(y wq / 2^261) from the product's columns
// 7..16 -- the columns below 7 sum to less than 2^235, so the estimate is q or q - 1 -- then
// r = y w - q p modulo 2^261, as y w + q (2^261 - p) with positive limbs only.  q <= y w / p and
// q >= y w / p - y / 2^261 - 2, so r is in [0, 3p) for any normalised y < 2^261, exact modulo
// 2^261.  143 multiply-adds and no Montgomery multipliers (mul29: 162 + 9 v_mul_lo).  The product
// is not divided by any power of two, so y in Montgomery form gives y w in Montgomery form for
// the plain integer w.
template <class M>
EON_HD F29 mul29_shoup(const F29& y, const F29& w, const F29& wq) {
    uint64_t acc;
    uint32_t q[9];
    {
        uint32_t vb[8];
#pragma unroll
        for (int i = 0; i <= 7; i++) vb[i] = wq.l[7 - i];
        madcol<8, 0, true>(acc, y.l, vb, nullptr, nullptr);
        acc >>= 29;
    }
    {
        uint32_t vb[9];
#pragma unroll
        for (int i = 0; i <= 8; i++) vb[i] = wq.l[8 - i];
        madcol<9, 0>(acc, y.l, vb, nullptr, nullptr);
        acc >>= 29;
    }
    static_for<9, 17>([&](auto kc) {
        constexpr int k = EON_K(kc), n = 17 - k;
        uint32_t vb[n];
#pragma unroll
        for (int i = k - 8; i < 9; i++) vb[i - (k - 8)] = wq.l[k - i];
        madcol<n, 0>(acc, y.l + (k - 8), vb, nullptr, nullptr);
        q[k - 9] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    q[8] = (uint32_t)acc;  // q < y < 2^261
    F29 r;
    static_for<0, 9>([&](auto kc) {
        // column k: (k + 1) products of each half, at most 18 products < 2^58 (< 2^62.2 with carry)
        constexpr int k = EON_K(kc);
        uint32_t vb[k + 1], sb[k + 1];
#pragma unroll
        for (int i = 0; i <= k; i++) {
            vb[i] = w.l[k - i];
            sb[i] = R29<M>::NEGP261[k - i];
        }
        madcol<k + 1, k + 1, k == 0>(acc, y.l, vb, q, sb);
        r.l[k] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    return r;
}

// mul29_shoup with w and wq wave-uniform (a kernel argument, an evaluation point): their limbs are
// the SGPR operand of every multiply-add, so the pair costs no VGPRs.  Same contract and result.
template <class M>
EON_HD F29 mul29_shoup_u(const F29& y, const F29& w, const F29& wq) {
    uint64_t acc;
    uint32_t q[9];
    {
        uint32_t sb[8];
#pragma unroll
        for (int i = 0; i <= 7; i++) sb[i] = wq.l[7 - i];
        madcol<0, 8, true>(acc, nullptr, nullptr, y.l, sb);
        acc >>= 29;
    }
    {
        uint32_t sb[9];
#pragma unroll
        for (int i = 0; i <= 8; i++) sb[i] = wq.l[8 - i];
        madcol<0, 9>(acc, nullptr, nullptr, y.l, sb);
        acc >>= 29;
    }
    static_for<9, 17>([&](auto kc) {
        constexpr int k = EON_K(kc), n = 17 - k;
        uint32_t sb[n];
#pragma unroll
        for (int i = k - 8; i < 9; i++) sb[i - (k - 8)] = wq.l[k - i];
        madcol<0, n>(acc, nullptr, nullptr, y.l + (k - 8), sb);
        q[k - 9] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    q[8] = (uint32_t)acc;
    F29 r;
    static_for<0, 9>([&](auto kc) {
        constexpr int k = EON_K(kc);
        uint32_t sa[2 * k + 2], sb[2 * k + 2];
#pragma unroll
        for (int i = 0; i <= k; i++) {
            sa[i] = y.l[i];
            sb[i] = w.l[k - i];
            sa[k + 1 + i] = q[i];
            sb[k + 1 + i] = R29<M>::NEGP261[k - i];
        }
        madcol<0, 2 * k + 2, k == 0>(acc, nullptr, nullptr, sa, sb);
        r.l[k] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    return r;
}

// The twiddle pair of mul29_shoup from T = w 2^261 mod p (canonical; the Montgomery form of 32 w,
// which is how the twiddle tables are first built): w = T 2^-261 mod p (a product by the integer
// 1, canonicalised) and wq = floor(w 2^261 / p) = (w 2^261 - T) / p, an exact quotient, i.e.
// (2^261 - T) p^-1 mod 2^261 (a low-half product).
template <class M>
EON_HD void shoup_pair29(const F29& T, F29& w, F29& wq) {
    F29 one;
#pragma unroll
    for (int i = 0; i < 9; i++) one.l[i] = i == 0 ? 1u : 0u;
    w = canon29<M>(mul29<M>(T, one));
    uint32_t n[9];
    uint32_t c = 1;
#pragma unroll
    for (int i = 0; i < 9; i++) {  // 2^261 - T = (2^261 - 1 - T) + 1
        const uint32_t v = (M29 - T.l[i]) + c;
        n[i] = v & M29;
        c = v >> 29;
    }
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
#pragma unroll
        for (int i = 0; i <= k; i++) acc += (uint64_t)n[i] * R29<M>::PINV261[k - i];
        wq.l[k] = (uint32_t)acc & M29;
        acc >>= 29;
    }
}

// a - q p with q = floor(a_8 / (p_8 + 1)) (a normalised, any value < 2^261): q p <= a_8 2^232
// <= a, and a - q p < p + (q + 1) 2^232 < 2p (q <= 169 for Fr, 2^232 < p / 3.1e6) -- one
// small-quotient step instead of a chain of conditional subtractions, so lazy values can grow
template <class M>
EON_HD F29 reduce_top29(const F29& a) {
    const uint32_t q = a.l[8] / (R29<M>::P[8] + 1);
    F29 r;
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int64_t t = (int64_t)a.l[i] - (int64_t)q * R29<M>::P[i] + c;
        r.l[i] = (uint32_t)t & M29;
        c = t >> 29;  // arithmetic
    }
    return r;
}

// canonical x 2^256 (the radix-2^32 ABI form, < p) -> x 2^261 in 29-bit limbs: the bits of
// 32 (x 2^256) re-split at offset -5, an integer < 2^259 < 32p (shl5_raw, normalised limbs), or
// brought below 2p by one reduce_top29 step (shl5_to261) -- about a quarter of the Montgomery
// product by 2^266 that to261 costs
template <class M>
EON_HD F29 shl5_raw(const Fe<M>& a) {
    F29 r;
    r.l[0] = (a.v[0] << 5) & M29;
#pragma unroll
    for (int i = 1; i < 9; i++) {
        const int bit = 29 * i - 5, w = bit >> 5, s = bit & 31;
        uint64_t v = a.v[w];
        if (w + 1 < 8) v |= (uint64_t)a.v[w + 1] << 32;
        r.l[i] = (uint32_t)(v >> s) & M29;
    }
    return r;
}

template <class M>
EON_HD F29 shl5_to261(const Fe<M>& a) {
    return reduce_top29<M>(shl5_raw(a));
}

// a^2 2^-261 mod p (limbs < 2^30, a^2 < 0.99 p 2^261, as mul29): each column's cross products
// once, summed apart and doubled by a shift (45 instead of 81 limb products; cross sums < 2^62)
//
// EON_SQR_DOUBLED (default): the cross products are taken against a doubled copy 2 a_i (i < 8,
// limbs < 2^31) straight into the column's accumulator -- 8 limb doublings instead of one
// shift-and-add of a separate cross sum per column (15); the column sums are the same numbers.
#ifndef EON_SQR_DOUBLED
#define EON_SQR_DOUBLED 1
#endif
template <class M, int U = 8>
EON_HD F29 sqr29(const F29& a) {
    uint32_t m[9];
    F29 r;
    uint64_t acc;
#if EON_SQR_DOUBLED
    uint32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = a.l[i] << 1;
    static_for<0, 9>([&](auto kc) {
        // column k: 2 a_i a_(k-i) for i < k - i, a_(k/2)^2 (k even), m_i p_(k-i)
        constexpr int k = EON_K(kc), nc = (k + 1) / 2, nq = (k & 1) ? 0 : 1, nv = nc + nq;
        uint32_t va[nv], vb[nv], sa[k + 1], sb[k + 1];
#pragma unroll
        for (int i = 0; i < nc; i++) {
            va[i] = d[i];
            vb[i] = a.l[k - i];
        }
        if constexpr (nq) {
            va[nc] = a.l[k / 2];
            vb[nc] = a.l[k / 2];
        }
#pragma unroll
        for (int i = 0; i < k; i++) {
            sa[i] = m[i];
            sb[i] = R29<M>::P[k - i];
        }
        madcol<nv, k, k == 0>(acc, va, vb, sa, sb);
        m[k] = k < U ? (uint32_t)acc * R29<M>::INV : ((uint32_t)acc * R29<M>::INV) & M29;
        mad29_vs(acc, m[k], R29<M>::P[0]);
        acc >>= 29;
    });
    static_for<9, 17>([&](auto kc) {
        // cross pairs (i, k - i), k - 8 <= i < k - i; the smaller index is < 8
        constexpr int k = EON_K(kc), nc = (k - 1) / 2 - (k - 8) + 1, nq = (k & 1) ? 0 : 1, n = 17 - k;
        constexpr int ncp = nc > 0 ? nc : 0, nv = ncp + nq;
        uint32_t va[nv > 0 ? nv : 1], vb[nv > 0 ? nv : 1], sa[n], sb[n];
#pragma unroll
        for (int i = 0; i < ncp; i++) {
            va[i] = d[k - 8 + i];
            vb[i] = a.l[8 - i];
        }
        if constexpr (nq) {
            va[ncp] = a.l[k / 2];
            vb[ncp] = a.l[k / 2];
        }
#pragma unroll
        for (int i = k - 8; i < 9; i++) {
            sa[i - (k - 8)] = m[i];
            sb[i - (k - 8)] = R29<M>::P[k - i];
        }
        madcol<nv, n>(acc, va, vb, sa, sb);
        r.l[k - 9] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    r.l[8] = (uint32_t)acc;
    return r;
#else
    static_for<0, 9>([&](auto kc) {
        constexpr int k = EON_K(kc), nc = (k + 1) / 2, nq = (k & 1) ? 0 : 1;
        if constexpr (nc > 0) {
            uint64_t cross;
            uint32_t va[nc], vb[nc];
#pragma unroll
            for (int i = 0; i < nc; i++) {
                va[i] = a.l[i];
                vb[i] = a.l[k - i];
            }
            madcol<nc, 0, true>(cross, va, vb, nullptr, nullptr);
            acc += cross << 1;
        }
        uint32_t va[1] = {a.l[k / 2]}, sa[k + 1], sb[k + 1];
#pragma unroll
        for (int i = 0; i < k; i++) {
            sa[i] = m[i];
            sb[i] = R29<M>::P[k - i];
        }
        madcol<nq, k, k == 0>(acc, va, va, sa, sb);
        m[k] = k < U ? (uint32_t)acc * R29<M>::INV : ((uint32_t)acc * R29<M>::INV) & M29;
        mad29_vs(acc, m[k], R29<M>::P[0]);
        acc >>= 29;
    });
    static_for<9, 17>([&](auto kc) {
        constexpr int k = EON_K(kc), nc = (k - 1) / 2 - (k - 8) + 1, nq = (k & 1) ? 0 : 1, n = 17 - k;
        if constexpr (nc > 0) {
            uint64_t cross;
            uint32_t va[nc], vb[nc];
#pragma unroll
            for (int i = 0; i < nc; i++) {
                va[i] = a.l[k - 8 + i];
                vb[i] = a.l[8 - i];
            }
            madcol<nc, 0, true>(cross, va, vb, nullptr, nullptr);
            acc += cross << 1;
        }
        uint32_t va[1] = {a.l[k / 2]}, sa[n], sb[n];
#pragma unroll
        for (int i = k - 8; i < 9; i++) {
            sa[i - (k - 8)] = m[i];
            sb[i - (k - 8)] = R29<M>::P[k - i];
        }
        madcol<nq, n>(acc, va, va, sa, sb);
        r.l[k - 9] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    r.l[8] = (uint32_t)acc;
    return r;
#endif
}

// (a b + c d) 2^-261 mod p with one reduction: 27 terms per column, so a, c and d must be
// normalised (limbs < 2^29) and b's limbs < 2^31 (a sub29_lazy output); a b + c d < 0.99 p 2^261
// gives an output < 2p.  Six unmasked reduction multipliers (see mul29): widest column 0.91 of
// 2^64 with such a b.
template <class M>
EON_HD F29 mul29_sum2(const F29& a, const F29& b, const F29& c, const F29& d) {
    uint32_t m[9];
    F29 r;
    uint64_t acc;
    static_for<0, 9>([&](auto kc) {
        constexpr int k = EON_K(kc);
        uint32_t va[2 * k + 2], vb[2 * k + 2], sa[k + 1], sb[k + 1];
#pragma unroll
        for (int i = 0; i <= k; i++) {
            va[i] = a.l[i];
            vb[i] = b.l[k - i];
            va[k + 1 + i] = c.l[i];
            vb[k + 1 + i] = d.l[k - i];
        }
#pragma unroll
        for (int i = 0; i < k; i++) {
            sa[i] = m[i];
            sb[i] = R29<M>::P[k - i];
        }
        madcol<2 * k + 2, k, k == 0>(acc, va, vb, sa, sb);
        m[k] = k < 6 ? (uint32_t)acc * R29<M>::INV : ((uint32_t)acc * R29<M>::INV) & M29;
        mad29_vs(acc, m[k], R29<M>::P[0]);
        acc >>= 29;
    });
    static_for<9, 17>([&](auto kc) {
        constexpr int k = EON_K(kc), n = 17 - k;
        uint32_t va[2 * n], vb[2 * n], sa[n], sb[n];
#pragma unroll
        for (int i = k - 8; i < 9; i++) {
            const int j = i - (k - 8);
            va[j] = a.l[i];
            vb[j] = b.l[k - i];
            va[n + j] = c.l[i];
            vb[n + j] = d.l[k - i];
            sa[j] = m[i];
            sb[j] = R29<M>::P[k - i];
        }
        madcol<2 * n, n>(acc, va, vb, sa, sb);
        r.l[k - 9] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    r.l[8] = (uint32_t)acc;
    return r;
}

// mul29_sum2 with a and c wave-uniform (the Horner powers of a quotient fold): their limbs are
// read as the SGPR operand of each multiply-add, so the pair costs no VGPRs.  The caller makes
// them uniform (uniform29).  Same contract and result as mul29_sum2.
template <class M>
EON_HD F29 mul29_sum2_u(const F29& a, const F29& b, const F29& c, const F29& d) {
    uint32_t m[9];
    F29 r;
    uint64_t acc;
    static_for<0, 9>([&](auto kc) {
        constexpr int k = EON_K(kc);
        uint32_t sa[3 * k + 2], sb[3 * k + 2];
#pragma unroll
        for (int i = 0; i <= k; i++) {
            sa[i] = b.l[k - i];
            sb[i] = a.l[i];
            sa[k + 1 + i] = d.l[k - i];
            sb[k + 1 + i] = c.l[i];
        }
#pragma unroll
        for (int i = 0; i < k; i++) {
            sa[2 * k + 2 + i] = m[i];
            sb[2 * k + 2 + i] = R29<M>::P[k - i];
        }
        madcol<0, 3 * k + 2, k == 0>(acc, nullptr, nullptr, sa, sb);
        m[k] = k < 6 ? (uint32_t)acc * R29<M>::INV : ((uint32_t)acc * R29<M>::INV) & M29;
        mad29_vs(acc, m[k], R29<M>::P[0]);
        acc >>= 29;
    });
    static_for<9, 17>([&](auto kc) {
        constexpr int k = EON_K(kc), n = 17 - k;
        uint32_t sa[3 * n], sb[3 * n];
#pragma unroll
        for (int i = k - 8; i < 9; i++) {
            const int j = i - (k - 8);
            sa[j] = b.l[k - i];
            sb[j] = a.l[i];
            sa[n + j] = d.l[k - i];
            sb[n + j] = c.l[i];
            sa[2 * n + j] = m[i];
            sb[2 * n + j] = R29<M>::P[k - i];
        }
        madcol<0, 3 * n>(acc, nullptr, nullptr, sa, sb);
        r.l[k - 9] = (uint32_t)acc & M29;
        acc >>= 29;
    });
    r.l[8] = (uint32_t)acc;
    return r;
}

// a value the whole wave holds alike, marked uniform limb by limb (SGPRs)
EON_HD F29 uniform29(const F29& a) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) {
#ifdef __HIP_DEVICE_COMPILE__
        r.l[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.l[i]);
#else
        r.l[i] = a.l[i];
#endif
    }
    return r;
}

// Whole products as one asm statement each (prod_asm.h, generated by tools/gen_prod_asm.py): the
// same column schedule and results as mul29 / sqr29 / mul29_sum2, without the wait state hipcc
// puts after every asm statement (one per column above).  EON_PRODUCT_ASM=0 routes the *_x
// entry points to the column-block versions (A/B).
#ifndef EON_PRODUCT_ASM
#define EON_PRODUCT_ASM 1
#endif
}  // namespace eon
#include "prod_asm.h"
namespace eon {
template <class M>
EON_HD F29 mul29_x(const F29& a, const F29& b) {
#if defined(__HIP_DEVICE_COMPILE__) && EON_PRODUCT_ASM
    return mul29_asm<M>(a, b);
#else
    return mul29<M>(a, b);
#endif
}
template <class M>
EON_HD F29 sqr29_x(const F29& a) {
#if defined(__HIP_DEVICE_COMPILE__) && EON_PRODUCT_ASM && EON_SQR_DOUBLED
    return sqr29_asm<M>(a);
#else
    return sqr29<M>(a);
#endif
}
template <class M>
EON_HD F29 mul29_sum2_x(const F29& a, const F29& b, const F29& c, const F29& d) {
#if defined(__HIP_DEVICE_COMPILE__) && EON_PRODUCT_ASM
    return mul29_sum2_asm<M>(a, b, c, d);
#else
    return mul29_sum2<M>(a, b, c, d);
#endif
}
// in place: a = a b, c = a b + c d (a loop-carried accumulator updated without a register copy)
template <class M>
EON_HD void mul29_ip(F29& a, const F29& b) {
#if defined(__HIP_DEVICE_COMPILE__) && EON_PRODUCT_ASM
    mul29_asm_ip<M>(a, b);
#else
    a = mul29<M>(a, b);
#endif
}
template <class M>
EON_HD void mul29_sum2_ip(const F29& a, const F29& b, F29& c, const F29& d) {
#if defined(__HIP_DEVICE_COMPILE__) && EON_PRODUCT_ASM
    mul29_sum2_asm_ip<M>(a, b, c, d);
#else
    c = mul29_sum2<M>(a, b, c, d);
#endif
}

// ---- compile-time overflow guard for the unmasked Montgomery multipliers --------------------------
// Worst case of every 64-bit column accumulator of mul29 / sqr29 / mul29_sum2: every operand limb
// at its contract maximum (`prod_max` = the operand products one column position can add), every
// unmasked multiplier m_k at 2^32 - 1 (masked ones at 2^29 - 1), the actual limbs of the modulus,
// and the carry in from the previous column at its own worst case.
template <class M>
constexpr bool columns_fit_u64(unsigned __int128 prod_max, int unmasked) {
    unsigned __int128 carry = 0;
    for (int k = 0; k < 17; k++) {
        unsigned __int128 col = carry;
        for (int i = 0; i < 9; i++) {
            const int j = k - i;
            if (j < 0 || j > 8) continue;
            col += prod_max;
            const unsigned __int128 m_max = i < unmasked ? 0xffffffffu : M29;
            col += m_max * R29<M>::P[j];  // reduction products m_i p_j
        }
        if (col >= ((unsigned __int128)1 << 64)) return false;
        carry = col >> 29;
    }
    return true;
}
constexpr unsigned __int128 L29 = M29, L30 = (1u << 30) - 1, L31 = (1u << 31) - 1;
// mul29 / sqr29 (U = 8 unmasked multipliers), operand limbs < 2^30 (add29_lazy outputs):
// 0.876 (Fq) / 0.93 (Fr) of 2^64
static_assert(columns_fit_u64<FqP>(L30 * L30, 8), "mul29<Fq> column overflow");
static_assert(columns_fit_u64<FrP>(L30 * L30, 8), "mul29<Fr> column overflow");
// mul29_sum2: a, c, d normalised, b < 2^31 (a sub29_lazy output), 6 unmasked multipliers
static_assert(columns_fit_u64<FqP>(L29 * L31 + L29 * L29, 6), "mul29_sum2<Fq> column overflow");
static_assert(columns_fit_u64<FrP>(L29 * L31 + L29 * L29, 6), "mul29_sum2<Fr> column overflow");

// mul29_shoup's columns for y limbs < ly: the quotient columns 7..16 of y wq (wq normalised, the
// low columns' carry into column 7 included) and the remainder columns 0..8 of y w + q (2^261 - p)
template <class M>
constexpr bool shoup_columns_fit_u64(unsigned __int128 ly) {
    unsigned __int128 carry = 0;
    for (int k = 0; k < 17; k++) {
        unsigned __int128 col = carry;
        for (int i = 0; i < 9; i++)
            if (k - i >= 0 && k - i <= 8) col += ly * M29;
        if (col >= ((unsigned __int128)1 << 64)) return false;
        carry = col >> 29;
    }
    carry = 0;
    for (int k = 0; k < 9; k++) {
        unsigned __int128 col = carry;
        for (int i = 0; i <= k; i++) col += ly * M29 + (unsigned __int128)M29 * R29<M>::NEGP261[k - i];
        if (col >= ((unsigned __int128)1 << 64)) return false;
        carry = col >> 29;
    }
    return true;
}
// the DIT NTT normalises every third stage: two carry-free stages take limbs from < 2^29 to
// < 1.5 2^30 (x + t, x + (4p borrowed) - t) and then < 2.5 2^30, the widest Shoup input
static_assert(shoup_columns_fit_u64<FrP>((unsigned __int128)5 << 29), "mul29_shoup<Fr> column overflow");

// Same with the product and reduction terms of a column in two accumulators (shorter dependency
// chains), merged once per column.
template <class M>
EON_HD F29 mul29_2acc(const F29& a, const F29& b) {
    uint32_t m[9];
    F29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        uint64_t pa = 0, pb = 0;
#pragma unroll
        for (int i = 0; i <= k; i += 2) pa += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
        for (int i = 1; i <= k; i += 2) pb += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
        for (int i = 0; i < k; i++) pb += (uint64_t)m[i] * R29<M>::P[k - i];
        acc += pa + pb;
        m[k] = ((uint32_t)acc * R29<M>::INV) & M29;
        acc += (uint64_t)m[k] * R29<M>::P[0];
        acc >>= 29;
    }
#pragma unroll
    for (int k = 9; k < 17; k++) {
        uint64_t pa = 0, pb = 0;
#pragma unroll
        for (int i = k - 8; i < 9; i++) {
            pa += (uint64_t)a.l[i] * b.l[k - i];
            pb += (uint64_t)m[i] * R29<M>::P[k - i];
        }
        acc += pa + pb;
        r.l[k - 9] = (uint32_t)acc & M29;
        acc >>= 29;
    }
    r.l[8] = (uint32_t)acc;
    return r;
}

}  // namespace eon
