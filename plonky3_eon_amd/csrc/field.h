// BN254 prime-field arithmetic for gfx950, 8 x 32-bit limbs in VGPRs.
//
// Element layout is the reference's: a 256-bit little-endian Montgomery residue a*2^256 mod m,
// canonical (< m).  `Fr` is bit-identical to p3_bn254::Fr ([u64;4] LE, bn254/src/field.rs:98-105);
// limb i of the u64 view is v[2i] | v[2i+1] << 32.  `Fq` is the G1 base field (halo2curves'
// layout, R = 2^256 mod q).
//
// Multiplication is the "no-carry" CIOS Montgomery product (valid because the top limb of both
// moduli is < 2^31 - 1), computed as 32x32->64 multiply-adds (v_mad_u64_u32).  The reference uses
// 64-bit interleaved reduction with mu = p^-1 and a subtraction (bn254/src/helpers.rs:168-205);
// both return the unique canonical representative of a*b*2^-256 mod m, so results are bit-exact.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define EON_HD __host__ __device__ __forceinline__

namespace eon {

struct FrP {
    static constexpr uint32_t P[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                      0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    static constexpr uint32_t ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                        0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
    static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                       0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
    static constexpr uint32_t INV = 0xefffffffu;  // -m^-1 mod 2^32
};

struct FqP {
    static constexpr uint32_t P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                      0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    static constexpr uint32_t ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                        0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
    static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                       0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
    static constexpr uint32_t INV = 0xe4866389u;
};

template <class M>
struct alignas(16) Fe {
    uint32_t v[8];

    EON_HD static Fe zero() {
        Fe r;
#pragma unroll
        for (int i = 0; i < 8; i++) r.v[i] = 0;
        return r;
    }
    EON_HD static Fe one() {
        Fe r;
#pragma unroll
        for (int i = 0; i < 8; i++) r.v[i] = M::ONE[i];
        return r;
    }
    EON_HD bool is_zero() const {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) acc |= v[i];
        return acc == 0;
    }
    EON_HD bool operator==(const Fe& o) const {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) acc |= v[i] ^ o.v[i];
        return acc == 0;
    }
    EON_HD bool operator!=(const Fe& o) const { return !(*this == o); }
};

using Fr = Fe<FrP>;
using Fq = Fe<FqP>;

// r = a + b mod m   (a, b canonical; a + b < 2^255 so no 256-bit overflow)
template <class M>
EON_HD Fe<M> add(const Fe<M>& a, const Fe<M>& b) {
    Fe<M> s, d;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)a.v[i] + b.v[i];
        s.v[i] = (uint32_t)c;
        c >>= 32;
    }
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        br += (int64_t)s.v[i] - M::P[i];
        d.v[i] = (uint32_t)br;
        br >>= 32;  // arithmetic shift: 0 or -1
    }
    return br < 0 ? s : d;
}

// r = a - b mod m
template <class M>
EON_HD Fe<M> sub(const Fe<M>& a, const Fe<M>& b) {
    Fe<M> d, e;
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        br += (int64_t)a.v[i] - b.v[i];
        d.v[i] = (uint32_t)br;
        br >>= 32;
    }
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)d.v[i] + M::P[i];
        e.v[i] = (uint32_t)c;
        c >>= 32;
    }
    return br < 0 ? e : d;
}

template <class M>
EON_HD Fe<M> neg(const Fe<M>& a) {
    return sub(Fe<M>::zero(), a);
}

template <class M>
EON_HD Fe<M> dbl(const Fe<M>& a) {
    return add(a, a);
}

// Montgomery product a*b*2^-256 mod m, canonical output.  No-carry CIOS (needs m[7] < 2^31-1).
// Host-side (setup) path; the device path is mul_fips below (measured 1.27e11 vs 9.9e10
// mulmod/s on MI355X, tools/ubench_mulmod.hip).
template <class M>
EON_HD Fe<M> mul_cios(const Fe<M>& a, const Fe<M>& b) {
    uint32_t t[8];
#pragma unroll
    for (int j = 0; j < 8; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t bi = b.v[i];
        uint64_t s = (uint64_t)a.v[0] * bi + t[0];
        uint32_t A = (uint32_t)(s >> 32);
        const uint32_t t0 = (uint32_t)s;
        const uint32_t m = t0 * M::INV;
        s = (uint64_t)m * M::P[0] + t0;
        uint32_t C = (uint32_t)(s >> 32);
#pragma unroll
        for (int j = 1; j < 8; j++) {
            s = (uint64_t)a.v[j] * bi + t[j] + A;
            A = (uint32_t)(s >> 32);
            const uint32_t tj = (uint32_t)s;
            s = (uint64_t)m * M::P[j] + tj + C;
            C = (uint32_t)(s >> 32);
            t[j - 1] = (uint32_t)s;
        }
        t[7] = C + A;
    }
    Fe<M> r, d;
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r.v[i] = t[i];
        br += (int64_t)t[i] - M::P[i];
        d.v[i] = (uint32_t)br;
        br >>= 32;
    }
    return br < 0 ? r : d;
}

// Product-scanning (FIPS) Montgomery product with explicit carry chains: each 32x32 term is one
// v_mad_u64_u32 into a 64-bit column accumulator whose carry-out feeds a 32-bit overflow word via
// v_addc_co_u32.  Same result as mul() (canonical a*b*2^-256 mod m).
struct Acc96 {
    uint64_t lo;
    uint32_t ov;
};

__device__ __forceinline__ void mac(Acc96& acc, uint32_t x, uint32_t y) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc.lo), "=s"(cc) : "v"(x), "v"(y));
    asm("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(acc.ov), "=s"(cc) : "s"(cc));
}

// Same, with a wave-uniform (modulus-limb) multiplier held in an SGPR.
__device__ __forceinline__ void mac_s(Acc96& acc, uint32_t x, uint32_t y) {
    uint64_t cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc.lo), "=s"(cc) : "v"(x), "s"(y));
    asm("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(acc.ov), "=s"(cc) : "s"(cc));
}

template <class M>
__device__ __forceinline__ Fe<M> mul_fips(const Fe<M>& a, const Fe<M>& b) {
    uint32_t m[8], t[8];
    Acc96 acc{0, 0};
#pragma unroll
    for (int k = 0; k < 8; k++) {
#pragma unroll
        for (int i = 0; i <= k; i++) mac(acc, a.v[i], b.v[k - i]);
#pragma unroll
        for (int i = 0; i < k; i++) mac_s(acc, m[i], M::P[k - i]);
        m[k] = (uint32_t)acc.lo * M::INV;
        mac_s(acc, m[k], M::P[0]);
        acc.lo = (acc.lo >> 32) | ((uint64_t)acc.ov << 32);
        acc.ov = 0;
    }
#pragma unroll
    for (int k = 8; k < 15; k++) {
#pragma unroll
        for (int i = k - 7; i < 8; i++) mac(acc, a.v[i], b.v[k - i]);
#pragma unroll
        for (int i = k - 7; i < 8; i++) mac_s(acc, m[i], M::P[k - i]);
        t[k - 8] = (uint32_t)acc.lo;
        acc.lo = (acc.lo >> 32) | ((uint64_t)acc.ov << 32);
        acc.ov = 0;
    }
    t[7] = (uint32_t)acc.lo;
    Fe<M> r, d;
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r.v[i] = t[i];
        br += (int64_t)t[i] - M::P[i];
        d.v[i] = (uint32_t)br;
        br >>= 32;
    }
    return br < 0 ? r : d;
}

template <class M>
EON_HD Fe<M> mul(const Fe<M>& a, const Fe<M>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return mul_fips(a, b);
#else
    return mul_cios(a, b);
#endif
}

// A dedicated square (36 + 64 products instead of 128) measured slower than mul(a, a) on gfx950:
// the doubling adds VOP3 instructions that cost what the saved products did
// (tools/ubench_mulmod.hip, profiles/r01_ubench_isa.txt).
template <class M>
EON_HD Fe<M> sqr(const Fe<M>& a) {
    return mul(a, a);
}

// Convert a small integer to Montgomery form.
template <class M>
EON_HD Fe<M> from_u64(uint64_t x) {
    Fe<M> a = Fe<M>::zero(), r2;
    a.v[0] = (uint32_t)x;
    a.v[1] = (uint32_t)(x >> 32);
#pragma unroll
    for (int i = 0; i < 8; i++) r2.v[i] = M::R2[i];
    return mul(a, r2);
}

// Montgomery residue -> canonical integer limbs (multiply by 1).
template <class M>
EON_HD Fe<M> to_canonical(const Fe<M>& a) {
    Fe<M> one_int = Fe<M>::zero();
    one_int.v[0] = 1;
    return mul(a, one_int);
}

// base^e for a 64-bit exponent (square-and-multiply, MSB first).
template <class M>
EON_HD Fe<M> pow_u64(Fe<M> base, uint64_t e) {
    Fe<M> r = Fe<M>::one();
    for (int bit = 63; bit >= 0; bit--) {
        r = sqr(r);
        if ((e >> bit) & 1) r = mul(r, base);
    }
    return r;
}

// base^(m-2): the inverse for nonzero base (Fermat).  Host-side setup only; not a hot path.
template <class M>
EON_HD Fe<M> inverse(const Fe<M>& a) {
    uint32_t e[8];
    int64_t br = -2;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        br += (int64_t)M::P[i];
        e[i] = (uint32_t)br;
        br >>= 32;
    }
    Fe<M> r = Fe<M>::one();
    for (int w = 7; w >= 0; w--)
        for (int bit = 31; bit >= 0; bit--) {
            r = sqr(r);
            if ((e[w] >> bit) & 1) r = mul(r, a);
        }
    return r;
}

EON_HD uint32_t reverse_bits_len(uint32_t x, uint32_t bits) {
    // reference: p3_util::reverse_bits_len (util/src/lib.rs)
    return bits == 0 ? 0u : (__builtin_bitreverse32(x) >> (32 - bits));
}

// Register-pinned element loads.  A field element read through a pointer and then used by
// inlined multiplies can be "rematerialised" by the compiler -- re-loaded from memory at every use
// instead of kept in VGPRs -- which turned one 128-byte point read into ~360 L2 requests in the
// MSM combine kernels.  The empty asm makes every limb an opaque register value.
template <class M>
__device__ __forceinline__ void pin(Fe<M>& x) {
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("" : "+v"(x.v[i]));
}

template <class M>
__device__ __forceinline__ Fe<M> ld_pinned(const Fe<M>* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    Fe<M> x;
    x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
    x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
    pin(x);
    return x;
}

template <class M>
__device__ __forceinline__ void st_vec(Fe<M>* p, const Fe<M>& x) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    q[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}

}  // namespace eon

