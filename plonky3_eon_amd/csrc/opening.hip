// KZG opening bases.  KzgPcs::open commits, per (matrix, point z, column f), the synthetic-division
// quotient of f by (X - z) (kzg/src/pcs.rs:305-316, quotient_and_eval kzg/src/util.rs:100-111):
//   W = sum_{i<n-1} q_i G_i,   q_i = sum_{j>i} c_j z^(j-1-i).
// Re-associated over the coefficients c_j of f itself:
//   W = sum_{j<n} c_j H_j(z),  H_j(z) = sum_{i<j} z^(j-1-i) G_i   (H_0 = identity),
// so the witness is an MSM of the very scalars the commitment used, against bases that depend on
// z only: the digit pairs sorted for the commitment (eon_msm_g1_columns_prepare_dev) serve every
// opening point, and the per-column quotient never exists.  The bases, for z != 0:
//   P_i = z^-i G_i  (i < n-1),   S_j = sum_{i<j} P_i  (exclusive prefix sum),   H_j = z^(j-1) S_j;
// for z = 0 the quotient is the coefficient shift q_i = c_(i+1), i.e. H_j = G_(j-1).
// Cost per point: 2 variable-base scalar multiplications (double-and-add, ~3.6k Fq products) and
// two additions of the scan, then the fixed-base window table of the SRS layout (msm.hip).
#include "context.h"
#include "ec.h"
#include "ec29.h"
#include "msm.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

using namespace eon;

namespace {

// points summed per thread at each level of the prefix sum: 16 for long scans (fewer levels, the
// chip full anyway); 4 below 2^16 points (a sharded slice), where the levels' serial chains of
// additions on a few waves set the time
constexpr uint32_t SCAN = 16, SCAN_SMALL = 4;
inline uint32_t scan_chunk(uint64_t len) { return len >= (1ull << 16) ? SCAN : SCAN_SMALL; }
// scratch points of scan_exclusive over len points: len / chunk + len / chunk^2 + ... < len / (chunk - 1)
inline uint64_t scan_tmp_points(uint64_t len) { return len / (SCAN_SMALL - 1) + 64; }

// k * G for an affine G and a canonical 254-bit k (double-and-add, MSB first)
__device__ G1Xyzz smul_affine(const G1Affine& g, const Fr& k) {
    G1Xyzz acc = xyzz_inf();
    if (is_inf(g)) return acc;
    for (int w = 7; w >= 0; w--) {
        const uint32_t word = k.v[w];
        for (int bit = 31; bit >= 0; bit--) {
            acc = xyzz_dbl(acc);
            if ((word >> bit) & 1) acc = xyzz_add_affine(acc, g);
        }
    }
    return acc;
}

// out[i] = z^-i G_i for i < n - 1; out[n - 1] = identity (the scan's unused last term)
__global__ void k_open_scale(const G1Affine* g, uint64_t n, Fr zinv, G1Xyzz* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i + 1 == n) {
        st_xyzz(out + i, xyzz_inf());
        return;
    }
    const Fr k = to_canonical(pow_u64(zinv, i));
    st_xyzz(out + i, smul_affine(ld_affine(g + i), k));
}

// tot[t] = sum of a[chunk t .. chunk t + chunk)
__global__ void k_scan_totals(const G1Xyzz* a, uint64_t len, uint32_t chunk, G1Xyzz* tot) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * chunk;
    if (i0 >= len) return;
    const uint64_t i1 = i0 + chunk < len ? i0 + chunk : len;
    G1Xyzz acc = ld_xyzz(a + i0);
    for (uint64_t i = i0 + 1; i < i1; i++) acc = xyzz_add(acc, ld_xyzz(a + i));
    st_xyzz(tot + t, acc);
}

// a <- exclusive prefix sums, chunk t starting from carry[t] (the exclusive prefix of the totals)
__global__ void k_scan_apply(G1Xyzz* a, uint64_t len, uint32_t chunk, const G1Xyzz* carry) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * chunk;
    if (i0 >= len) return;
    const uint64_t i1 = i0 + chunk < len ? i0 + chunk : len;
    G1Xyzz acc = ld_xyzz(carry + t);
    for (uint64_t i = i0; i < i1; i++) {
        const G1Xyzz v = ld_xyzz(a + i);
        st_xyzz(a + i, acc);
        acc = xyzz_add(acc, v);
    }
}

// exclusive prefix sums of a short array, one thread
__global__ void k_scan_serial(G1Xyzz* a, uint64_t len) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    G1Xyzz acc = xyzz_inf();
    for (uint64_t i = 0; i < len; i++) {
        const G1Xyzz v = ld_xyzz(a + i);
        st_xyzz(a + i, acc);
        acc = xyzz_add(acc, v);
    }
}

// h[j] = z^(j-1) S_j for 0 < j < n, h[0] = identity
__global__ void k_open_finish(const G1Affine* s, uint64_t n, Fr z, G1Xyzz* h) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    if (j == 0) {
        st_xyzz(h, xyzz_inf());
        return;
    }
    const Fr k = to_canonical(pow_u64(z, j - 1));
    st_xyzz(h + j, smul_affine(ld_affine(s + j), k));
}

// z = 0: h[j] = G_(j-1), h[0] = identity
__global__ void k_open_shift(const G1Affine* g, uint64_t n, G1Affine* h) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    G1Affine r;
    if (j == 0) {
        r.x = Fq::zero();
        r.y = Fq::zero();
    } else {
        r = ld_affine(g + j - 1);
    }
    st_affine(h + j, r);
}

// ---- radix-2^29 path (r29 SRS bases with the c = 16, 16-window table) --------------------------

constexpr uint32_t TC = 16, TW = 16;  // table window bits and windows of the fast path

__device__ __forceinline__ void ld_affine29(const G1Affine* p, bool neg_y, F29& x, F29& y) {
    G1Affine a = ld_affine(p);
    if (neg_y) a.y = neg(a.y);  // p - y on the integer (29-Montgomery canonical) representation
    x = unpack29(a.x);
    y = unpack29(a.y);
}

// acc += (x, y) (affine, canonical 29-form, not the identity) with the exceptional cases
__device__ __forceinline__ void madd29_any(G1X29& acc, bool& inf, const F29& x, const F29& y) {
    if (inf) {
        acc.X = x;
        acc.Y = y;
        acc.ZZ = const29<FqP>(R29<FqP>::ONE);
        acc.ZZZ = acc.ZZ;
        inf = false;
    } else if (!madd29(acc, x, y)) {
        inf = madd29_exceptional(acc, x, y);
    }
}

// P_i = z^-i G_i from the SRS window table T_(i,w) = 2^(16 w) G_i (29-form) and its triple
// 3 T_(i,w) (bases_table3_29): k = z^-i made odd (k + 1 when even, G_i subtracted at the end) is
// recoded into 16 odd signed 16-bit digits d_w, each written in radix 4 with digits in
// {-3, -1, 1, 3} (bit pairs of (d_w + 2^16 - 1) / 2, every bit read as +-1), so that every level
// adds every window's entry +-T or +-3T (no lane divergence): 14 doublings + 128 mixed
// additions, against 15 + 256 with +-1 digits (tab3 == null keeps that radix-2 form).
// rows i = lo + t, t < cnt (a rank's slice; rows >= n - 1 are the identity).  SPLIT (a short
// slice, where a thread per row leaves SIMDs idle and the time is one row's chain): two adjacent
// lanes per row, each adding 8 of the 16 windows at every level (both double), and the odd lane's
// sum is passed to the even one by DPP and added there -- half the additions on the chain for 9 %
// more work in total.
template <bool SPLIT>
__global__ void __launch_bounds__(64) k_open_scale29(const G1Affine* tab, const G1Affine* tab3, uint64_t n,
                                                     uint64_t lo, uint64_t cnt, Fr zinv, G1Xyzz* out_slice) {
    const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t t = SPLIT ? gt >> 1 : gt;
    const uint32_t half = SPLIT ? (uint32_t)(gt & 1) : 0u;
    const uint32_t w_lo = SPLIT ? half * (TW / 2) : 0u, w_hi = SPLIT ? w_lo + TW / 2 : TW;
    if (t >= cnt) return;
    const uint64_t i = lo + t;
    G1Xyzz* out = out_slice - lo;
    if (i + 1 >= n) {
        if (half == 0) st_xyzz(out + i, xyzz_inf());
        return;
    }
    const G1Affine* row = tab + i * TW;
    {
        const G1Affine g = ld_affine(row);
        if (is_inf(g)) {  // the identity's table row is all identity
            if (half == 0) st_xyzz(out + i, xyzz_inf());
            return;
        }
    }
    Fr k = to_canonical(pow_u64(zinv, i));
    const bool even = (k.v[0] & 1) == 0;
    if (even) k.v[0] += 1;  // no carry: k even
    // odd recoding: d_w = (k mod 2^17) - 2^16, k <- (k - d_w) / 2^16; u_w = (d_w + 2^16 - 1) / 2
    uint32_t u[TW];
    uint32_t kw[9];
#pragma unroll
    for (int j = 0; j < 8; j++) kw[j] = k.v[j];
    kw[8] = 0;
#pragma unroll
    for (uint32_t w = 0; w < TW; w++) {
        int32_t d;
        if (w + 1 < TW) {
            d = (int32_t)(kw[0] & 0x1FFFFu) - 0x10000;
        } else {
            d = (int32_t)kw[0];  // the rest, odd, < 2^15
        }
        u[w] = (uint32_t)((d + 0xFFFF) >> 1);
        // k - d (d odd, |d| < 2^16), then >> 16 (exact)
        uint64_t borrow_or_carry;
        if (d >= 0) {
            uint64_t t = (uint64_t)kw[0] - (uint32_t)d;
            kw[0] = (uint32_t)t;
            borrow_or_carry = (t >> 63) & 1;  // borrow
#pragma unroll
            for (int j = 1; j < 9; j++) {
                t = (uint64_t)kw[j] - borrow_or_carry;
                kw[j] = (uint32_t)t;
                borrow_or_carry = (t >> 63) & 1;
            }
        } else {
            uint64_t t = (uint64_t)kw[0] + (uint32_t)(-d);
            kw[0] = (uint32_t)t;
            borrow_or_carry = t >> 32;
#pragma unroll
            for (int j = 1; j < 9; j++) {
                t = (uint64_t)kw[j] + borrow_or_carry;
                kw[j] = (uint32_t)t;
                borrow_or_carry = t >> 32;
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) kw[j] = (kw[j] >> 16) | (kw[j + 1] << 16);
        kw[8] >>= 16;
    }
    G1X29 acc;
    bool inf = true;
    F29 x, y;
    if (tab3) {
        const G1Affine* row3 = tab3 + i * TW;
        for (int b = (int)TC / 2 - 1; b >= 0; b--) {
            if (!inf) {
                dbl29(acc);
                dbl29(acc);
            }
            for (uint32_t w = w_lo; w < w_hi; w++) {
                // bit pair (hi, lo) of u_w: f = 2 e_hi + e_lo, e = +-1: 3 -> +3, 2 -> +1, 1 -> -1, 0 -> -3
                const uint32_t two = (u[w] >> (2 * b)) & 3u;
                const bool three = two == 3u || two == 0u;
                ld_affine29((three ? row3 : row) + w, two <= 1u, x, y);
                madd29_any(acc, inf, x, y);
            }
        }
    } else {
        for (int b = (int)TC - 1; b >= 0; b--) {
            if (!inf) dbl29(acc);
            for (uint32_t w = w_lo; w < w_hi; w++) {
                ld_affine29(row + w, ((u[w] >> b) & 1) == 0, x, y);
                madd29_any(acc, inf, x, y);
            }
        }
    }
    if (even && half == 0) {
        ld_affine29(row, true, x, y);
        madd29_any(acc, inf, x, y);
    }
    if (SPLIT) {
        // the partner lane's (odd -> even) accumulator, word by word over DPP quad_perm(1, 0, 3, 2)
        G1X29 o;
        F29* dst[4] = {&o.X, &o.Y, &o.ZZ, &o.ZZZ};
        const F29* src[4] = {&acc.X, &acc.Y, &acc.ZZ, &acc.ZZZ};
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int l = 0; l < 9; l++)
                dst[c]->l[l] = (uint32_t)__builtin_amdgcn_mov_dpp((int)src[c]->l[l], 0xB1, 0xf, 0xf, false);
        const bool o_inf = __builtin_amdgcn_mov_dpp((int)inf, 0xB1, 0xf, 0xf, false) != 0;
        if (half) return;
        acc29(acc, inf, o, o_inf);
    }
    st_xyzz(out + i, x29_to_xyzz(acc, inf));
}

// short slices (a sharded rank's rows) split each row over two lanes
inline bool scale_split(uint64_t rows) { return rows <= (1ull << 15); }
void launch_open_scale29(uint64_t rows, const G1Affine* tab, const G1Affine* tab3, uint64_t n, uint64_t lo, Fr zinv,
                         G1Xyzz* out, hipStream_t st) {
    if (scale_split(rows))
        hipLaunchKernelGGL(k_open_scale29<true>, dim3((unsigned)((2 * rows + 63) / 64)), dim3(64), 0, st, tab, tab3, n,
                           lo, rows, zinv, out);
    else
        hipLaunchKernelGGL(k_open_scale29<false>, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, st, tab, tab3, n, lo,
                           rows, zinv, out);
}

// GLV for BN254 G1: phi(x, y) = (beta x, y) = lambda (x, y) with lambda^2 + lambda + 1 = 0 mod r
// (beta a cube root of unity in Fq; the pair is fixed by phi(G) = lambda G for the generator,
// tools/glv_consts.py).  k = k1 + k2 lambda mod r with |k1|, |k2| < 2^127 from the reduced lattice
// basis (a1, b1), (a2, b2) of {(a, b) : a + b lambda = 0 mod r} (Gallant-Lambert-Vanstone):
// c1 = floor(k g1 / 2^256), c2 = floor(k g2 / 2^256) with g1 = round(b2 2^256 / r),
// g2 = round(-b1 2^256 / r); k1 = k - c1 a1 - c2 a2, k2 = -c1 b1 - c2 b2.  32-bit limbs.
namespace glv {
constexpr uint32_t G1[3] = {0xc7e0b3d7u, 0xd91d232eu, 0x2u};
constexpr uint32_t G2[5] = {0x391eb18eu, 0x7a7bd9d4u, 0xa773d2cfu, 0x4ccef014u, 0x2u};
constexpr uint32_t A1[2] = {0x94d213e3u, 0x89d32568u};                           // a1 = b2
constexpr uint32_t A2[4] = {0x1221250bu, 0xbe4e154u, 0xeeb859fdu, 0x6f4d8248u};
constexpr uint32_t NB1[4] = {0x7d4f1128u, 0x8211bbebu, 0xeeb859fcu, 0x6f4d8248u};  // -b1
// beta in 29-Montgomery form (beta 2^261 mod q)
constexpr uint32_t BETA29[9] = {0xa337995u, 0x158d1d23u, 0x189c9b98u, 0x12fa4e45u, 0x185faadcu,
                                0x176f16du,  0xeed93bau,  0x14291140u, 0xc0afeu};
}  // namespace glv

// acc -= x c or acc += x c, modulo 2^160 (5 limbs); x, c small little-endian limb arrays
template <int NX, int NC>
__device__ __forceinline__ void mac160(uint32_t acc[5], const uint32_t (&x)[NX], const uint32_t (&c)[NC], bool sub) {
    uint32_t p[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < NX; i++) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = 0; j < NC; j++) {
            if (i + j >= 5) break;
            const uint64_t t = (uint64_t)x[i] * c[j] + p[i + j] + carry;
            p[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
        if (i + NC < 5) p[i + NC] = (uint32_t)carry;
    }
    uint64_t t = 0;
    if (sub) {
        uint32_t br = 0;
#pragma unroll
        for (int i = 0; i < 5; i++) {
            t = (uint64_t)acc[i] - p[i] - br;
            acc[i] = (uint32_t)t;
            br = (uint32_t)(t >> 63);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 5; i++) {
            t = (uint64_t)acc[i] + p[i] + (t >> 32);
            acc[i] = (uint32_t)t;
        }
    }
}

// floor(k g / 2^256) for the canonical k (8 limbs) and a constant g: the product's limbs >= 8
template <int NG, int NOUT>
__device__ __forceinline__ void mul_hi256(const uint32_t (&k)[8], const uint32_t (&g)[NG], uint32_t (&out)[NOUT]) {
    uint32_t p[8 + NG];
#pragma unroll
    for (int i = 0; i < 8 + NG; i++) p[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = 0; j < NG; j++) {
            const uint64_t t = (uint64_t)k[i] * g[j] + p[i + j] + carry;
            p[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
        p[i + NG] = (uint32_t)carry;
    }
#pragma unroll
    for (int i = 0; i < NOUT; i++) out[i] = p[8 + i];
}

// |k_i| (4 limbs, < 2^127) and sign of the GLV halves of the canonical k
__device__ __forceinline__ void glv_split(const Fr& k, uint32_t (&u1)[4], bool& neg1, uint32_t (&u2)[4], bool& neg2) {
    uint32_t kk[8];
#pragma unroll
    for (int i = 0; i < 8; i++) kk[i] = k.v[i];
    uint32_t c1[3], c2[4];
    mul_hi256(kk, glv::G1, c1);
    mul_hi256(kk, glv::G2, c2);
    uint32_t k1[5] = {kk[0], kk[1], kk[2], kk[3], kk[4]}, k2[5] = {0, 0, 0, 0, 0};
    mac160(k1, c1, glv::A1, true);
    mac160(k1, c2, glv::A2, true);
    mac160(k2, c1, glv::NB1, false);
    mac160(k2, c2, glv::A1, true);  // b2 = a1
    auto mag = [](uint32_t (&v)[5], uint32_t (&u)[4], bool& neg) __attribute__((always_inline)) {
        neg = (v[4] >> 31) != 0;  // |v| < 2^127: bit 159 is the sign
        uint64_t t = neg ? 1 : 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            t += neg ? (uint64_t)(~v[i]) : (uint64_t)v[i];
            u[i] = (uint32_t)t;
            t >>= 32;
        }
    };
    mag(k1, u1, neg1);
    mag(k2, u2, neg2);
}

// odd u (< 2^128) -> 32 odd digits in [-15, 15]: nibble i of dg[] = (|d_i| - 1) / 2 | sign << 3,
// digit 31 the remaining top in [1, 15] (u = sum d_i 16^i)
__device__ __forceinline__ void recode_odd128(uint32_t (&kw)[4], uint32_t (&dg)[4]) {
#pragma unroll
    for (int q = 0; q < 4; q++) dg[q] = 0;
#pragma unroll
    for (int i = 0; i < 31; i++) {
        const int32_t d = (int32_t)(kw[0] & 31u) - 16;
        if (d >= 0) {
            uint64_t c = (uint64_t)kw[0] - (uint32_t)d;
            kw[0] = (uint32_t)c;
            uint32_t br = (uint32_t)(c >> 63);
#pragma unroll
            for (int q = 1; q < 4; q++) {
                c = (uint64_t)kw[q] - br;
                kw[q] = (uint32_t)c;
                br = (uint32_t)(c >> 63);
            }
        } else {
            uint64_t c = (uint64_t)kw[0] + (uint32_t)(-d);
            kw[0] = (uint32_t)c;
            uint32_t cy = (uint32_t)(c >> 32);
#pragma unroll
            for (int q = 1; q < 4; q++) {
                c = (uint64_t)kw[q] + cy;
                kw[q] = (uint32_t)c;
                cy = (uint32_t)(c >> 32);
            }
        }
#pragma unroll
        for (int q = 0; q < 3; q++) kw[q] = (kw[q] >> 4) | (kw[q + 1] << 28);
        kw[3] >>= 4;
        const uint32_t mag = (uint32_t)(d < 0 ? -d : d);
        dg[i >> 3] |= (((mag - 1) >> 1) | (d < 0 ? 8u : 0u)) << (4 * (i & 7));
    }
    dg[3] |= ((kw[0] - 1) >> 1) << 28;
}

// H_j = z^(j-1) S_j, then its window table 2^(16 w) H_j, w < TW, by doublings: tmp[j TW + w]
// (radix-2^32 XYZZ).  The scalar multiplication is GLV + Straus: z^(j-1) = k1 + k2 lambda, and
// k1 S + k2 phi(S) runs one doubling chain for both halves (~127 doublings instead of ~254).  Each
// half is made odd (|k| + 1 when even, that S or phi(S) subtracted at the end) and recoded into 32
// odd signed 4-bit digits, so every level adds one entry of each half: the odd multiples S, 3S, ..,
// 15S live in the thread's column of `mtab` (MTAB raw accumulators per thread, coalesced across
// threads) and phi of an entry is beta times its X.  128 doublings + 64 additions + 8 multiples,
// against 252 + 64 + 8 for the plain signed windows.
// rows j = lo + t, t < cnt; s and tmp are the slice's (rows >= n are the identity)
constexpr uint32_t MTAB = 8;

// S_j arrives as the scan left it (radix-2^32 XYZZ, no affine conversion pass)
__global__ void __launch_bounds__(64) k_open_finish29(const G1Xyzz* s_slice, uint64_t n, uint64_t lo, uint64_t cnt,
                                                      Fr z, G1Raw29* mtab, G1Xyzz* tmp_slice) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint64_t j = lo + t;
    const G1Xyzz* s = s_slice - lo;
    G1Xyzz* tmp = tmp_slice - lo * TW;
    G1X29 acc;
    bool inf = true;
    const G1Xyzz a = (j && j < n) ? ld_xyzz(s + j) : xyzz_inf();
    if (!is_inf(a)) {
        uint32_t u1[4], u2[4];
        bool neg1, neg2;
        glv_split(to_canonical(pow_u64(z, j - 1)), u1, neg1, u2, neg2);
        const bool even1 = (u1[0] & 1) == 0, even2 = (u2[0] & 1) == 0;
        u1[0] |= 1u;  // + 1 when even (no carry)
        u2[0] |= 1u;
        // the odd multiples (2m + 1) S, m < MTAB
        {
            G1X29 m;
            m.X = unpack29(to_fq261(a.X));
            m.Y = unpack29(to_fq261(a.Y));
            m.ZZ = unpack29(to_fq261(a.ZZ));
            m.ZZZ = unpack29(to_fq261(a.ZZZ));
            G1X29 two = m;
            dbl29(two);
            bool m_inf = false;
            st_raw29(mtab + t, m);
            for (uint32_t q = 1; q < MTAB; q++) {
                acc29(m, m_inf, two, false);  // S has odd order: the multiples are never O
                st_raw29(mtab + (uint64_t)q * cnt + t, m);
            }
        }
        uint32_t dg1[4], dg2[4];
        recode_odd128(u1, dg1);
        recode_odd128(u2, dg2);
        // the table entry of digit nibble `nib` of a half, times -1 when the half is negative
        auto entry = [&](uint32_t nib, bool phi, bool neg) __attribute__((always_inline)) {
            G1X29 e;
            (void)ld_raw29(mtab + (uint64_t)(nib & 7u) * cnt + t, e);
            if (phi) e.X = mul29<FqP>(e.X, const29<FqP>(glv::BETA29));
            if (((nib >> 3) & 1u) != (uint32_t)neg) e.Y = sub29<FqP, 4>(F29{}, e.Y);  // -(x, y): Y < 4p
            return e;
        };
        // digits are consumed from the top: nibble 31 of each word stream, then the stream shifts
        // left by 4 (no dynamically indexed digit array, which would live in scratch)
        auto shl4 = [](uint32_t (&d)[4]) __attribute__((always_inline)) {
            d[3] = (d[3] << 4) | (d[2] >> 28);
            d[2] = (d[2] << 4) | (d[1] >> 28);
            d[1] = (d[1] << 4) | (d[0] >> 28);
            d[0] <<= 4;
        };
        acc = entry((dg1[3] >> 28) & 7u, false, neg1);
        inf = false;
        acc29(acc, inf, entry((dg2[3] >> 28) & 7u, true, neg2), false);
        for (int i = 30; i >= 0; i--) {
            shl4(dg1);
            shl4(dg2);
            if (!inf) {
                dbl29(acc);
                dbl29(acc);
                dbl29(acc);
                dbl29(acc);
            }
#pragma unroll 1
            for (int h = 0; h < 2; h++) {  // one copy of the addition for both halves
                const uint32_t nib = (h ? dg2[3] : dg1[3]) >> 28;
                acc29(acc, inf, entry(nib, h == 1, h ? neg2 : neg1), false);
            }
        }
        // the +1 of an even half: add the digit -1 of that half (its sign folded in)
        if (even1) acc29(acc, inf, entry(8u, false, neg1), false);
        if (even2) acc29(acc, inf, entry(8u, true, neg2), false);
    }
    G1Xyzz* dst = tmp + j * TW;
    for (uint32_t w = 0; w < TW; w++) {
        st_xyzz(dst + w, x29_to_xyzz(acc, inf));
        if (!inf && w + 1 < TW)
            for (uint32_t d = 0; d < TC; d++) dbl29(acc);
    }
}

__global__ void k_set_inf(G1Xyzz* p) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st_xyzz(p, xyzz_inf());
}

// sharded scan: s[t] += sum of the slice totals of the ranks before this one
__global__ void k_add_rank_offset(G1Xyzz* s, uint64_t cnt, const G1Affine* totals, uint32_t npoints,
                                  uint32_t point, uint32_t rank) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    G1Xyzz acc = ld_xyzz(s + t);
    for (uint32_t g = 0; g < rank; g++) acc = xyzz_add_affine(acc, ld_affine(totals + (uint64_t)g * npoints + point));
    st_xyzz(s + t, acc);
}

unsigned grid_for(uint64_t threads, uint32_t block) { return (unsigned)((threads + block - 1) / block); }

// exclusive prefix sum of a[0..len) in place; tmp holds scan_tmp_points(len) points
void scan_exclusive(G1Xyzz* a, uint64_t len, G1Xyzz* tmp, hipStream_t st, uint32_t chunk = 0) {
    if (!chunk) chunk = scan_chunk(len);
    if (len <= chunk) {
        hipLaunchKernelGGL(k_scan_serial, dim3(1), dim3(1), 0, st, a, len);
        return;
    }
    const uint64_t nt = (len + chunk - 1) / chunk;
    hipLaunchKernelGGL(k_scan_totals, dim3(grid_for(nt, 64)), dim3(64), 0, st, a, len, chunk, tmp);
    scan_exclusive(tmp, nt, tmp + nt, st, chunk);
    hipLaunchKernelGGL(k_scan_apply, dim3(grid_for(nt, 64)), dim3(64), 0, st, a, len, chunk, tmp);
}

// one point's scratch, alive until its stream is synchronised; taken from and given back to the
// context's DevPool (the next proof builds the same sizes)
struct Scratch {
    DevBuf h_aff, pts, tmp, aff, table_tmp, mtab;
    DevPool* pool = nullptr;
    hipError_t take(DevBuf& b, size_t need) { return pool ? pool->take(b, need) : b.ensure(need); }
    void release() {
        for (DevBuf* b : {&h_aff, &pts, &tmp, &aff, &table_tmp, &mtab}) {
            if (pool) pool->give(*b);
            b->release();
        }
    }
};

// radix-2^29 fast path: P_i from the SRS table, one kernel for H_j and its window table
Status opening_bases_async29(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const Fr& z, hipStream_t st,
                             Scratch& sc, eon_msm_bases** out) {
    EON_HIP(sc.take(sc.pts, n * sizeof(G1Xyzz)));
    EON_HIP(sc.take(sc.tmp, scan_tmp_points(n) * sizeof(G1Xyzz)));
    EON_HIP(sc.take(sc.table_tmp, n * TW * sizeof(G1Xyzz)));
    eon_msm_bases* b = nullptr;
    EON_TRY(bases_alloc_table(ctx, n, TC, &b));
    EON_HIP(sc.take(sc.mtab, n * MTAB * sizeof(G1Raw29)));
    const G1Affine* tab3 = bases_table3_29(srs, st);  // null (radix 2) if it cannot be built
    // radix 4: 14 dbl (6M+3S) + 129 madd (8M+2S); radix 2: 15 dbl + 257 madd
    ctx->prof.begin("k_open_scale29", n * (TW * 64ull + 128ull), st, n * (tab3 ? 1416ull : 2705ull));
    launch_open_scale29(n, bases_table29(srs), tab3, n, 0ull, inverse(z), sc.pts.as<G1Xyzz>(), st);
    ctx->prof.end(st);
    scan_exclusive(sc.pts.as<G1Xyzz>(), n, sc.tmp.as<G1Xyzz>(), st);
    // GLV: 124 dbl + 64 add (12M+2S) + 8 multiples, then 240 dbl for the window table
    ctx->prof.begin("k_open_finish29", n * (128ull + TW * 128ull), st, n * 4170ull);
    hipLaunchKernelGGL(k_open_finish29, dim3(grid_for(n, 64)), dim3(64), 0, st, sc.pts.as<G1Xyzz>(), n, 0ull, n, z,
                       sc.mtab.as<G1Raw29>(), sc.table_tmp.as<G1Xyzz>());
    ctx->prof.end(st);
    hipError_t e = launch_batch_to_affine(sc.table_tmp.as<G1Xyzz>(), n * TW, bases_table_mut(b), st);
    Status s = e == hipSuccess ? bases_seal_table(b, st) : Status::err(EON_E_DEVICE, hipGetErrorString(e));
    if (s.bad()) {
        (void)hipStreamSynchronize(st);
        bases_free(b);
        return s;
    }
    *out = b;
    return Status::ok();
}

// enqueue the bases of point z on st (no host sync)
Status opening_bases_async(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const Fr& z, hipStream_t st,
                           Scratch& sc, eon_msm_bases** out) {
    if (!z.is_zero() && bases_table29(srs) && bases_window(srs) == TC && bases_windows(srs) == TW &&
        n >= 2)
        return opening_bases_async29(ctx, srs, n, z, st, sc, out);
    const G1Affine* g = bases_points(srs);
    EON_HIP(sc.take(sc.h_aff, n * sizeof(G1Affine)));
    if (z.is_zero()) {
        hipLaunchKernelGGL(k_open_shift, dim3(grid_for(n, 256)), dim3(256), 0, st, g, n, sc.h_aff.as<G1Affine>());
        EON_HIP(hipGetLastError());
    } else {
        EON_HIP(sc.take(sc.pts, n * sizeof(G1Xyzz)));
        EON_HIP(sc.take(sc.tmp, scan_tmp_points(n) * sizeof(G1Xyzz)));
        EON_HIP(sc.take(sc.aff, n * sizeof(G1Affine)));
        // algorithmic cost: 2 scalar multiplications per point, ~254 dbl (6M+3S) + ~127 madd (8M+2S)
        ctx->prof.begin("k_open_scale", n * (64ull + 128ull), st, n * 3556ull);
        hipLaunchKernelGGL(k_open_scale, dim3(grid_for(n, 64)), dim3(64), 0, st, g, n, inverse(z),
                           sc.pts.as<G1Xyzz>());
        ctx->prof.end(st);
        scan_exclusive(sc.pts.as<G1Xyzz>(), n, sc.tmp.as<G1Xyzz>(), st);
        EON_HIP(launch_batch_to_affine(sc.pts.as<G1Xyzz>(), n, sc.aff.as<G1Affine>(), st));
        ctx->prof.begin("k_open_finish", n * (64ull + 128ull), st, n * 3556ull);
        hipLaunchKernelGGL(k_open_finish, dim3(grid_for(n, 64)), dim3(64), 0, st, sc.aff.as<G1Affine>(), n, z,
                           sc.pts.as<G1Xyzz>());
        ctx->prof.end(st);
        EON_HIP(launch_batch_to_affine(sc.pts.as<G1Xyzz>(), n, sc.h_aff.as<G1Affine>(), st));
        EON_HIP(hipGetLastError());
    }
    // same window layout as the SRS, so scalars prepared against the SRS serve these bases
    return bases_create(ctx, reinterpret_cast<const eon_g1_affine*>(sc.h_aff.as<G1Affine>()), n,
                        bases_precomputed(srs) ? EON_MSM_PRECOMPUTE : 0u, true, out, bases_window(srs), st,
                        &sc.table_tmp);
}

// Sharded over the context's process group (every rank calls with the same arguments): rank g
// computes rows [g m, (g+1) m), m = ceil(n / world), of every point's bases -- P_i, the slice's
// exclusive prefix sums and total, H_j and its window table -- with two all-gathers: the slice
// totals (each rank adds those of the ranks before it) and the finished table slices.
Status opening_bases_sharded(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const std::vector<Fr>& zs,
                             eon_msm_bases** outs) {
    const eon_collective& coll = ctx->coll;
    const uint32_t world = coll.world, rank = coll.rank, np = (uint32_t)zs.size();
    const uint64_t m = (n + world - 1) / world, lo = (uint64_t)rank * m;
    hipStream_t streams[3] = {ctx->stream, ctx->side(ctx->msm_side), ctx->side(ctx->msm_side2)};
    // per point: slice points (+1 for the total), scan scratch, affine slice, table slice
    std::vector<Scratch> sc(np);
    for (auto& x : sc) x.pool = &ctx->pool;
    DevBuf totals_x, totals_a, all_totals, send, recv;
    struct Release {  // every exit: drain the streams, then the buffers go back to the pool
        std::vector<Scratch>& sc;
        DevBuf* b[5];
        DevPool& pool;
        hipStream_t* streams;
        ~Release() {
            for (int i = 0; i < 3; i++) (void)hipStreamSynchronize(streams[i]);
            for (auto& x : sc) x.release();
            for (DevBuf* x : b) pool.give(*x);
        }
    } release{sc, {&totals_x, &totals_a, &all_totals, &send, &recv}, ctx->pool, streams};
    EON_HIP(ctx->pool.take(totals_x, np * sizeof(G1Xyzz)));
    EON_HIP(ctx->pool.take(totals_a, np * sizeof(G1Affine)));
    EON_HIP(ctx->pool.take(all_totals, (uint64_t)world * np * sizeof(G1Affine)));
    const uint64_t slice_entries = m * TW;  // per point
    EON_HIP(ctx->pool.take(send, np * slice_entries * sizeof(G1Affine)));
    EON_HIP(ctx->pool.take(recv, (uint64_t)world * np * slice_entries * sizeof(G1Affine)));
    EON_HIP(hipEventRecord(ctx->msm_ev[0], ctx->stream));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side, ctx->msm_ev[0], 0));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side2, ctx->msm_ev[0], 0));
    // phase 1: P_i of the slice and its exclusive prefix sums; the total lands at index m
    for (uint32_t t = 0; t < np; t++) {
        hipStream_t st = streams[t % 3];
        EON_HIP(sc[t].take(sc[t].pts, (m + 1) * sizeof(G1Xyzz)));
        EON_HIP(sc[t].take(sc[t].tmp, scan_tmp_points(m + 1) * sizeof(G1Xyzz)));
        EON_HIP(sc[t].take(sc[t].table_tmp, slice_entries * sizeof(G1Xyzz)));
        EON_HIP(sc[t].take(sc[t].mtab, m * MTAB * sizeof(G1Raw29)));
        const G1Affine* tab3 = bases_table3_29(srs, st);  // null (radix 2) if it cannot be built
        ctx->prof.begin("k_open_scale29", m * (TW * 64ull + 128ull), st, m * (tab3 ? 1416ull : 2705ull));
        launch_open_scale29(m, bases_table29(srs), tab3, n, lo, inverse(zs[t]), sc[t].pts.as<G1Xyzz>(), st);
        ctx->prof.end(st);
        // one identity past the slice: the exclusive scan leaves the slice total there
        hipLaunchKernelGGL(k_set_inf, dim3(1), dim3(1), 0, st, sc[t].pts.as<G1Xyzz>() + m);
        scan_exclusive(sc[t].pts.as<G1Xyzz>(), m + 1, sc[t].tmp.as<G1Xyzz>(), st);
        EON_HIP(hipMemcpyAsync(totals_x.as<G1Xyzz>() + t, sc[t].pts.as<G1Xyzz>() + m, sizeof(G1Xyzz),
                               hipMemcpyDeviceToDevice, st));
        EON_HIP(hipEventRecord(ctx->msm_ev[1 + (t % 2)], st));
        EON_HIP(hipStreamWaitEvent(ctx->stream, ctx->msm_ev[1 + (t % 2)], 0));
    }
    EON_HIP(launch_batch_to_affine(totals_x.as<G1Xyzz>(), np, totals_a.as<G1Affine>(), ctx->stream));
    if (coll.all_gather(coll.user, totals_a.p, all_totals.p, np * sizeof(G1Affine), ctx->stream) != 0)
        return Status::err(EON_E_DEVICE, "collective all_gather failed (opening bases totals)");
    EON_HIP(hipEventRecord(ctx->msm_ev[0], ctx->stream));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side, ctx->msm_ev[0], 0));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side2, ctx->msm_ev[0], 0));
    // phase 2: S_j = the ranks' offset + the slice's prefix sums; H_j and its table slice
    for (uint32_t t = 0; t < np; t++) {
        hipStream_t st = streams[t % 3];
        if (rank)
            hipLaunchKernelGGL(k_add_rank_offset, dim3(grid_for(m, 64)), dim3(64), 0, st, sc[t].pts.as<G1Xyzz>(), m,
                               all_totals.as<G1Affine>(), np, t, rank);
        ctx->prof.begin("k_open_finish29", m * (128ull + TW * 128ull), st, m * 4170ull);
        hipLaunchKernelGGL(k_open_finish29, dim3(grid_for(m, 64)), dim3(64), 0, st, sc[t].pts.as<G1Xyzz>(), n, lo,
                           m, zs[t], sc[t].mtab.as<G1Raw29>(), sc[t].table_tmp.as<G1Xyzz>());
        ctx->prof.end(st);
        EON_HIP(launch_batch_to_affine(sc[t].table_tmp.as<G1Xyzz>(), slice_entries,
                                       send.as<G1Affine>() + (uint64_t)t * slice_entries, st));
        EON_HIP(hipEventRecord(ctx->msm_ev[1 + (t % 2)], st));
        EON_HIP(hipStreamWaitEvent(ctx->stream, ctx->msm_ev[1 + (t % 2)], 0));
    }
    if (coll.all_gather(coll.user, send.p, recv.p, np * slice_entries * sizeof(G1Affine), ctx->stream) != 0)
        return Status::err(EON_E_DEVICE, "collective all_gather failed (opening bases tables)");
    // phase 3: every point's table from the ranks' slices (rank order = row order), then sealed
    for (uint32_t t = 0; t < np; t++) outs[t] = nullptr;
    Status s = Status::ok();
    for (uint32_t t = 0; t < np && !s.bad(); t++) {
        s = bases_alloc_table(ctx, n, TC, outs + t);
        if (s.bad()) break;
        for (uint32_t g = 0; g < world; g++) {
            const uint64_t r0 = (uint64_t)g * m;
            if (r0 >= n) break;
            const uint64_t rows = std::min<uint64_t>(m, n - r0);
            const G1Affine* src = recv.as<G1Affine>() + ((uint64_t)g * np + t) * slice_entries;
            const hipError_t e = hipMemcpyAsync(bases_table_mut(outs[t]) + r0 * TW, src, rows * TW * sizeof(G1Affine),
                                                hipMemcpyDeviceToDevice, ctx->stream);
            if (e != hipSuccess) s = Status::err(EON_E_DEVICE, hipGetErrorString(e));
        }
        if (!s.bad()) s = bases_seal_table(outs[t], ctx->stream);
    }
    for (hipStream_t st : streams) (void)hipStreamSynchronize(st);
    if (s.bad())
        for (uint32_t t = 0; t < np; t++)
            if (outs[t]) {
                bases_free(outs[t]);
                outs[t] = nullptr;
            }
    return s;
}

// every point's bases at once: point t's whole pipeline on stream t % 3 (the latency-bound
// scalar multiplications of different points overlap)
Status opening_bases_many(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const eon_fr* points,
                          uint32_t npoints, eon_msm_bases** outs) {
    if (!srs || (npoints && (!points || !outs))) return Status::err(EON_E_ARG, "null argument");
    if (n == 0) return Status::err(EON_E_SHAPE, "opening bases need n >= 1");
    if (n - 1 > eon_msm_bases_len(srs)) return Status::err(EON_E_SHAPE, "more opening bases than SRS points");
    std::vector<Fr> zs(npoints);
    for (uint32_t t = 0; t < npoints; t++) {
        zs[t] = fr_from_abi(points + t);
        if (!fr_is_canonical(zs[t])) return Status::err(EON_E_ARG, "point is not a canonical Fr");
        outs[t] = nullptr;
    }
    // sharded when the context is bound to a process group and every point takes the radix-2^29
    // path (a uniform decision: every rank has the same points and SRS)
    bool fast = bases_table29(srs) && bases_window(srs) == TC && bases_windows(srs) == TW && n >= 2;
    for (const Fr& z : zs) fast = fast && !z.is_zero();
    if (fast && ctx->coll.world > 1 && npoints) return opening_bases_sharded(ctx, srs, n, zs, outs);
    hipStream_t streams[3] = {ctx->stream, ctx->side(ctx->msm_side), ctx->side(ctx->msm_side2)};
    EON_HIP(hipEventRecord(ctx->msm_ev[0], ctx->stream));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side, ctx->msm_ev[0], 0));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side2, ctx->msm_ev[0], 0));
    std::vector<Scratch> sc(npoints);
    for (auto& x : sc) x.pool = &ctx->pool;
    Status s = Status::ok();
    for (uint32_t t = 0; t < npoints && !s.bad(); t++)
        s = opening_bases_async(ctx, srs, n, zs[t], streams[t % 3], sc[t], outs + t);
    for (hipStream_t st : streams) (void)hipStreamSynchronize(st);
    for (auto& x : sc) x.release();
    if (s.bad())
        for (uint32_t t = 0; t < npoints; t++)
            if (outs[t]) {
                bases_free(outs[t]);
                outs[t] = nullptr;
            }
    return s;
}

}  // namespace

extern "C" {

int eon_kzg_opening_bases_create(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const eon_fr* point,
                                 eon_msm_bases** out) {
    if (!ctx) return EON_E_ARG;
    if (!point || !out) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = opening_bases_many(ctx, srs, n, point, 1, out);
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

int eon_kzg_opening_bases_create_many(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const eon_fr* points,
                                      uint32_t npoints, eon_msm_bases** outs) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = opening_bases_many(ctx, srs, n, points, npoints, outs);
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // extern "C"
