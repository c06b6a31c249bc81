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

constexpr uint32_t SCAN = 16;  // points summed per thread at each level of the prefix sum

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

// tot[t] = sum of a[SCAN t .. SCAN t + SCAN)
__global__ void k_scan_totals(const G1Xyzz* a, uint64_t len, G1Xyzz* tot) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * SCAN;
    if (i0 >= len) return;
    const uint64_t i1 = i0 + SCAN < len ? i0 + SCAN : len;
    G1Xyzz acc = ld_xyzz(a + i0);
    for (uint64_t i = i0 + 1; i < i1; i++) acc = xyzz_add(acc, ld_xyzz(a + i));
    st_xyzz(tot + t, acc);
}

// a <- exclusive prefix sums, chunk t starting from carry[t] (the exclusive prefix of the totals)
__global__ void k_scan_apply(G1Xyzz* a, uint64_t len, const G1Xyzz* carry) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * SCAN;
    if (i0 >= len) return;
    const uint64_t i1 = i0 + SCAN < len ? i0 + SCAN : len;
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
// rows i = lo + t, t < cnt (a rank's slice; rows >= n - 1 are the identity)
__global__ void __launch_bounds__(64) k_open_scale29(const G1Affine* tab, const G1Affine* tab3, uint64_t n,
                                                     uint64_t lo, uint64_t cnt, Fr zinv, G1Xyzz* out_slice) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint64_t i = lo + t;
    G1Xyzz* out = out_slice - lo;
    if (i + 1 >= n) {
        st_xyzz(out + i, xyzz_inf());
        return;
    }
    const G1Affine* row = tab + i * TW;
    {
        const G1Affine g = ld_affine(row);
        if (is_inf(g)) {  // the identity's table row is all identity
            st_xyzz(out + i, xyzz_inf());
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
            for (uint32_t w = 0; w < TW; w++) {
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
            for (uint32_t w = 0; w < TW; w++) {
                ld_affine29(row + w, ((u[w] >> b) & 1) == 0, x, y);
                madd29_any(acc, inf, x, y);
            }
        }
    }
    if (even) {
        ld_affine29(row, true, x, y);
        madd29_any(acc, inf, x, y);
    }
    st_xyzz(out + i, x29_to_xyzz(acc, inf));
}

// H_j = z^(j-1) S_j, then its window table 2^(16 w) H_j, w < TW, by doublings: tmp[j TW + w]
// (radix-2^32 XYZZ).  The scalar multiplication uses REGULAR signed 4-bit windows (no lane
// divergence: every lane adds at every window): k = z^(j-1) made odd (k + 1 when even, S_j
// subtracted at the end) is recoded into 64 odd digits in [-15, 15] (d = (k mod 32) - 16,
// k <- (k - d) / 16), and the odd multiples S, 3S, .., 15S live in the thread's column of `mtab`
// (MTAB raw accumulators per thread, coalesced across threads): 256 doublings + 64 additions,
// against ~254 + ~254 (divergent) for double-and-add.
// rows j = lo + t, t < cnt; s and tmp are the slice's (rows >= n are the identity)
constexpr uint32_t MTAB = 8;

__global__ void __launch_bounds__(64) k_open_finish29(const G1Affine* s_slice, uint64_t n, uint64_t lo, uint64_t cnt,
                                                      Fr z, G1Raw29* mtab, G1Xyzz* tmp_slice) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint64_t j = lo + t;
    const G1Affine* s = s_slice - lo;
    G1Xyzz* tmp = tmp_slice - lo * TW;
    G1X29 acc;
    bool inf = true;
    const G1Affine a = (j && j < n) ? ld_affine(s + j) : G1Affine{Fq::zero(), Fq::zero()};
    if (!is_inf(a)) {
        const F29 x = unpack29(to_fq261(a.x)), y = unpack29(to_fq261(a.y));
        Fr k = to_canonical(pow_u64(z, j - 1));
        const bool even = (k.v[0] & 1) == 0;
        if (even) k.v[0] += 1;  // no carry: k even
        // the odd multiples (2m + 1) S, m < MTAB
        {
            G1X29 two = dbl29_affine(x, y), m;
            m.X = x;
            m.Y = y;
            m.ZZ = const29<FqP>(R29<FqP>::ONE);
            m.ZZZ = m.ZZ;
            bool m_inf = false;
            st_raw29(mtab + t, m);
            for (uint32_t q = 1; q < MTAB; q++) {
                acc29(m, m_inf, two, false);  // S has odd order: the multiples are never O
                st_raw29(mtab + (uint64_t)q * cnt + t, m);
            }
        }
        // recoding: 64 odd digits, nibble i of dg[] = (|d_i| - 1) / 2 | sign << 3
        uint32_t dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        uint32_t kw[8];
#pragma unroll
        for (int q = 0; q < 8; q++) kw[q] = k.v[q];
#pragma unroll
        for (int i = 0; i < 63; i++) {
            const int32_t d = (int32_t)(kw[0] & 31u) - 16;
            // k - d (|d| <= 15, odd), then >> 4 (exact)
            if (d >= 0) {
                uint64_t c = (uint64_t)kw[0] - (uint32_t)d;
                kw[0] = (uint32_t)c;
                uint32_t br = (uint32_t)(c >> 63);
#pragma unroll
                for (int q = 1; q < 8; q++) {
                    c = (uint64_t)kw[q] - br;
                    kw[q] = (uint32_t)c;
                    br = (uint32_t)(c >> 63);
                }
            } else {
                uint64_t c = (uint64_t)kw[0] + (uint32_t)(-d);
                kw[0] = (uint32_t)c;
                uint32_t cy = (uint32_t)(c >> 32);
#pragma unroll
                for (int q = 1; q < 8; q++) {
                    c = (uint64_t)kw[q] + cy;
                    kw[q] = (uint32_t)c;
                    cy = (uint32_t)(c >> 32);
                }
            }
#pragma unroll
            for (int q = 0; q < 7; q++) kw[q] = (kw[q] >> 4) | (kw[q + 1] << 28);
            kw[7] >>= 4;
            const uint32_t mag = (uint32_t)(d < 0 ? -d : d);
            dg[i >> 3] |= (((mag - 1) >> 1) | (d < 0 ? 8u : 0u)) << (4 * (i & 7));
        }
        // the top digit: the rest, odd, in [1, 15] (k < 2^254)
        dg[7] |= ((kw[0] - 1) >> 1) << 28;
        G1X29 e;
        (void)ld_raw29(mtab + (uint64_t)((dg[7] >> 28) & 7u) * cnt + t, e);
        acc = e;
        inf = false;
        for (int i = 62; i >= 0; i--) {
            dbl29(acc);
            dbl29(acc);
            dbl29(acc);
            dbl29(acc);
            const uint32_t nib = (dg[i >> 3] >> (4 * (i & 7))) & 15u;
            (void)ld_raw29(mtab + (uint64_t)(nib & 7u) * cnt + t, e);
            if (nib & 8u) e.Y = sub29<FqP, 4>(F29{}, e.Y);  // -(x, y): Y < 4p
            acc29(acc, inf, e, false);
        }
        if (even) {
            const F29 ny = sub29<FqP, 1>(F29{}, y);  // y canonical < p
            madd29_any(acc, inf, x, ny);
        }
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

// exclusive prefix sum of a[0..len) in place; tmp holds >= len / SCAN + len / SCAN^2 + ... points
void scan_exclusive(G1Xyzz* a, uint64_t len, G1Xyzz* tmp, hipStream_t st) {
    if (len <= SCAN) {
        hipLaunchKernelGGL(k_scan_serial, dim3(1), dim3(1), 0, st, a, len);
        return;
    }
    const uint64_t nt = (len + SCAN - 1) / SCAN;
    hipLaunchKernelGGL(k_scan_totals, dim3(grid_for(nt, 64)), dim3(64), 0, st, a, len, tmp);
    scan_exclusive(tmp, nt, tmp + nt, st);
    hipLaunchKernelGGL(k_scan_apply, dim3(grid_for(nt, 64)), dim3(64), 0, st, a, len, tmp);
}

// one point's scratch, alive until its stream is synchronised
struct Scratch {
    DevBuf h_aff, pts, tmp, aff, table_tmp, mtab;
    void release() {
        for (DevBuf* b : {&h_aff, &pts, &tmp, &aff, &table_tmp, &mtab}) b->release();
    }
};

// radix-2^29 fast path: P_i from the SRS table, one kernel for H_j and its window table
Status opening_bases_async29(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n, const Fr& z, hipStream_t st,
                             Scratch& sc, eon_msm_bases** out) {
    EON_HIP(sc.pts.ensure(n * sizeof(G1Xyzz)));
    EON_HIP(sc.tmp.ensure((n / (SCAN - 1) + 64) * sizeof(G1Xyzz)));
    EON_HIP(sc.aff.ensure(n * sizeof(G1Affine)));
    EON_HIP(sc.table_tmp.ensure(n * TW * sizeof(G1Xyzz)));
    eon_msm_bases* b = nullptr;
    EON_TRY(bases_alloc_table(ctx, n, TC, &b));
    // ~15 dbl (6M+3S) + 257 madd (8M+2S) and ~254 dbl + ~127 madd + 240 dbl per point
    EON_HIP(sc.mtab.ensure(n * MTAB * sizeof(G1Raw29)));
    const G1Affine* tab3 = bases_table3_29(srs, st);  // null (radix 2) if it cannot be built
    // radix 4: 14 dbl (6M+3S) + 129 madd (8M+2S); radix 2: 15 dbl + 257 madd
    ctx->prof.begin("k_open_scale29", n * (TW * 64ull + 128ull), st, n * (tab3 ? 1416ull : 2705ull));
    hipLaunchKernelGGL(k_open_scale29, dim3(grid_for(n, 64)), dim3(64), 0, st, bases_table29(srs), tab3, n, 0ull,
                       n, inverse(z), sc.pts.as<G1Xyzz>());
    ctx->prof.end(st);
    scan_exclusive(sc.pts.as<G1Xyzz>(), n, sc.tmp.as<G1Xyzz>(), st);
    EON_HIP(launch_batch_to_affine(sc.pts.as<G1Xyzz>(), n, sc.aff.as<G1Affine>(), st));
    // 256 dbl + 64 add (12M+2S) + 8 multiples, then 240 dbl for the window table
    ctx->prof.begin("k_open_finish29", n * (64ull + TW * 128ull), st, n * 5300ull);
    hipLaunchKernelGGL(k_open_finish29, dim3(grid_for(n, 64)), dim3(64), 0, st, sc.aff.as<G1Affine>(), n, 0ull, n, z,
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
    EON_HIP(sc.h_aff.ensure(n * sizeof(G1Affine)));
    if (z.is_zero()) {
        hipLaunchKernelGGL(k_open_shift, dim3(grid_for(n, 256)), dim3(256), 0, st, g, n, sc.h_aff.as<G1Affine>());
        EON_HIP(hipGetLastError());
    } else {
        EON_HIP(sc.pts.ensure(n * sizeof(G1Xyzz)));
        EON_HIP(sc.tmp.ensure((n / (SCAN - 1) + 64) * sizeof(G1Xyzz)));
        EON_HIP(sc.aff.ensure(n * sizeof(G1Affine)));
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
    DevBuf totals_x, totals_a, all_totals, send, recv;
    struct Release {
        std::vector<Scratch>& sc;
        DevBuf* b[5];
        ~Release() {
            for (auto& x : sc) x.release();
            for (DevBuf* x : b) x->release();
        }
    } release{sc, {&totals_x, &totals_a, &all_totals, &send, &recv}};
    EON_HIP(totals_x.ensure(np * sizeof(G1Xyzz)));
    EON_HIP(totals_a.ensure(np * sizeof(G1Affine)));
    EON_HIP(all_totals.ensure((uint64_t)world * np * sizeof(G1Affine)));
    const uint64_t slice_entries = m * TW;  // per point
    EON_HIP(send.ensure(np * slice_entries * sizeof(G1Affine)));
    EON_HIP(recv.ensure((uint64_t)world * np * slice_entries * sizeof(G1Affine)));
    EON_HIP(hipEventRecord(ctx->msm_ev[0], ctx->stream));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side, ctx->msm_ev[0], 0));
    EON_HIP(hipStreamWaitEvent(ctx->msm_side2, ctx->msm_ev[0], 0));
    // phase 1: P_i of the slice and its exclusive prefix sums; the total lands at index m
    for (uint32_t t = 0; t < np; t++) {
        hipStream_t st = streams[t % 3];
        EON_HIP(sc[t].pts.ensure((m + 1) * sizeof(G1Xyzz)));
        EON_HIP(sc[t].tmp.ensure(((m + 1) / (SCAN - 1) + 64) * sizeof(G1Xyzz)));
        EON_HIP(sc[t].aff.ensure(m * sizeof(G1Affine)));
        EON_HIP(sc[t].table_tmp.ensure(slice_entries * sizeof(G1Xyzz)));
        EON_HIP(sc[t].mtab.ensure(m * MTAB * sizeof(G1Raw29)));
        const G1Affine* tab3 = bases_table3_29(srs, st);  // null (radix 2) if it cannot be built
        ctx->prof.begin("k_open_scale29", m * (TW * 64ull + 128ull), st, m * (tab3 ? 1416ull : 2705ull));
        hipLaunchKernelGGL(k_open_scale29, dim3(grid_for(m, 64)), dim3(64), 0, st, bases_table29(srs), tab3, n, lo, m,
                           inverse(zs[t]), sc[t].pts.as<G1Xyzz>());
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
        EON_HIP(launch_batch_to_affine(sc[t].pts.as<G1Xyzz>(), m, sc[t].aff.as<G1Affine>(), st));
        ctx->prof.begin("k_open_finish29", m * (64ull + TW * 128ull), st, m * 5300ull);
        hipLaunchKernelGGL(k_open_finish29, dim3(grid_for(m, 64)), dim3(64), 0, st, sc[t].aff.as<G1Affine>(), n, lo,
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
