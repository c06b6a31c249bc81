// Batched radix-2 NTT over BN254 Fr on row-major matrices (gfx950).
//
// Semantics: p3-dft's TwoAdicSubgroupDft<Fr> (dft/src/traits.rs:27-249), with the output-order
// conventions of Radix2Dit (natural, dft/src/radix_2_dit.rs:61-77) and Radix2DitParallel
// (bit-reversed storage, dft/src/radix_2_dit_parallel.rs:146-228).  Any correct NTT returns the
// same canonical field elements, so outputs are bit-exact with the reference.
//
// Structure (MI355X-first, not a translation of the rayon row-chunk schedule):
//   * A size-2^L network is run as P "passes"; a pass executes k consecutive radix-2 stages
//     [s0, s0+k) on every group of 2^k rows that share all index bits outside [s0, s0+k).
//   * One workgroup = one group x CB adjacent columns.  The 2^k x CB tile is staged in LDS as two
//     16-byte half-planes (conflict-free ds_read/write_b128), the pass's 2^k - 1 twiddles are
//     staged beside it, and each thread does butterflies with the 256-bit Montgomery product in
//     registers (field.h).  Global reads/writes are row segments of CB*32 contiguous bytes.
//   * The first pass folds in the input permutation (bit-reversal gather, LDE spread, zero pad)
//     and the coset/inverse scaling; the last pass folds in the output scaling.  No standalone
//     permutation or scaling sweep touches HBM.
//   * Twiddles: one stage-concatenated table tw[2^s + j] = w_{2^(s+1)}^j (inverse table with
//     w^-1), built once on device for the largest size seen; smaller transforms use its prefix.
#include "ntt.h"
#include "field29.h"

namespace eon {

struct PassArgs {
    const Fr* src;
    Fr* dst;
    const Fr* tw;          // plain roots
    const uint32_t* twq;   // their Shoup quotients (TWQ_STRIDE words per entry)
    const Fr* load_scale;   // indexed by source row, or null
    const Fr* store_scale;  // indexed by output row, or null
    Fr load_const;
    uint64_t width;
    uint32_t s0;
    uint32_t k;
    uint32_t load_mode;
    uint32_t load_param;
    uint32_t has_load_const;
    uint32_t col_tiles;
    uint32_t last;  // the network's last pass: canonical output (earlier passes store values < 2p)
    // DIT networks of several passes: the passes between them exchange the tile limbs as they are
    // (normalised, unreduced: values below (2 + 4 x stages) p < 169 p, the Shoup products' input
    // range) in three planes -- limbs 0-3 at mid[i], 4-7 at mid[mid_n + i], 8 at the u32 array
    // after them -- instead of reduced and packed into 32 bytes (no reduce / pack / unpack)
    uint4* mid;
    uint64_t mid_n;
    uint32_t in_mid, out_mid;
};

__device__ __forceinline__ F29 mid_get(const uint4* mid, uint64_t n, uint64_t i) {
    const uint4 a = mid[i], b = mid[n + i];
    F29 x;
    x.l[0] = a.x; x.l[1] = a.y; x.l[2] = a.z; x.l[3] = a.w;
    x.l[4] = b.x; x.l[5] = b.y; x.l[6] = b.z; x.l[7] = b.w;
    x.l[8] = reinterpret_cast<const uint32_t*>(mid + 2 * n)[i];
    return x;
}
__device__ __forceinline__ void mid_put(uint4* mid, uint64_t n, uint64_t i, const F29& x) {
    mid[i] = make_uint4(x.l[0], x.l[1], x.l[2], x.l[3]);
    mid[n + i] = make_uint4(x.l[4], x.l[5], x.l[6], x.l[7]);
    reinterpret_cast<uint32_t*>(mid + 2 * n)[i] = x.l[8];
}

// LDS bytes of one twiddle set (roots or quotients) of nt entries: two 16-B planes and a 4-B one,
// rounded up to 16 B so the next set's planes stay aligned
__host__ __device__ constexpr uint32_t tw_set_bytes(uint32_t nt) { return 32u * nt + ((4u * nt + 15u) & ~15u); }

__device__ __forceinline__ Fr gload(const Fr* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    Fr x;
    x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
    x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
    return x;
}

__device__ __forceinline__ void gstore(Fr* p, const Fr& x) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    q[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}

// ---- the pass kernel ----------------------------------------------------------------------------
// The tile is held in LDS as 9 x 29-bit limbs (three planes: limbs 0-3, 4-7, 8)
// and lazy values: the butterfly product is Shoup's by the plain root w with its precomputed
// quotient floor(w 2^261 / p) (mul29_shoup: 143 carry-free multiply-adds, no Montgomery
// multipliers, output < 3p), so y w 2^256 comes out in the radix-2^32 Montgomery form and staging
// a twiddle is two loads and an unpack.  The input / output scalings (coset powers, 1/n) are
// tables and constants in the 32 c form (ntt_scale_form), applied with mul29.

__device__ __forceinline__ void lds_put29(uint4* lo, uint4* hi, uint32_t* top, uint32_t i, const F29& x) {
    lo[i] = make_uint4(x.l[0], x.l[1], x.l[2], x.l[3]);
    hi[i] = make_uint4(x.l[4], x.l[5], x.l[6], x.l[7]);
    top[i] = x.l[8];
}

__device__ __forceinline__ F29 lds_get29(const uint4* lo, const uint4* hi, const uint32_t* top, uint32_t i) {
    const uint4 a = lo[i], b = hi[i];
    F29 x;
    x.l[0] = a.x; x.l[1] = a.y; x.l[2] = a.z; x.l[3] = a.w;
    x.l[4] = b.x; x.l[5] = b.y; x.l[6] = b.z; x.l[7] = b.w;
    x.l[8] = top[i];
    return x;
}

// DIT stages between carry propagations (k_ntt_pass29; 2 or 3 -- see the bound there)
#ifndef EON_NTT_NORM_EVERY
#define EON_NTT_NORM_EVERY 3
#endif
constexpr uint32_t NTT_NORM_EVERY = EON_NTT_NORM_EVERY;
static_assert(NTT_NORM_EVERY == 2 || NTT_NORM_EVERY == 3, "EON_NTT_NORM_EVERY: 2 or 3");

// KS > 0: the pass's stage count as a compile-time constant, launched with exactly CB 2^KS / 2
// threads (one butterfly per thread and stage): the stage loop unrolls, its index arithmetic folds
// to constants and the lazy / normalising stage choice is resolved at compile time.  KS = 0 reads
// the count from the arguments (any block size).
template <bool DIF, int LOG_CB, int KS = 0>
__global__ void __launch_bounds__(1024) k_ntt_pass29(PassArgs a) {
    constexpr uint32_t CB = 1u << LOG_CB;
    extern __shared__ __attribute__((aligned(16))) uint4 lds[];
    const uint32_t k = KS ? (uint32_t)KS : a.k;
    const uint32_t ne = CB << k;
    uint4* lo = lds;
    uint4* hi = lds + ne;
    uint32_t* top = reinterpret_cast<uint32_t*>(lds + 2 * ne);
    // twiddles in 29-form, three planes like the tile (limbs 0-3, 4-7, 8: one ds_read_b128 pair
    // and a ds_read_b32 per twiddle); packing them to 32 B for a fourth resident tile per CU
    // measured slower (the per-butterfly unpack costs more than the occupancy gains)
    const uint32_t nt = 1u << k;
    uint4* tlo = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + ((36u * ne + 15u) & ~15u));
    uint4* thi = tlo + nt;
    uint32_t* ttop = reinterpret_cast<uint32_t*>(thi + nt);
    // the Shoup quotients of the same twiddles, three planes again (after the roots' top plane,
    // 16-B aligned)
    uint4* qlo = reinterpret_cast<uint4*>(reinterpret_cast<char*>(tlo) + tw_set_bytes(nt));
    uint4* qhi = qlo + nt;
    uint32_t* qtop = reinterpret_cast<uint32_t*>(qhi + nt);

    const uint32_t s0 = a.s0;
    const uint64_t g = blockIdx.x / a.col_tiles;
    const uint64_t low = g & ((1ull << s0) - 1);
    const uint64_t base_row = low + ((g >> s0) << (s0 + k));
    const uint64_t col0 = (uint64_t)(blockIdx.x % a.col_tiles) * CB;
    const uint64_t width = a.width;
    const uint32_t T = KS ? (CB << KS) / 2 : blockDim.x;

    for (uint32_t q = threadIdx.x + 1; q < (1u << k); q += T) {
        const uint32_t l = 31 - __builtin_clz(q);
        const uint32_t r = q - (1u << l);
        const uint64_t s = s0 + l;
        const uint64_t ti = (1ull << s) + low + ((uint64_t)r << s0);
        lds_put29(tlo, thi, ttop, q, unpack29(gload(a.tw + ti)));
        const uint4* wq = reinterpret_cast<const uint4*>(a.twq + ti * TWQ_STRIDE);
        const uint4 q0 = wq[0], q1 = wq[1], q2 = wq[2];
        qlo[q] = q0;
        qhi[q] = q1;
        qtop[q] = q2.x;
    }

    for (uint32_t e = threadIdx.x; e < ne; e += T) {
        const uint32_t c = e & (CB - 1);
        const uint32_t m = e >> LOG_CB;
        const uint64_t p = base_row + ((uint64_t)m << s0);
        const uint64_t col = col0 + c;
        F29 x = unpack29(Fr::zero());
        if (col < width && a.in_mid) {
            x = mid_get(a.mid, a.mid_n, p * width + col);
        } else if (col < width) {
            uint64_t r = p;
            bool present = true;
            switch (a.load_mode) {
                case LOAD_BITREV:
                    r = a.load_param ? (__builtin_bitreverse64(p) >> (64 - a.load_param)) : 0;
                    break;
                case LOAD_SPREAD: r = p >> a.load_param; break;
                case LOAD_ZEROPAD: present = p < a.load_param; break;
                case LOAD_BITREV_SPREAD: {
                    const uint32_t nb = a.load_param >> 8;
                    const uint64_t q = p >> (a.load_param & 0xff);
                    r = nb ? (__builtin_bitreverse64(q) >> (64 - nb)) : 0;
                    break;
                }
                default: break;
            }
            if (present) {
                // canonical in, below 2p out of a product (the first stage's input bound)
                x = unpack29(gload(a.src + r * width + col));
                if (a.load_scale) x = mul29<FrP>(x, unpack29(ld_pinned(a.load_scale + r)));
                if (a.has_load_const) x = mul29<FrP>(x, unpack29(a.load_const));
            }
        }
        lds_put29(lo, hi, top, e, x);
    }
    __syncthreads();

    auto tw29 = [&](uint32_t q) {
        F29 w = lds_get29(tlo, thi, ttop, q);
        pin29(w);
        return w;
    };
    auto twq29 = [&](uint32_t q) {
        F29 w = lds_get29(qlo, qhi, qtop, q);
        pin29(w);
        return w;
    };
#pragma unroll
    for (uint32_t it = 0; it < (KS ? (uint32_t)KS : k); it++) {
        const uint32_t l = DIF ? (k - 1 - it) : it;
        const uint32_t half = 1u << l;
        for (uint32_t b = threadIdx.x; b < (ne >> 1); b += T) {
            const uint32_t c = b & (CB - 1);
            const uint32_t j = b >> LOG_CB;
            const uint32_t r = j & (half - 1);
            const uint32_t m0 = ((j >> l) << (l + 1)) | r;
            const uint32_t i0 = (m0 << LOG_CB) | c;
            const uint32_t i1 = ((m0 + half) << LOG_CB) | c;
            const F29 x = lds_get29(lo, hi, top, i0);
            const F29 y = lds_get29(lo, hi, top, i1);
            // the twiddle-free butterflies are skipped only where a whole stage is twiddle-free
            // (half = 1 at low = 0: a uniform branch); elsewhere a unit twiddle is multiplied like
            // any other (its 29-form is 2^261 mod p), as a per-lane choice would run both paths
            // (not on unreduced inputs from a previous pass: t = y would break the < 3p bound the
            // lazy subtraction needs; the unit root is multiplied, which reduces y below 3p)
            const bool unit = half == 1 && low == 0 && !a.in_mid;
            F29 u, v;
            F29 w, wq;
            if (!unit) {
                w = tw29(half + r);
                wq = twq29(half + r);
            }
            if (!DIF) {
                // DitButterfly (dft/src/butterflies.rs:177-185): (x + w*y, x - w*y).  Lazy: t < 3p
                // (the Shoup product, or y itself at the unit stage, which is the pass's first and
                // sees loaded values < 2p), so both outputs are below x + 4p -- a pass of k <= 10
                // stages ends below 37p, inside the range mul29_shoup takes (any value
                // < 2^261 = 169p); the store brings it back below 2p (reduce_top29)
                const F29 t = unit ? y : mul29_shoup<FrP>(y, w, wq);
                // carries propagated every NTT_NORM_EVERY-th stage counted back from the pass's
                // last: a lazy stage takes limbs < L to < L + 2^30 (x + t; x + (4p borrowed) - t,
                // borrowed limbs < 2^30), so two lazy stages after normalised inputs leave limbs
                // < 2.5 2^30, which the next stage's Shoup product (field29.h:
                // shoup_columns_fit_u64) and its carry-propagating add / sub29_wide (< 3.5 2^30 +
                // carry per limb) take.  Values grow by <= 4p per stage: < 42p after 10
                if ((k - 1 - it) % NTT_NORM_EVERY) {
                    u = add29_lazy(x, t);
                    v = sub29_lazy<FrP, 4>(x, t);
                } else {
                    u = add29_norm(x, t);
                    v = sub29_wide<FrP, 3>(x, t);
                }
            } else {
                // DIF butterfly: (x + y, (x - y) * w).  The pass's inputs are below 2p; the sum is
                // brought back below 2p by reduce_top29 only at odd stages of the pass.  A Shoup
                // output is below 3p (2p when its quotient estimate is exact or one short -- the
                // dropped low columns can make it one shorter), so an even stage's inputs are below
                // 3p and its unreduced sum below 6p, which is the worst input of the odd stage after
                // it: the difference x - y + 6p (< 12p) never goes negative and stays well inside
                // the Shoup product's range (< 2^261 = 169p); the sum (< 12p) goes through
                // reduce_top29.  At the unit stage, the pass's last, the difference is kept and
                // reduce_top29 runs at the store.  (A carry-free difference into the product by
                // sub29_lazy measured slower: profiles/r03/ab_ntt_lazy.txt)
                const F29 sum = add29_norm(x, y);
                u = (it & 1) ? reduce_top29<FrP>(sum) : sum;
                const F29 d = sub29<FrP, 6>(x, y);
                v = unit ? d : mul29_shoup<FrP>(d, w, wq);
            }
            lds_put29(lo, hi, top, i0, u);
            lds_put29(lo, hi, top, i1, v);
        }
        __syncthreads();
    }

    for (uint32_t e = threadIdx.x; e < ne; e += T) {
        const uint32_t c = e & (CB - 1);
        const uint32_t m = e >> LOG_CB;
        const uint64_t p = base_row + ((uint64_t)m << s0);
        const uint64_t col = col0 + c;
        if (col < width && a.out_mid) {
            mid_put(a.mid, a.mid_n, p * width + col, lds_get29(lo, hi, top, e));
        } else if (col < width) {
            // below 2p (fits 256 bits) between passes, canonical after the last one
            F29 r = reduce_top29<FrP>(lds_get29(lo, hi, top, e));
            if (a.store_scale) r = mul29<FrP>(r, unpack29(ld_pinned(a.store_scale + p)));
            gstore(a.dst + p * width + col, pack29<FrP>(a.last ? canon29<FrP>(r) : r));
        }
    }
}

// out[idx(j)] = scale * base^j for j in [0, n); idx(j) = j, or reverse_bits(j, rev_log) when
// rev_log != NATURAL_IDX.  Each thread walks a contiguous chunk of exponents.
__global__ void k_powers(Fr* out, uint64_t n, Fr base, Fr scale, uint32_t rev_log, uint32_t chunk) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t j0 = t * chunk;
    if (j0 >= n) return;
    // base^j0 by square-and-multiply
    Fr acc = Fr::one(), b = base;
    for (uint64_t e = j0; e; e >>= 1) {
        if (e & 1) acc = mul(acc, b);
        b = sqr(b);
    }
    acc = mul(acc, scale);
    const uint64_t j1 = (j0 + chunk < n) ? j0 + chunk : n;
    for (uint64_t j = j0; j < j1; j++) {
        const uint64_t idx = rev_log == NATURAL_IDX ? j
                             : (rev_log == 0 ? 0 : (__builtin_bitreverse64(j) >> (64 - rev_log)));
        gstore(out + idx, acc);
        acc = mul(acc, base);
    }
}

// Every entry T = 32 w (Montgomery form, i.e. w 2^261 mod p) becomes the plain root w, and its
// Shoup quotient floor(w 2^261 / p) goes to twq (shoup_pair29).
__global__ void k_tw_shoup(Fr* tw, uint32_t* twq, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    F29 w, wq;
    shoup_pair29<FrP>(unpack29(gload(tw + i)), w, wq);
    gstore(tw + i, pack29<FrP>(w));
    uint4* q = reinterpret_cast<uint4*>(twq + i * TWQ_STRIDE);
    q[0] = make_uint4(wq.l[0], wq.l[1], wq.l[2], wq.l[3]);
    q[1] = make_uint4(wq.l[4], wq.l[5], wq.l[6], wq.l[7]);
    q[2] = make_uint4(wq.l[8], 0u, 0u, 0u);

}

// tw[2^s + j] = tw[2^(L-1) + (j << (L-1-s))] for s < L-1 (sub-sampling the largest stage).
__global__ void k_tw_fill_lower(Fr* tw, uint32_t L) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t top = 1ull << (L - 1);
    if (q == 0 || q >= top) return;
    const uint32_t s = 63 - __builtin_clzll(q);
    const uint64_t j = q - (1ull << s);
    tw[q] = tw[top + (j << (L - 1 - s))];
}

#ifndef EON_NTT_FIXED_K
#define EON_NTT_FIXED_K 1
#endif

static hipError_t launch_pass(bool dif, uint32_t log_cb, const PassArgs& a, uint64_t groups,
                              uint64_t col_tiles, uint32_t max_threads, hipStream_t st) {
    const uint32_t ne = (1u << log_cb) << a.k;
    // one butterfly per thread per stage: 512 threads per 1024-element (36 KiB) tile keeps the
    // CU at 32 waves with 4 LDS-bound tiles resident
    uint32_t threads = ne / 2;
    if (threads > max_threads) threads = max_threads;
    if (threads < 64) threads = 64;
    const size_t lds = (((size_t)ne * 36 + 15) & ~(size_t)15) + 2 * (size_t)tw_set_bytes(1u << a.k);
    dim3 grid((unsigned)(groups * col_tiles));
#define EON_LAUNCH(D, C) hipLaunchKernelGGL((k_ntt_pass29<D, C>), grid, dim3(threads), lds, st, a)
#define EON_LAUNCH_K(D, KK) hipLaunchKernelGGL((k_ntt_pass29<D, 3, KK>), grid, dim3((8u << KK) / 2), lds, st, a)
#if EON_NTT_FIXED_K
    // the network shapes of the prove and the LDE (8-column tiles of 2^5 .. 2^7 rows)
    if (log_cb == 3 && a.k >= 5 && a.k <= 7 && threads == ne / 2) {
        switch ((dif ? 8 : 0) + a.k) {
            case 5: EON_LAUNCH_K(false, 5); break;
            case 6: EON_LAUNCH_K(false, 6); break;
            case 7: EON_LAUNCH_K(false, 7); break;
            case 13: EON_LAUNCH_K(true, 5); break;
            case 14: EON_LAUNCH_K(true, 6); break;
            case 15: EON_LAUNCH_K(true, 7); break;
        }
        return hipGetLastError();
    }
#endif
    switch ((dif ? 4 : 0) + log_cb) {
        case 0: EON_LAUNCH(false, 0); break;
        case 1: EON_LAUNCH(false, 1); break;
        case 2: EON_LAUNCH(false, 2); break;
        case 3: EON_LAUNCH(false, 3); break;
        case 4: EON_LAUNCH(true, 0); break;
        case 5: EON_LAUNCH(true, 1); break;
        case 6: EON_LAUNCH(true, 2); break;
        case 7: EON_LAUNCH(true, 3); break;
    }
#undef EON_LAUNCH
#undef EON_LAUNCH_K
    return hipGetLastError();
}

hipError_t launch_powers(Fr* out, uint64_t n, const Fr& base, const Fr& scale, uint32_t rev_log,
                         hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint32_t chunk = n >= (1u << 16) ? 64 : 1;
    const uint64_t threads = (n + chunk - 1) / chunk;
    const uint32_t bs = 256;
    hipLaunchKernelGGL(k_powers, dim3((unsigned)((threads + bs - 1) / bs)), dim3(bs), 0, st, out, n,
                       base, scale, rev_log, chunk);
    return hipGetLastError();
}

hipError_t launch_twiddles(Fr* tw, uint32_t* twq, uint32_t L, const Fr& root_L, hipStream_t st) {
    // tw has 2^L entries; tw[0] unused.  Stage L-1 table = root_L^j, j < 2^(L-1), first built as
    // 32 root_L^j in Montgomery form, then split into the plain roots and their Shoup quotients
    if (L == 0) return hipSuccess;
    hipError_t e = launch_powers(tw + (1ull << (L - 1)), 1ull << (L - 1), root_L, ntt_scale_form(Fr::one()),
                                 NATURAL_IDX, st);
    if (e != hipSuccess) return e;
    const uint64_t n = 1ull << (L - 1);
    if (L > 1) {
        hipLaunchKernelGGL(k_tw_fill_lower, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, tw, L);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_tw_shoup, dim3((unsigned)((2 * n + 255) / 256)), dim3(256), 0, st, tw, twq, 2 * n);
    return hipGetLastError();
}

static uint32_t pick_log_cb(uint64_t width) {
    if (width >= 8) return 3;
    if (width >= 4) return 2;
    if (width >= 2) return 1;
    return 0;
}

// stages per pass at most, and the pass count, of the network run_network launches for `s`
static uint32_t plan_passes(const NetworkSpec& s, uint32_t log_cb, uint32_t* n_st_out) {
    const uint32_t log_tile = s.log_tile ? s.log_tile : 10;  // 2^10 elements per tile: 32 KiB of LDS
    uint32_t kmax = log_tile > log_cb ? log_tile - log_cb : 1;
    if (s.max_stages_per_pass && s.max_stages_per_pass < kmax) kmax = s.max_stages_per_pass;
    const uint32_t n_st = s.log_m > s.first_stage ? s.log_m - s.first_stage : 0;
    if (n_st_out) *n_st_out = n_st;
    return n_st == 0 ? 1 : (n_st + kmax - 1) / kmax;
}

uint32_t network_passes(const NetworkSpec& s) {
    return plan_passes(s, s.log_cb_override >= 0 ? (uint32_t)s.log_cb_override : pick_log_cb(s.width), nullptr);
}

hipError_t run_network(const NetworkSpec& s, hipStream_t st, Profiler* prof) {
    const uint32_t log_cb = s.log_cb_override >= 0 ? (uint32_t)s.log_cb_override : pick_log_cb(s.width);
    const uint32_t log_tile = s.log_tile ? s.log_tile : 10;
    const uint32_t lo_stage = s.first_stage;
    uint32_t n_st = 0;
    const uint32_t passes = plan_passes(s, log_cb, &n_st);
    const uint64_t col_tiles = (s.width + (1u << log_cb) - 1) >> log_cb;
    // balanced chunk sizes, assigned bottom-up (stage ranges ascending)
    uint32_t ks[32], s0s[32];
    uint32_t acc = lo_stage;
    for (uint32_t i = 0; i < passes; i++) {
        ks[i] = n_st / passes + (i < n_st % passes ? 1 : 0);
        s0s[i] = acc;
        acc += ks[i];
    }
    for (uint32_t it = 0; it < passes; it++) {
        // DIT runs the stage chunks low -> high, DIF high -> low
        const uint32_t i = s.dif ? passes - 1 - it : it;
        PassArgs a{};
        const bool first = it == 0, last = it == passes - 1;
        a.src = first ? s.src : s.dst;
        a.dst = s.dst;
        a.tw = s.tw;
        a.twq = s.twq;
        a.width = s.width;
        a.s0 = s0s[i];
        a.k = ks[i];
        if (first) {
            a.load_mode = s.load_mode;
            a.load_param = s.load_param;
            a.load_scale = s.load_scale;
            a.has_load_const = s.has_load_const;
            a.load_const = s.load_const;
        } else {
            a.load_mode = LOAD_DIRECT;
        }
        a.store_scale = last ? s.store_scale : nullptr;
        a.last = last ? 1u : 0u;
        if (!s.dif && s.mid && passes > 1) {
            a.mid = s.mid;
            a.mid_n = (1ull << s.log_m) * s.width;
            a.in_mid = first ? 0u : 1u;
            a.out_mid = last ? 0u : 1u;
        }
        const uint64_t groups = (1ull << s.log_m) >> a.k;
        static const char* names[8] = {"k_ntt_pass29<false, 0>", "k_ntt_pass29<false, 1>",
                                         "k_ntt_pass29<false, 2>", "k_ntt_pass29<false, 3>",
                                         "k_ntt_pass29<true, 0>",  "k_ntt_pass29<true, 1>",
                                         "k_ntt_pass29<true, 2>",  "k_ntt_pass29<true, 3>"};
        // mulmods: one per butterfly (the BASELINE.md count), plus the fused input/output scalings
        const uint64_t elems = (1ull << s.log_m) * s.width;
        const uint64_t mm = elems / 2 * a.k + (a.load_scale ? elems : 0) + (a.has_load_const ? elems : 0) +
                            (a.store_scale ? elems : 0);
        if (prof) prof->begin(names[(s.dif ? 4 : 0) + log_cb], 64ull * elems, st, mm);
        a.col_tiles = (uint32_t)col_tiles;
        const uint32_t tpb = s.max_threads ? s.max_threads : (log_tile > 10 ? 1024 : 512);
        hipError_t e = launch_pass(s.dif, log_cb, a, groups, col_tiles, tpb, st);
        if (prof) prof->end(st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace eon
