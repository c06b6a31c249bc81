// Pippenger multi-scalar multiplication on BN254 G1 for gfx950.
//
// Replaces G1::multi_exp (bn254/src/curve.rs:158-179 -> halo2curves::msm::msm_best) and the KZG
// column commitment commit_column (kzg/src/util.rs:37-40).  The value sum_i s_i * P_i is unique,
// so the result (returned in affine form) is bit-identical to the reference's.
//
// Pipeline (all on device, one stream):
//   1. k_msm_digits     scalars (Montgomery) -> canonical -> signed c-bit digits; one
//                       (bucket key, point reference | sign) pair per nonzero digit.
//   2. radix sort       hipCUB DeviceRadixSort on the c-bit keys (zero digits sort last).
//   3. k_bucket_start   bucket boundaries in the sorted pairs.
//   4. pieces           every bucket is cut into pieces of <= PIECE entries (load balance under
//                       skewed scalars); exclusive scan of piece counts.
//   5. k_piece_sum      one thread per piece: XYZZ mixed additions of affine bases.
//   6. k_partial_combine levels of <= PIECE-way sums until each bucket holds one partial
//                       (log-depth under any skew, e.g. all-equal scalars), k_bucket_final.
//   7. k_segment_sum /  sum_d d * B_d per group: segments of SEG buckets by running sums, the
//      k_tree_sum       segment offset applied by a short double-and-add, then LDS tree sums.
//   8. k_window_horner  (per-window buckets only) sum_w 2^(c*w) G_w per MSM; batched affine.
//
// Batched mode (eon_msm_g1_columns*): one pipeline run handles many MSMs at once -- the columns
// of a row-major coefficient matrix, as KzgPcs::commit commits every column against the same
// SRS prefix (kzg/src/pcs.rs:244-251) -- with the column index in the high bits of the key.
//
// Fixed-base mode (eon_msm_bases_create with EON_MSM_PRECOMPUTE; the KZG SRS): the bases object
// stores 2^(c*w) * P_i in affine for every window w, so every window's digits land in ONE bucket
// set (groups = 1): no per-window bucket reduction and no serial doubling chain at the end.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "context.h"
#include "ec.h"
#include "msm.h"

using namespace eon;

struct eon_msm_bases {
    eon_ctx* ctx = nullptr;
    uint64_t n = 0;
    DevBuf points;  // n affine bases
    bool precomputed = false;
    uint32_t c = 0, windows = 0;
    DevBuf table;  // precomputed: n * windows affine points, entry i * windows + w = 2^(c*w) P_i
};

namespace eon {

constexpr uint32_t PIECE = 32;  // max mixed additions per piece
constexpr uint32_t SEG = 8;     // buckets per reduction segment
constexpr uint32_t TREE = 256;  // points per tree-reduction block

__device__ __forceinline__ uint32_t window_bits(const uint32_t* s, uint32_t pos, uint32_t c) {
    // bits [pos, pos + c) of the 256-bit canonical scalar s (little-endian u32 limbs), c <= 24
    const uint32_t li = pos >> 5, off = pos & 31;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) {
        lo = (j == li) ? s[j] : lo;
        hi = (j == li + 1) ? s[j] : hi;
    }
    const uint64_t v = ((uint64_t)hi << 32 | lo) >> off;
    return (uint32_t)v & ((1u << c) - 1);
}

// One thread per (row i, MSM column col): the scalar is scalars[i * ld + col] (a row-major
// matrix column; ld = 1, cols = 1 for a single MSM).  Group of a digit: the column (fixed-base
// mode: every window shares the column's bucket set) or (column, window).
__global__ void k_msm_digits(const Fr* scalars, uint64_t n, uint64_t ld, uint32_t cols, uint32_t c,
                             uint32_t windows, uint32_t precomputed, uint32_t* keys, uint32_t* vals) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * cols) return;
    const uint32_t col = (uint32_t)(t % cols);
    const uint64_t i = t / cols;
    Fr s = to_canonical(ld_pinned(scalars + i * ld + col));
    pin(s);
    const uint32_t B = 1u << (c - 1);
    const uint32_t sentinel = (precomputed ? cols : cols * windows) * B;
    uint32_t carry = 0;
    for (uint32_t w = 0; w < windows; w++) {
        const uint32_t raw = window_bits(s.v, w * c, c) + carry;
        uint32_t mag;
        uint32_t neg;
        if (raw > B) {  // signed digit raw - 2^c in [-(B-1), -1], carry into the next window
            mag = (1u << c) - raw;
            neg = 1;
            carry = 1;
        } else {
            mag = raw;
            neg = 0;
            carry = 0;
        }
        const uint64_t e = ((uint64_t)w * n + i) * cols + col;
        if (mag == 0) {
            keys[e] = sentinel;
            vals[e] = 0;
        } else {
            const uint32_t g = precomputed ? col : col * windows + w;
            keys[e] = g * B + mag - 1;
            const uint32_t ref = precomputed ? (uint32_t)(i * windows + w) : (uint32_t)i;
            vals[e] = ref | (neg << 31);
        }
    }
}

// per-window sums -> per-column result: sum_w 2^(c*w) * G[col*W + w] (one thread per column)
__global__ void k_window_horner(const G1Xyzz* gs, uint32_t cols, uint32_t W, uint32_t c,
                                G1Xyzz* out) {
    const uint32_t col = blockIdx.x * blockDim.x + threadIdx.x;
    if (col >= cols) return;
    const G1Xyzz* g = gs + (uint64_t)col * W;
    G1Xyzz acc = ld_xyzz(g + W - 1);
    for (int w = (int)W - 2; w >= 0; w--) {
        for (uint32_t k = 0; k < c; k++) acc = xyzz_dbl(acc);
        acc = xyzz_add(acc, ld_xyzz(g + w));
    }
    st_xyzz(out + col, acc);
}

// start[b] = index of the first sorted pair with key >= b, for b in [0, nb]
__global__ void k_bucket_start(const uint32_t* keys, uint64_t E, uint32_t nb, uint32_t* start) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > E) return;
    const int64_t prev = i == 0 ? -1 : (int64_t)min(keys[i - 1], nb);
    const int64_t cur = i == E ? (int64_t)nb : (int64_t)min(keys[i], nb);
    for (int64_t b = prev + 1; b <= cur; b++) start[b] = (uint32_t)i;
}

__global__ void k_piece_owner(const uint32_t* piece_off, uint32_t nb, uint32_t* owner) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    for (uint32_t p = piece_off[b]; p < piece_off[b + 1]; p++) owner[p] = b;
}

__global__ void k_piece_sum(const uint32_t* vals, const uint32_t* start, const uint32_t* piece_off,
                            const uint32_t* owner, uint32_t n_pieces, const G1Affine* pts,
                            G1Xyzz* piece_sums) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pieces) return;
    const uint32_t b = owner[p];
    const uint32_t j = p - piece_off[b];
    const uint32_t e0 = start[b] + j * PIECE;
    const uint32_t e1 = min(e0 + PIECE, start[b + 1]);
    G1Xyzz acc = xyzz_inf();
    for (uint32_t e = e0; e < e1; e++) {
        const uint32_t v = vals[e];
        G1Affine a = ld_affine(pts + (v & 0x7fffffffu));
        if (v >> 31) a = affine_neg(a);
        acc = xyzz_add_affine(acc, a);
    }
    st_xyzz(piece_sums + p, acc);
}

// One combine level: new partial p of bucket b sums old partials
// [off_old[b] + PIECE*j, min(+PIECE, off_old[b+1])), j = p - off_new[b].
__global__ void k_partial_combine(const uint32_t* off_old, const uint32_t* off_new,
                                  const uint32_t* owner, uint32_t n_new, const G1Xyzz* in,
                                  G1Xyzz* out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_new) return;
    const uint32_t b = owner[p];
    const uint32_t j = p - off_new[b];
    const uint32_t e0 = off_old[b] + j * PIECE;
    const uint32_t e1 = min(e0 + PIECE, off_old[b + 1]);
    G1Xyzz acc = ld_xyzz(in + e0);
    for (uint32_t e = e0 + 1; e < e1; e++) acc = xyzz_add(acc, ld_xyzz(in + e));
    st_xyzz(out + p, acc);
}

// count[b] = ceil((off[b+1] - off[b]) / PIECE) (0 for the terminator)
__global__ void k_level_count(const uint32_t* off, uint32_t nb, uint32_t* count) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nb) return;
    count[b] = b == nb ? 0 : (off[b + 1] - off[b] + PIECE - 1) / PIECE;
}

// every bucket holds at most one partial: bucket_sums[b] = it, or the identity
__global__ void k_bucket_final(const uint32_t* off, uint32_t nb, const G1Xyzz* partials,
                               G1Xyzz* bucket_sums) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    st_xyzz(bucket_sums + b, off[b + 1] > off[b] ? ld_xyzz(partials + off[b]) : xyzz_inf());
}

// Segment s of group g covers buckets [lo, lo + SEG) (bucket b holds digit b + 1):
// out = sum_b (b + 1) * S_b = (running-sum form) + lo * (sum_b S_b)
__global__ void k_segment_sum(const G1Xyzz* bucket_sums, uint32_t B, uint32_t groups,
                              G1Xyzz* seg_out) {
    const uint32_t nseg = B / SEG;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg * groups) return;
    const uint32_t g = t / nseg, s = t % nseg;
    const uint32_t lo = s * SEG;
    const G1Xyzz* sb = bucket_sums + (uint64_t)g * B + lo;
    G1Xyzz run = xyzz_inf(), acc = xyzz_inf();
    for (int k = SEG - 1; k >= 0; k--) {
        run = xyzz_add(run, ld_xyzz(sb + k));
        acc = xyzz_add(acc, run);
    }
    if (lo) acc = xyzz_add(acc, xyzz_mul_small(run, lo));
    st_xyzz(seg_out + t, acc);
}

// out[g * gridDim.x + blk] = sum of in[g * n + blk * TREE .. + TREE)
__global__ void __launch_bounds__(TREE) k_tree_sum(const G1Xyzz* in, uint32_t n, G1Xyzz* out) {
    __shared__ G1Xyzz sh[TREE];
    const uint32_t g = blockIdx.y;
    const uint32_t i = blockIdx.x * TREE + threadIdx.x;
    G1Xyzz acc = i < n ? ld_xyzz(in + (uint64_t)g * n + i) : xyzz_inf();
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t w = TREE / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            G1Xyzz o = sh[threadIdx.x + w];
            pin(o);
            acc = xyzz_add(acc, o);
            sh[threadIdx.x] = acc;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) st_xyzz(out + (uint64_t)g * gridDim.x + blockIdx.x, acc);
}

// --- fixed-base precomputation ------------------------------------------------------------
// tmp[i * W + w] = 2^(c*w) * P_i (XYZZ)
__global__ void k_precompute_windows(const G1Affine* pts, uint64_t n, uint32_t c, uint32_t W,
                                     G1Xyzz* tmp) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    G1Xyzz p = xyzz_from_affine(ld_affine(pts + i));
    for (uint32_t w = 0; w < W; w++) {
        st_xyzz(tmp + i * W + w, p);
        if (w + 1 < W)
            for (uint32_t k = 0; k < c; k++) p = xyzz_dbl(p);
    }
}

// XYZZ -> affine with Montgomery's batch inversion over chunks of BATCH consecutive points; the
// prefix products are parked in the outputs' x coordinates (no per-lane array, no scratch)
__global__ void k_batch_to_affine(const G1Xyzz* in, uint64_t m, G1Affine* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * BATCH;
    if (i0 >= m) return;
    const uint64_t i1 = min(i0 + BATCH, m);
    Fq acc = Fq::one();
    for (uint64_t i = i0; i < i1; i++) {
        st_vec(&out[i].x, acc);
        if (!ld_pinned(&in[i].ZZ).is_zero()) acc = mul(acc, ld_pinned(&in[i].ZZZ));
    }
    Fq inv = inverse(acc);
    for (uint64_t i = i1; i-- > i0;) {
        const G1Xyzz p = ld_xyzz(in + i);
        if (is_inf(p)) {
            st_affine(out + i, xyzz_to_affine_with_inv(p, Fq::zero()));
            continue;
        }
        const Fq inv_zzz = mul(inv, ld_pinned(&out[i].x));
        inv = mul(inv, p.ZZZ);
        st_affine(out + i, xyzz_to_affine_with_inv(p, inv_zzz));
    }
}

static uint32_t choose_c(uint64_t n, bool precomputed) {
    // minimise mixed additions n * ceil(255 / c) plus the bucket reduction, ~6 full additions
    // per bucket (per window when the windows keep their own buckets)
    uint32_t best = 4;
    double best_cost = 1e300;
    for (uint32_t c = 4; c <= 20; c++) {
        const double W = (255 + c - 1) / c;
        const double buckets = (double)(1u << (c - 1)) * (precomputed ? 1.0 : W);
        const double cost = (double)n * W + 6.0 * buckets;
        if (cost < best_cost) {
            best_cost = cost;
            best = c;
        }
    }
    return best;
}

static G1Affine g1_from_abi(const eon_g1_affine& a) {
    G1Affine r;
    for (int i = 0; i < 4; i++) {
        r.x.v[2 * i] = (uint32_t)a.x[i];
        r.x.v[2 * i + 1] = (uint32_t)(a.x[i] >> 32);
        r.y.v[2 * i] = (uint32_t)a.y[i];
        r.y.v[2 * i + 1] = (uint32_t)(a.y[i] >> 32);
    }
    return r;
}

static eon_g1_affine g1_to_abi(const G1Affine& a) {
    eon_g1_affine r;
    for (int i = 0; i < 4; i++) {
        r.x[i] = (uint64_t)a.x.v[2 * i] | (uint64_t)a.x.v[2 * i + 1] << 32;
        r.y[i] = (uint64_t)a.y.v[2 * i] | (uint64_t)a.y.v[2 * i + 1] << 32;
    }
    return r;
}

static bool fq_canonical(const Fq& x) {
    for (int i = 7; i >= 0; i--) {
        if (x.v[i] < FqP::P[i]) return true;
        if (x.v[i] > FqP::P[i]) return false;
    }
    return false;
}

static inline unsigned blocks_for(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_batch_to_affine(const G1Xyzz* in, uint64_t m, G1Affine* out, hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_batch_to_affine, dim3(blocks_for((m + BATCH - 1) / BATCH, 128)), dim3(128),
                       0, st, in, m, out);
    return hipGetLastError();
}

Status bases_create(eon_ctx* ctx, const eon_g1_affine* bases, uint64_t n, uint32_t flags,
                    bool device_ptr, eon_msm_bases** out) {
    if (!out) return Status::err(EON_E_ARG, "null output handle");
    if (n && !bases) return Status::err(EON_E_ARG, "null bases");
    if (n > (1ull << 27)) return Status::err(EON_E_SHAPE, "at most 2^27 bases");
    if (!device_ptr) {
        for (uint64_t i = 0; i < n; i++) {
            const G1Affine a = g1_from_abi(bases[i]);
            if (!fq_canonical(a.x) || !fq_canonical(a.y))
                return Status::err(EON_E_ARG, "base coordinate is not a canonical Fq");
        }
    }
    eon_msm_bases* b = new eon_msm_bases();
    b->ctx = ctx;
    b->n = n;
    hipStream_t st = ctx->stream;
    auto fail = [&](Status s) {
        b->points.release();
        b->table.release();
        delete b;
        return s;
    };
    hipError_t e = b->points.ensure((n ? n : 1) * sizeof(G1Affine));
    if (e != hipSuccess) return fail(Status::err(EON_E_OOM, "bases allocation failed"));
    if (n) {
        e = hipMemcpyAsync(b->points.p, bases, n * sizeof(G1Affine),
                           device_ptr ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st);
        if (e != hipSuccess) return fail(Status::err(EON_E_DEVICE, hipGetErrorString(e)));
    }
    b->precomputed = (flags & EON_MSM_PRECOMPUTE) != 0 && n > 0;
    b->c = choose_c(n ? n : 1, b->precomputed);
    b->windows = (255 + b->c - 1) / b->c;
    if (b->precomputed) {
        const uint64_t m = n * b->windows;
        DevBuf tmp;
        if (tmp.ensure(m * sizeof(G1Xyzz)) != hipSuccess ||
            b->table.ensure(m * sizeof(G1Affine)) != hipSuccess) {
            tmp.release();
            return fail(Status::err(EON_E_OOM, "precomputed table allocation failed"));
        }
        hipLaunchKernelGGL(k_precompute_windows, dim3(blocks_for(n, 128)), dim3(128), 0, st,
                           b->points.as<G1Affine>(), n, b->c, b->windows, tmp.as<G1Xyzz>());
        e = launch_batch_to_affine(tmp.as<G1Xyzz>(), m, b->table.as<G1Affine>(), st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        tmp.release();
        if (e != hipSuccess) return fail(Status::err(EON_E_DEVICE, hipGetErrorString(e)));
    }
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(Status::err(EON_E_DEVICE, hipGetErrorString(e)));
    *out = b;
    return Status::ok();
}

// One batch of `cols` MSMs of length n over bases[0..n): MSM j uses scalars[i * ld + j].
// Results (affine) are written to the device array `out_dev` (cols entries).
static Status msm_batch(eon_ctx* ctx, const eon_msm_bases* b, const Fr* scalars, uint64_t n,
                        uint64_t ld, uint32_t cols, G1Affine* out_dev) {
    hipStream_t st = ctx->stream;
    MsmWork& wk = ctx->msm;
    const uint32_t c = b->precomputed ? b->c : choose_c(n, false);
    const uint32_t W = b->precomputed ? b->windows : (255 + c - 1) / c;
    const uint32_t B = 1u << (c - 1);
    const uint32_t groups = b->precomputed ? cols : cols * W;
    const uint32_t nb = groups * B;
    const uint64_t E = n * W * cols;
    if (E >= (1ull << 32)) return Status::err(EON_E_SHAPE, "MSM too large for 32-bit pair indices");
    uint32_t key_bits = 1;
    while ((1ull << key_bits) <= nb) key_bits++;

    EON_HIP(wk.keys.ensure(E * 4));
    EON_HIP(wk.vals.ensure(E * 4));
    EON_HIP(wk.keys2.ensure(E * 4));
    EON_HIP(wk.vals2.ensure(E * 4));
    EON_HIP(wk.start.ensure((nb + 1) * 4ull));
    EON_HIP(wk.count.ensure((nb + 1) * 4ull));
    EON_HIP(wk.piece_off.ensure((nb + 1) * 4ull));
    size_t sort_bytes = 0, scan_bytes = 0;
    EON_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, wk.keys.as<uint32_t>(),
                                               wk.keys2.as<uint32_t>(), wk.vals.as<uint32_t>(),
                                               wk.vals2.as<uint32_t>(), (int)E, 0, key_bits, st));
    EON_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, wk.count.as<uint32_t>(),
                                             wk.piece_off.as<uint32_t>(), (int)(nb + 1), st));
    EON_HIP(wk.temp.ensure(std::max(sort_bytes, scan_bytes)));

    Profiler* prof = &ctx->prof;
    prof->begin("k_msm_digits", n * cols * 32 + E * 8, st);
    hipLaunchKernelGGL(k_msm_digits, dim3(blocks_for(n * cols, 256)), dim3(256), 0, st, scalars, n,
                       ld, cols, c, W, (uint32_t)b->precomputed, wk.keys.as<uint32_t>(),
                       wk.vals.as<uint32_t>());
    prof->end(st);
    EON_HIP(hipGetLastError());
    prof->begin("radix_sort_pairs", E * 16, st);
    EON_HIP(hipcub::DeviceRadixSort::SortPairs(wk.temp.p, sort_bytes, wk.keys.as<uint32_t>(),
                                               wk.keys2.as<uint32_t>(), wk.vals.as<uint32_t>(),
                                               wk.vals2.as<uint32_t>(), (int)E, 0, key_bits, st));
    prof->end(st);
    hipLaunchKernelGGL(k_bucket_start, dim3(blocks_for(E + 1, 256)), dim3(256), 0, st,
                       wk.keys2.as<uint32_t>(), E, nb, wk.start.as<uint32_t>());
    hipLaunchKernelGGL(k_level_count, dim3(blocks_for(nb + 1, 256)), dim3(256), 0, st,
                       wk.start.as<uint32_t>(), nb, wk.count.as<uint32_t>());
    EON_HIP(hipcub::DeviceScan::ExclusiveSum(wk.temp.p, scan_bytes, wk.count.as<uint32_t>(),
                                             wk.piece_off.as<uint32_t>(), (int)(nb + 1), st));
    const uint64_t max_pieces = E / PIECE + nb + 1;  // >= the real piece count
    EON_HIP(wk.owner.ensure(max_pieces * 4));
    EON_HIP(wk.piece_sums.ensure(max_pieces * sizeof(G1Xyzz)));
    EON_HIP(wk.bucket_sums.ensure((uint64_t)nb * sizeof(G1Xyzz)));
    EON_HIP(wk.off2.ensure((nb + 1) * 4ull));
    hipLaunchKernelGGL(k_piece_owner, dim3(blocks_for(nb, 256)), dim3(256), 0, st,
                       wk.piece_off.as<uint32_t>(), nb, wk.owner.as<uint32_t>());
    // launches are sized by the real counts (8-byte read-back: pieces, nonzero digits)
    uint32_t counts[2] = {0, 0};
    EON_HIP(hipMemcpyAsync(&counts[0], wk.piece_off.as<uint32_t>() + nb, 4, hipMemcpyDeviceToHost, st));
    EON_HIP(hipMemcpyAsync(&counts[1], wk.start.as<uint32_t>() + nb, 4, hipMemcpyDeviceToHost, st));
    EON_HIP(hipStreamSynchronize(st));
    uint32_t n_pieces = counts[0];
    const uint32_t n_pairs = counts[1];
    static const bool debug = getenv("EON_MSM_DEBUG") != nullptr;
    if (debug)
        fprintf(stderr, "msm_batch n=%llu cols=%u c=%u W=%u nb=%u E=%llu pairs=%u pieces=%u\n",
                (unsigned long long)n, cols, c, W, nb, (unsigned long long)E, n_pairs, n_pieces);
    const G1Affine* pts = b->precomputed ? b->table.as<G1Affine>() : b->points.as<G1Affine>();
    // algorithmic bytes: every nonzero digit reads its 4-byte reference and a 64-byte affine
    // base; every piece writes one 128-byte XYZZ partial
    prof->begin("k_piece_sum", (uint64_t)n_pairs * 68 + (uint64_t)n_pieces * 128, st);
    if (n_pieces)
        hipLaunchKernelGGL(k_piece_sum, dim3(blocks_for(n_pieces, 64)), dim3(64), 0, st,
                           wk.vals2.as<uint32_t>(), wk.start.as<uint32_t>(),
                           wk.piece_off.as<uint32_t>(), wk.owner.as<uint32_t>(), n_pieces, pts,
                           wk.piece_sums.as<G1Xyzz>());
    prof->end(st);
    // combine levels until every bucket holds one partial (skewed scalars put many pieces in a
    // bucket: all-equal scalars put n pieces in one bucket per window)
    uint32_t* off_cur = wk.piece_off.as<uint32_t>();
    uint32_t* off_nxt = wk.off2.as<uint32_t>();
    G1Xyzz* part_cur = wk.piece_sums.as<G1Xyzz>();
    EON_HIP(wk.piece_sums2.ensure(max_pieces * sizeof(G1Xyzz)));
    G1Xyzz* part_nxt = wk.piece_sums2.as<G1Xyzz>();
    for (int level = 0; level < 8; level++) {
        hipLaunchKernelGGL(k_level_count, dim3(blocks_for(nb + 1, 256)), dim3(256), 0, st, off_cur,
                           nb, wk.count.as<uint32_t>());
        EON_HIP(hipcub::DeviceScan::ExclusiveSum(wk.temp.p, scan_bytes, wk.count.as<uint32_t>(),
                                                 off_nxt, (int)(nb + 1), st));
        uint32_t n_new = 0;
        EON_HIP(hipMemcpyAsync(&n_new, off_nxt + nb, 4, hipMemcpyDeviceToHost, st));
        EON_HIP(hipStreamSynchronize(st));
        if (debug) fprintf(stderr, "  level %d: %u -> %u partials\n", level, n_pieces, n_new);
        if (n_new == n_pieces) break;  // every bucket already holds at most one partial
        hipLaunchKernelGGL(k_piece_owner, dim3(blocks_for(nb, 256)), dim3(256), 0, st, off_nxt, nb,
                           wk.owner.as<uint32_t>());
        prof->begin("k_partial_combine", (uint64_t)(n_pieces + n_new) * 128, st);
        hipLaunchKernelGGL(k_partial_combine, dim3(blocks_for(n_new, 64)), dim3(64), 0, st, off_cur,
                           off_nxt, wk.owner.as<uint32_t>(), n_new, part_cur, part_nxt);
        prof->end(st);
        std::swap(off_cur, off_nxt);
        std::swap(part_cur, part_nxt);
        n_pieces = n_new;
    }
    hipLaunchKernelGGL(k_bucket_final, dim3(blocks_for(nb, 256)), dim3(256), 0, st, off_cur, nb,
                       part_cur, wk.bucket_sums.as<G1Xyzz>());
    // sum_d d * B_d per group
    const uint32_t nseg = B / SEG;  // c >= 4, so B >= SEG
    EON_HIP(wk.red_a.ensure((uint64_t)groups * nseg * sizeof(G1Xyzz)));
    EON_HIP(wk.red_b.ensure((uint64_t)groups * nseg * sizeof(G1Xyzz)));
    prof->begin("k_segment_sum", (uint64_t)nb * 128 + (uint64_t)groups * nseg * 128, st);
    hipLaunchKernelGGL(k_segment_sum, dim3(blocks_for((uint64_t)nseg * groups, 64)), dim3(64), 0, st,
                       wk.bucket_sums.as<G1Xyzz>(), B, groups, wk.red_a.as<G1Xyzz>());
    prof->end(st);
    G1Xyzz* cur = wk.red_a.as<G1Xyzz>();
    G1Xyzz* nxt = wk.red_b.as<G1Xyzz>();
    uint32_t len = nseg;
    while (len > 1) {
        const uint32_t blk = (len + TREE - 1) / TREE;
        prof->begin("k_tree_sum", (uint64_t)groups * (len + blk) * 128, st);
        hipLaunchKernelGGL(k_tree_sum, dim3(blk, groups), dim3(TREE), 0, st, cur, len, nxt);
        prof->end(st);
        std::swap(cur, nxt);
        len = blk;
    }
    EON_HIP(hipGetLastError());
    // `cur` holds one point per group; per column: the group itself (fixed base) or the
    // Horner combination of its windows; then batched XYZZ -> affine on device
    G1Xyzz* per_col = cur;
    if (!b->precomputed) {
        hipLaunchKernelGGL(k_window_horner, dim3(blocks_for(cols, 64)), dim3(64), 0, st, cur, cols, W,
                           c, nxt);
        per_col = nxt;
    }
    EON_HIP(launch_batch_to_affine(per_col, cols, out_dev, st));
    return Status::ok();
}

Status msm_run_columns(eon_ctx* ctx, const eon_msm_bases* b, const Fr* scalars, uint64_t n,
                       uint32_t width, G1Affine* out_host) {
    if (n > b->n) return Status::err(EON_E_SHAPE, "more scalars than bases");
    if (width == 0) return Status::ok();
    if (n == 0) {  // G1::multi_exp returns the identity for empty input (curve.rs:163-165)
        for (uint32_t j = 0; j < width; j++) {
            out_host[j].x = Fq::zero();
            out_host[j].y = Fq::zero();
        }
        return Status::ok();
    }
    const uint32_t c = b->precomputed ? b->c : choose_c(n, false);
    const uint64_t W = (255 + c - 1) / c;
    // columns per batch: keep the digit pairs of one batch at <= 2^28 (4 GiB of sort buffers)
    uint64_t cpb = (1ull << 28) / (n * W);
    if (cpb < 1) cpb = 1;
    const uint64_t max_groups = b->precomputed ? cpb : cpb * W;
    if (max_groups > 65535) cpb = b->precomputed ? 65535 : 65535 / W;
    EON_HIP(ctx->msm.results.ensure(width * sizeof(G1Affine)));
    G1Affine* res = ctx->msm.results.as<G1Affine>();
    for (uint32_t j0 = 0; j0 < width; j0 += (uint32_t)cpb) {
        const uint32_t cols = (uint32_t)std::min<uint64_t>(cpb, width - j0);
        EON_TRY(msm_batch(ctx, b, scalars + j0, n, width, cols, res + j0));
    }
    EON_HIP(hipMemcpyAsync(out_host, res, width * sizeof(G1Affine), hipMemcpyDeviceToHost, ctx->stream));
    EON_HIP(hipStreamSynchronize(ctx->stream));
    return Status::ok();
}

Status msm_run(eon_ctx* ctx, const eon_msm_bases* b, const Fr* scalars, uint64_t n,
               G1Affine* result) {
    return msm_run_columns(ctx, b, scalars, n, 1, result);
}

}  // namespace eon

namespace {

int finish(eon_ctx* ctx, const Status& s) {
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

}  // namespace

extern "C" {

int eon_msm_bases_create(eon_ctx* ctx, const eon_g1_affine* bases, uint64_t n, uint32_t flags,
                         eon_msm_bases** out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    return finish(ctx, bases_create(ctx, bases, n, flags, false, out));
}

int eon_msm_bases_create_dev(eon_ctx* ctx, const eon_g1_affine* bases, uint64_t n, uint32_t flags,
                             eon_msm_bases** out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    return finish(ctx, bases_create(ctx, bases, n, flags, true, out));
}

void eon_msm_bases_destroy(eon_msm_bases* b) {
    if (!b) return;
    std::lock_guard<std::mutex> lk(b->ctx->mu);
    (void)hipSetDevice(b->ctx->device);
    (void)hipStreamSynchronize(b->ctx->stream);
    b->points.release();
    b->table.release();
    delete b;
}

uint64_t eon_msm_bases_len(const eon_msm_bases* b) { return b ? b->n : 0; }

int eon_msm_g1(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* scalars, uint64_t n,
               eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (!bases || !out || (n && !scalars)) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s;
    if (n > bases->n) {
        s = Status::err(EON_E_SHAPE, "more scalars than bases");
    } else {
        s = [&]() -> Status {
            EON_HIP(ctx->stage_in.ensure((n ? n : 1) * sizeof(Fr)));
            if (n)
                EON_HIP(hipMemcpyAsync(ctx->stage_in.p, scalars, n * sizeof(Fr),
                                       hipMemcpyHostToDevice, ctx->stream));
            G1Affine r;
            EON_TRY(msm_run(ctx, bases, ctx->stage_in.as<Fr>(), n, &r));
            *out = g1_to_abi(r);
            return Status::ok();
        }();
    }
    return finish(ctx, s);
}

int eon_msm_g1_dev(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* scalars, uint64_t n,
                   eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (!bases || !out || (n && !scalars)) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    G1Affine r;
    Status s = msm_run(ctx, bases, reinterpret_cast<const Fr*>(scalars), n, &r);
    if (!s.bad()) *out = g1_to_abi(r);
    return finish(ctx, s);
}

int eon_msm_g1_columns_dev(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* mat,
                           uint64_t rows, uint32_t width, eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (!bases || (width && !out) || (rows && width && !mat)) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    std::vector<G1Affine> r(width);
    Status s = msm_run_columns(ctx, bases, reinterpret_cast<const Fr*>(mat), rows, width, r.data());
    if (!s.bad())
        for (uint32_t j = 0; j < width; j++) out[j] = g1_to_abi(r[j]);
    return finish(ctx, s);
}

int eon_msm_g1_columns(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* mat, uint64_t rows,
                       uint32_t width, eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (!bases || (width && !out) || (rows && width && !mat)) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    std::vector<G1Affine> r(width);
    Status s = [&]() -> Status {
        if (rows > bases->n) return Status::err(EON_E_SHAPE, "more rows than bases");
        const size_t bytes = (size_t)rows * width * sizeof(Fr);
        EON_HIP(ctx->stage_in.ensure(bytes ? bytes : 32));
        if (bytes) EON_HIP(hipMemcpyAsync(ctx->stage_in.p, mat, bytes, hipMemcpyHostToDevice, ctx->stream));
        return msm_run_columns(ctx, bases, ctx->stage_in.as<Fr>(), rows, width, r.data());
    }();
    if (!s.bad())
        for (uint32_t j = 0; j < width; j++) out[j] = g1_to_abi(r[j]);
    return finish(ctx, s);
}

int eon_g1_multi_exp(eon_ctx* ctx, const eon_g1_affine* points, const eon_fr* scalars, uint64_t n,
                     eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (!out || (n && (!points || !scalars))) return EON_E_ARG;
    eon_msm_bases* b = nullptr;
    int rc = eon_msm_bases_create(ctx, points, n, 0, &b);
    if (rc) return rc;
    rc = eon_msm_g1(ctx, b, scalars, n, out);
    eon_msm_bases_destroy(b);
    return rc;
}

}  // extern "C"
