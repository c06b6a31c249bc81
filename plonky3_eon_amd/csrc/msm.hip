// Pippenger multi-scalar multiplication on BN254 G1 for gfx950.
//
// Replaces G1::multi_exp (bn254/src/curve.rs:158-179 -> halo2curves::msm::msm_best) and the KZG
// column commitment commit_column (kzg/src/util.rs:37-40).  The value sum_i s_i * P_i is unique,
// so the result (returned in affine form) is bit-identical to the reference's.
//
// Pipeline (all on device, one stream):
//   1. k_msm_digits     scalars (Montgomery) -> canonical -> signed c-bit digits; one
//                       (bucket key, point reference | sign) pair per nonzero digit.
//   2. radix sort       radix_sort_pairs (sort.hip: stable LSD, 8-bit digits, LDS-ranked tiles
//                       with a decoupled look-back) on the low c key bits of the
//                       group-major pairs: buckets b' = magnitude * groups + group, zero digits
//                       last (see k_msm_digits).
//   3. k_bucket_start   bucket boundaries in the sorted pairs.
//   4. pieces           a piece is the part of a bucket inside one chunk (2^log_chunk aligned
//                       sorted pairs); exclusive scan of the per-bucket piece counts.
//   5. k_piece_sum29    one thread per chunk of sorted pairs (every lane does the same number of
//                       XYZZ mixed additions of affine bases, radix 2^29), flushing a partial per
//                       piece.
//   6. k_partial_combine levels of <= PIECE-way sums until each bucket holds one partial
//                       (log-depth under any skew, e.g. all-equal scalars), k_bucket_final.
//   7. k_bucket_reduce29 sum_d d * B_d per group: T_j / U_j the plain / locally weighted sums of
//      (k_seg_level) /  segment j (SEG buckets, by running sums), then
//      k_group_finish   sum_j U_j + SEG sum_j j T_j + sum_j T_j per group (deferred to one launch
//                       per call).  Batches with < 64 groups (a single MSM) use the shorter-chain
//                       k_segment_sum (running sums + lo * run) + k_tree_sum instead: there
//                       latency, not additions, sets the time.
//   8. k_window_horner  (per-window buckets only) sum_w 2^(c*w) G_w per MSM; batched affine.
//
// Batched mode (eon_msm_g1_columns*): one pipeline run handles many MSMs at once -- the columns
// of a row-major coefficient matrix, as KzgPcs::commit commits every column against the same
// SRS prefix (kzg/src/pcs.rs:244-251) -- with the column index in the high bits of the key.
//
// Fixed-base mode (eon_msm_bases_create with EON_MSM_PRECOMPUTE; the KZG SRS): the bases object
// stores 2^(c*w) * P_i in affine for every window w, so every window's digits land in ONE bucket
// set (groups = 1): no per-window bucket reduction and no serial doubling chain at the end.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "context.h"
#include "ec.h"
#include "ec29.h"
#include "msm.h"
#include "sort.h"
#include "sort_pass.h"
#include "fq_host.h"

using namespace eon;

struct eon_msm_bases {
    eon_ctx* ctx = nullptr;
    uint64_t n = 0;
    DevBuf points;  // n affine bases
    bool precomputed = false;
    uint32_t c = 0, windows = 0;
    DevBuf table;  // precomputed: n * windows affine points, entry i * windows + w = 2^(c*w) P_i
    // the piece sums read 29-Montgomery coordinates from `table` (precomputed) or `points29`;
    // `points` stays in the ABI form (the KZG opening bases are derived from it)
    DevBuf points29;
    // 3 * table (29-form affine, same layout), built on first use by the KZG opening bases'
    // radix-4 fixed-base multiplications (bases_table3_29)
    DevBuf table3;
    // points / table come from (and return to) the context's DevPool (the opening bases)
    bool pooled = false;
    const G1Affine* piece_source() const {
        return precomputed ? table.as<G1Affine>() : points29.as<G1Affine>();
    }
};

namespace eon {

// sorted pairs per k_piece_sum thread: 2^log_chunk, sized so a batch launches ~2^20 threads
// (>= 4 waves on every SIMD) within [2^4, 2^7]
constexpr uint32_t LOG_CHUNK_MIN = 4, LOG_CHUNK_MAX = 7;
// a batch's chunks grow while its piece sums keep >= 2^EON_PIECE_THREADS_LOG threads
#ifndef EON_PIECE_THREADS_LOG
#define EON_PIECE_THREADS_LOG 20
#endif
constexpr uint32_t PIECE = 32;   // partials per combine step
constexpr uint32_t SEG = 8;     // buckets per reduction segment
// buckets per segment of the call-wide (deferred-finish) reduction: k_bucket_reduce29 walks RED_SEG
// buckets per lane, k_group_finish29 combines B / RED_SEG segments per group
#ifndef EON_RED_SEG
#define EON_RED_SEG 8
#endif
constexpr uint32_t RED_SEG = EON_RED_SEG;
constexpr uint32_t TREE = 256;  // points per tree-reduction block
constexpr uint32_t FINISH_THREADS = 256;  // threads per group of k_group_finish / k_group_finish29

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

// Digit pairs.  Key of a nonzero digit: (group << c) | (|digit| - 1), group = the column
// (fixed-base mode: every window shares the column's bucket set) or (column, window); zero digits
// get the sentinel 0xFFFFFFFF.  Pairs are emitted group-major (e = group * n + i: (col * W + w) * n
// + i in both modes) and radix-sorted on the low c key bits only -- 2 passes of the stable
// onesweep instead of 3 on the full key -- so equal magnitudes stay in group order: the sorted
// pairs run over buckets b' = (|digit| - 1) * groups + group, each contiguous.
constexpr uint32_t DIGIT_COLS = 4;  // widest scalar tile of one 256-thread block: 64 rows x 4 cols

// The digit sort's per-pass histograms of the keys (radix_sort_histograms) are counted here, in
// LDS per block and added to the global bins once per block, so the sort never re-reads the keys
// for them.  Blocks walk row tiles grid-stride (the grid is capped near DIGIT_BLOCKS): every block
// adds its bins to the same few hundred global counters, so one block per tile would put
// ~E / 8 atomics on those addresses.
constexpr uint32_t DIGIT_BLOCKS = 4096;

// canonical x from its Montgomery form x 2^256 (any 256-bit input): the radix-2^29 product by the
// plain integer 32 is x 2^256 32 2^-261 = x, under half the instructions of the radix-2^32
// to_canonical
__device__ __forceinline__ Fr canonical_from_mont(const Fr& a) {
    F29 thirty_two;
#pragma unroll
    for (int j = 0; j < 9; j++) thirty_two.l[j] = j == 0 ? 32u : 0u;
    return pack29<FrP>(canon29<FrP>(mul29<FrP>(unpack29(a), thirty_two)));
}

__global__ void __launch_bounds__(256) k_msm_digits(const Fr* scalars, uint64_t n, uint64_t ld,
                                                    uint32_t cols, uint32_t c, uint32_t windows,
                                                    uint32_t ref_windows, uint32_t precomputed,
                                                    uint32_t tile_cols, uint32_t* keys, uint32_t* vals,
                                                    RadixPasses pb, uint32_t* hist, Fr* /* k_msm_digits4's */) {
    __shared__ uint32_t h[RADIX_SORT_MAX_PASSES][256];
    for (uint32_t j = threadIdx.x; j < RADIX_SORT_MAX_PASSES * 256; j += 256) (&h[0][0])[j] = 0;
    __syncthreads();
    // a tile is 256 / tile_cols row segments of tile_cols adjacent columns (up to 128 contiguous
    // bytes), so the group-major writes stay in runs of consecutive rows
    const uint32_t col = blockIdx.y * tile_cols + threadIdx.x % tile_cols;
    const uint32_t rows = 256 / tile_cols;
    const uint32_t B = 1u << (c - 1);
    for (uint64_t i = (uint64_t)blockIdx.x * rows + threadIdx.x / tile_cols; col < cols && i < n;
         i += (uint64_t)gridDim.x * rows) {
        Fr s = canonical_from_mont(ld_pinned(scalars + i * ld + col));
        pin(s);
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
            const uint64_t e = ((uint64_t)col * windows + w) * n + i;
            uint32_t key;
            if (mag == 0) {
                key = 0xFFFFFFFFu;
                vals[e] = 0;
            } else {
                const uint32_t g = precomputed ? col : col * windows + w;
                key = (g << c) | (mag - 1);
                const uint32_t ref = precomputed ? (uint32_t)(i * ref_windows + w) : (uint32_t)i;
                vals[e] = ref | (neg << 31);
            }
            keys[e] = key;
#pragma unroll
            for (uint32_t p = 0; p < RADIX_SORT_MAX_PASSES; p++)
                if (p < pb.passes) atomicAdd(&h[p][(key >> pb.shift[p]) & ((1u << pb.bits[p]) - 1)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < pb.passes * 256; j += 256) {
        const uint32_t v = (&h[0][0])[j];
        if (v) atomicAdd(hist + j, v);
    }
}

// The same pairs with four consecutive rows per thread (n a multiple of 4): a lane writes a
// window's four keys and four references as one 16-byte store each, so a store instruction covers
// tile_cols runs of 16 * 4 rows (256 contiguous bytes per column) instead of tile_cols runs of 64
// bytes.  A tile is 256 / tile_cols row quads of tile_cols adjacent columns.  WRITE = false: the
// histograms and the canonical scalars column-major (canon[col n + i]) instead of the pairs, for
// the fused first sort pass (k_digit_sort_pass computes the pairs again from them).
template <bool WRITE>
__global__ void __launch_bounds__(256) k_msm_digits4(const Fr* scalars, uint64_t n, uint64_t ld,
                                                     uint32_t cols, uint32_t c, uint32_t windows,
                                                     uint32_t ref_windows, uint32_t precomputed,
                                                     uint32_t tile_cols, uint32_t* keys, uint32_t* vals,
                                                     RadixPasses pb, uint32_t* hist, Fr* canon) {
    __shared__ uint32_t h[RADIX_SORT_MAX_PASSES][256];
    for (uint32_t j = threadIdx.x; j < RADIX_SORT_MAX_PASSES * 256; j += 256) (&h[0][0])[j] = 0;
    __syncthreads();
    const uint32_t col = blockIdx.y * tile_cols + threadIdx.x % tile_cols;
    const uint32_t quads = 256 / tile_cols;
    const uint32_t B = 1u << (c - 1);
    for (uint64_t i = ((uint64_t)blockIdx.x * quads + threadIdx.x / tile_cols) * 4; col < cols && i < n;
         i += (uint64_t)gridDim.x * quads * 4) {
        Fr s[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            s[r] = canonical_from_mont(ld_pinned(scalars + (i + r) * ld + col));
            pin(s[r]);
        }
        if (!WRITE) {  // the canonical scalars, column-major, for the fused first sort pass
#pragma unroll
            for (int r = 0; r < 4; r++) st_vec(canon + (uint64_t)col * n + i + r, s[r]);
        }
        uint32_t carry[4] = {0, 0, 0, 0};
        for (uint32_t w = 0; w < windows; w++) {
            uint32_t key[4], val[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t raw = window_bits(s[r].v, w * c, c) + carry[r];
                uint32_t mag, neg;
                if (raw > B) {  // signed digit raw - 2^c in [-(B-1), -1], carry into the next window
                    mag = (1u << c) - raw;
                    neg = 1;
                    carry[r] = 1;
                } else {
                    mag = raw;
                    neg = 0;
                    carry[r] = 0;
                }
                if (mag == 0) {
                    key[r] = 0xFFFFFFFFu;
                    val[r] = 0;
                } else {
                    const uint32_t g = precomputed ? col : col * windows + w;
                    key[r] = (g << c) | (mag - 1);
                    const uint32_t ref = precomputed ? (uint32_t)((i + r) * ref_windows + w) : (uint32_t)(i + r);
                    val[r] = ref | (neg << 31);
                }
#pragma unroll
                for (uint32_t p = 0; p < RADIX_SORT_MAX_PASSES; p++)
                    if (p < pb.passes) atomicAdd(&h[p][(key[r] >> pb.shift[p]) & ((1u << pb.bits[p]) - 1)], 1u);
            }
            if (WRITE) {
                const uint64_t e = ((uint64_t)col * windows + w) * n + i;
                *reinterpret_cast<uint4*>(keys + e) = make_uint4(key[0], key[1], key[2], key[3]);
                *reinterpret_cast<uint4*>(vals + e) = make_uint4(val[0], val[1], val[2], val[3]);
            }
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < pb.passes * 256; j += 256) {
        const uint32_t v = (&h[0][0])[j];
        if (v) atomicAdd(hist + j, v);
    }
}

// The first (low-byte) pass of the digit sort fused with the digit extraction, for fixed-base
// tables with c = 16 and 16 windows: the pairs are ranked as they are computed from the scalars,
// never written unsorted nor read back (k_msm_digits4 + the first k_sort_pass moved 8 + 16 bytes
// per pair; this pass reads 2 of canonical scalar, coalesced, and writes 8; the histogram kernel
// before it writes the canonical scalars column-major).  Tile t covers rows [r0, r0 + SORT_THREADS)
// of column col = t / tiles_per_col (r0 = (t % tiles_per_col) SORT_THREADS, n a multiple of
// SORT_THREADS): thread (w, lane) takes row r0 + 64 w + lane and its 16 window digits are its 16
// items.  Within a column the pairs are ranked in another order than k_msm_digits' (window-major),
// but the tiles run column by column, so after both passes every bucket (digit, column) is still
// one contiguous run -- the only order the piece sums rely on (a bucket's sum is order-free).
struct DigitSource {
    const Fr* canon;  // canonical scalars, column-major (k_msm_digits4<false>)
    uint64_t n;
    uint32_t tiles_per_col, ref_windows;
    template <bool FULL>
    __device__ __forceinline__ void load(uint32_t tile, uint32_t w, uint32_t lane, uint32_t,
                                         uint32_t (&key)[sortpass::SORT_ITEMS],
                                         uint32_t (&val)[sortpass::SORT_ITEMS]) const {
        static_assert(sortpass::SORT_ITEMS == 16, "one item per 16-bit window of a 256-bit scalar");
        const uint32_t col = tile / tiles_per_col;
        const uint64_t i = (uint64_t)(tile - col * tiles_per_col) * sortpass::SORT_THREADS + w * 64 + lane;
        const Fr s = ld_pinned(canon + (uint64_t)col * n + i);
        uint32_t carry = 0;
#pragma unroll
        for (uint32_t j = 0; j < 16; j++) {
            const uint32_t raw = ((s.v[j >> 1] >> (16 * (j & 1))) & 0xffffu) + carry;
            uint32_t mag, neg;
            if (raw > (1u << 15)) {  // signed digit raw - 2^16, carry into the next window
                mag = (1u << 16) - raw;
                neg = 1;
                carry = 1;
            } else {
                mag = raw;
                neg = 0;
                carry = 0;
            }
            key[j] = mag ? (col << 16 | (mag - 1)) : 0xFFFFFFFFu;
            val[j] = mag ? ((uint32_t)(i * ref_windows + j) | neg << 31) : 0u;
        }
    }
};

// The lean tile's source (EON_SORT_LEAN, sort_pass.h): LEAN_THREADS x 2 pairs per tile, i.e.
// LEAN_THREADS / 8 rows of one column; thread t takes row r0 + t % R and the windows 2 (t / R),
// 2 (t / R) + 1 (R = LEAN_THREADS / 8), both in the scalar's word t / R.  The carry into window 2j
// of the signed recoding is 1 exactly when the scalar's low 32 j bits exceed 0x8000...8000 (every
// 16-bit window at 2^15: the largest low part the digits [-(2^15 - 1), 2^15] represent), a
// comparison the words below decide from the top -- almost always word j - 1 alone.
struct DigitSourceLean {
    const Fr* canon;
    uint64_t n;
    uint32_t tiles_per_col, ref_windows;
    template <bool FULL, uint32_t THREADS, uint32_t ITEMS>
    __device__ __forceinline__ void load(uint32_t tile, uint32_t w, uint32_t lane, uint32_t, uint32_t (&key)[ITEMS],
                                         uint32_t (&val)[ITEMS]) const {
        static_assert(ITEMS == 2, "two 16-bit windows per thread");
        constexpr uint32_t R = THREADS / 8;  // rows per tile
        const uint32_t t = w * 64 + lane;
        const uint32_t col = tile / tiles_per_col;
        const uint64_t i = (uint64_t)(tile - col * tiles_per_col) * R + t % R;
        const uint32_t j = t / R;  // the scalar's word: windows 2 j, 2 j + 1
        const uint32_t* s = reinterpret_cast<const uint32_t*>(canon + (uint64_t)col * n + i);
        const uint32_t word = s[j];
        uint32_t carry = 0;
        for (int k = (int)j - 1; k >= 0; k--) {  // low part > 0x8000..8000 ?
            const uint32_t x = s[k];
            if (x != 0x80008000u) {
                carry = x > 0x80008000u;
                break;
            }
        }
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t raw = ((word >> (16 * h)) & 0xffffu) + carry;
            uint32_t mag, neg;
            if (raw > (1u << 15)) {
                mag = (1u << 16) - raw;
                neg = 1;
                carry = 1;
            } else {
                mag = raw;
                neg = 0;
                carry = 0;
            }
            key[h] = mag ? (col << 16 | (mag - 1)) : 0xFFFFFFFFu;
            val[h] = mag ? ((uint32_t)(i * ref_windows + 2 * j + h) | neg << 31) : 0u;
        }
    }
};

__global__ void __launch_bounds__(sortpass::LEAN_THREADS) k_digit_sort_pass_lean(DigitSourceLean src, uint32_t* kd,
                                                                                 uint32_t* vd, uint32_t n, uint32_t shift,
                                                                                 const uint32_t* base, uint64_t* status,
                                                                                 uint32_t* tile_ctr) {
    sortpass::sort_pass_tile<8, DigitSourceLean, sortpass::LEAN_THREADS, sortpass::LEAN_ITEMS>(src, kd, vd, n, shift, 8,
                                                                                             base, status, tile_ctr);
}

__global__ void __launch_bounds__(sortpass::SORT_THREADS) k_digit_sort_pass(DigitSource src, uint32_t* kd, uint32_t* vd,
                                                                            uint32_t n, uint32_t shift,
                                                                            const uint32_t* base, uint64_t* status,
                                                                            uint32_t* tile_ctr) {
    sortpass::sort_pass_tile<8>(src, kd, vd, n, shift, 8, base, status, tile_ctr);
}

// OR of every canonical scalar into or_out[8] (zeroed before): its top set bit bounds the
// digits a single MSM needs (active windows, msm_run_columns)
constexpr uint32_t SCALAR_OR_COPIES = 64;
__global__ void __launch_bounds__(256) k_scalar_or(const Fr* scalars, uint64_t n, uint32_t* or_out) {
    __shared__ uint32_t acc[8];
    if (threadIdx.x < 8) acc[threadIdx.x] = 0;
    __syncthreads();
    uint32_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const Fr s = canonical_from_mont(ld_pinned(scalars + i));
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] |= s.v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
        uint32_t x = v[j];
        for (int o = 32; o > 0; o >>= 1) x |= (uint32_t)__shfl_xor(x, o);
        if ((threadIdx.x & 63) == 0 && x) atomicOr(&acc[j], x);
    }
    __syncthreads();
    // SCALAR_OR_COPIES copies of the 8 words (block b ORs into copy b % SCALAR_OR_COPIES): few
    // atomics per address -- one copy's 32k atomics from 4096 blocks took 56 us (profiles/r05/s14)
    if (threadIdx.x < 8 && acc[threadIdx.x])
        atomicOr(or_out + (blockIdx.x % SCALAR_OR_COPIES) * 8 + threadIdx.x, acc[threadIdx.x]);
}

// bucket index b' of a sorted key (nb for the zero-digit sentinel)
__device__ __forceinline__ uint32_t bucket_of(uint32_t key, uint32_t c, uint32_t groups, uint32_t nb) {
    return key == 0xFFFFFFFFu ? nb : (key & ((1u << (c - 1)) - 1)) * groups + (key >> c);
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

// start[b'] = index of the first sorted pair in bucket >= b', for b' in [0, nb]; each thread
// handles BS_KEYS consecutive pairs, its BS_KEYS / 4 16-byte loads issued together (more bytes in
// flight per wave: one 16-byte load per thread ran the kernel at ~3.8 TB/s), plus the key before
// its range; E a multiple of 4 (the MSM's pair counts), a partial last group per element
constexpr uint32_t BS_KEYS = 16;
__global__ void __launch_bounds__(256) k_bucket_start(const uint32_t* keys, uint64_t E, uint32_t c, uint32_t groups,
                                                      uint32_t nb, uint32_t* start) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * BS_KEYS;
    if (i0 > E) return;
    uint32_t k[BS_KEYS];
    if (i0 + BS_KEYS <= E && (E & 3) == 0) {
#pragma unroll
        for (uint32_t q = 0; q < BS_KEYS / 4; q++) {
            const uint4 v = *reinterpret_cast<const uint4*>(keys + i0 + 4 * q);
            k[4 * q] = v.x; k[4 * q + 1] = v.y; k[4 * q + 2] = v.z; k[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (uint32_t j = 0; j < BS_KEYS; j++) k[j] = i0 + j < E ? keys[i0 + j] : 0u;
    }
    int64_t prev = i0 == 0 ? -1 : (int64_t)bucket_of(keys[i0 - 1], c, groups, nb);
#pragma unroll
    for (uint32_t j = 0; j < BS_KEYS; j++) {
        const uint64_t i = i0 + j;
        if (i > E) break;
        const int64_t cur = i == E ? (int64_t)nb : (int64_t)bucket_of(k[j], c, groups, nb);
        for (int64_t b = prev + 1; b <= cur; b++) start[b] = (uint32_t)i;
        prev = cur;
    }
}

__global__ void k_piece_owner(const uint32_t* piece_off, uint32_t nb, uint32_t* owner) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    for (uint32_t p = piece_off[b]; p < piece_off[b + 1]; p++) owner[p] = b;
}

#ifndef EON_PIECE_MINWAVES
#define EON_PIECE_MINWAVES 4
#endif
// EON_PIECE_NEGSUM=0 builds the round-5 loop (madd29_unchecked, radix-2^32 base negation): A/B
#ifndef EON_PIECE_NEGSUM
#define EON_PIECE_NEGSUM 1
#endif
// EON_PIECE_MERGE: the two pieces of every bucket straddling one chunk boundary are summed into
// the first before k_bucket_reduce29, which then reads one piece for such a bucket -- 2 (default):
// by k_piece_sum29's lane t for the boundary with lane t + 1 of its wave, and by k_piece_merge29
// for the boundaries between waves; 1: all by k_piece_merge29; 0: the reduction sums them itself
#ifndef EON_PIECE_MERGE
#define EON_PIECE_MERGE 2
#endif

// Thread t sums the sorted pairs [t 2^log_chunk, (t+1) 2^log_chunk) (nonzero digits only): one
// partial per bucket run, stored at piece_off[b] + t - (start[b] >> log_chunk).  The XYZZ
// accumulator is in 29-bit limbs (ec29.h: lazy bounds, no carry captures in the products) and the
// bases are read in 29-Montgomery form (k_table_to29).  Each bucket run stores its raw accumulator (144 bytes,
// ZZ = 0 for the identity); k_raw29_to_xyzz converts the pieces for the combine levels.
//
// The additions are unchecked (madd29_unchecked): x(acc) == x(A) -- a duplicate base, or a base
// meeting its negation -- leaves ZZ = 0 mod p for the rest of the run, so the run's ZZ is tested
// once at its flush and such a run is summed again with the checked additions (piece_run29).
// An identity base ((0, 0) in the table) is recognised by y = 0 alone: G1 has prime order, so no
// curve point has y = 0.

// sum of the bases of sorted pairs [e_begin, e_end) with every exceptional case resolved;
// returns whether the sum is the identity
__device__ __forceinline__ bool piece_run29(const uint32_t* vals, const G1Affine* pts29, uint32_t e_begin,
                                            uint32_t e_end, G1X29& acc) {
    bool inf = true;
    for (uint32_t e = e_begin; e < e_end; e++) {
        const uint32_t v = vals[e];
        G1Affine a = ld_affine(pts29 + (v & 0x7fffffffu));
        if (a.y.is_zero()) continue;
        if (v >> 31) a.y = neg(a.y);
        const F29 ax = unpack29(a.x), ay = unpack29(a.y);
        if (inf) {
            acc.X = ax;
            acc.Y = ay;
            acc.ZZ = const29<FqP>(R29<FqP>::ONE);
            acc.ZZZ = acc.ZZ;
            inf = false;
        } else if (!madd29(acc, ax, ay)) {
            inf = madd29_exceptional(acc, ax, ay);
        }
    }
    return inf;
}

__global__ void __launch_bounds__(64, EON_PIECE_MINWAVES) k_piece_sum29(
    const uint32_t* keys, const uint32_t* vals, const uint32_t* start, const uint32_t* piece_off,
    uint32_t log_chunk, uint32_t c, uint32_t groups, uint32_t nb, const G1Affine* pts29, G1Raw29* piece_raw) {
    // the nonzero-digit pairs (start[nb]): read here, so that the launch need not wait for the
    // count read-back (the grid covers every pair of the batch)
    const uint32_t n_pairs = start[nb];
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; ((uint64_t)t << log_chunk) < n_pairs;
         t += gridDim.x * blockDim.x) {
        const uint32_t e0 = t << log_chunk;
        const uint32_t e1 = min(e0 + (1u << log_chunk), n_pairs);
        uint32_t b = keys[e0];
        uint32_t run = e0;  // first pair of the current bucket run
        G1X29 acc;
        bool inf = true;
#if EON_PIECE_NEGSUM
        // the accumulator holds (-1)^flip times the run's sum (madd29_negsum returns the negated
        // sum; a run opening with a negative digit starts from the unnegated base with flip set)
        bool flip = false;
#endif
        auto flush = [&](uint32_t e_end) __attribute__((always_inline)) {
            if (!inf && is_zero_mod29<FqP>(acc.ZZ)) {
                inf = piece_run29(vals, pts29, run, e_end, acc);
#if EON_PIECE_NEGSUM
                flip = false;
#endif
            }
#if EON_PIECE_NEGSUM
            if (flip) acc.ZZZ = neg29_lazy<3>(acc.ZZZ);  // ZZZ < 2p normalised -> 3p - ZZZ
#endif
            const uint32_t bb = bucket_of(b, c, groups, nb);
            G1Raw29* dst = piece_raw + piece_off[bb] + t - (start[bb] >> log_chunk);
#if EON_PIECE_NEGSUM
            // an identity piece is any raw accumulator with ZZ = 0 (every reader tests ZZ alone):
            // one store of acc either way, instead of selecting all 36 words between acc and zeros
            if (inf) acc.ZZ = F29{};
            st_raw29(dst, acc);
#else
            if (inf)
                st_raw29_inf(dst);
            else
                st_raw29(dst, acc);
#endif
        };
#ifndef EON_PIECE_SCALAR_PAIRS
        // 16-byte loads of four keys and four references every fourth pair (chunks are aligned to
        // 2^LOG_CHUNK_MIN pairs; a chunk cut short by n_pairs reads one pair at a time): a quarter
        // of the pair-stream requests (prove -2.5 % A/B; EON_PIECE_SCALAR_PAIRS restores the
        // one-pair loads)
        const bool vec = ((e0 | e1) & 3) == 0;
        uint4 kq = make_uint4(0, 0, 0, 0), vq = kq;
#endif
        for (uint32_t e = e0;; e++) {
            // one flush site (the run's end or the chunk's), so the checked re-sum is emitted once
            const bool last = e == e1;
#ifndef EON_PIECE_SCALAR_PAIRS
            // the pair is always picked from the register quads (a chunk cut short reloads
            // component 0 every pair): a pick written as "vec ? quad component : *p" was compiled
            // as one load through a selected pointer, which kept the quads in scratch (eight
            // scratch stores per quad, a flat load and a wait per pair)
            const uint32_t sub = vec ? (e & 3) : 0;
            if (!last && sub == 0) {
                if (vec) {
                    kq = *reinterpret_cast<const uint4*>(keys + e);
                    vq = *reinterpret_cast<const uint4*>(vals + e);
                } else {
                    kq.x = keys[e];
                    vq.x = vals[e];
                }
            }
            auto pick = [&](const uint4& q) __attribute__((always_inline)) {
                return sub == 0 ? q.x : sub == 1 ? q.y : sub == 2 ? q.z : q.w;
            };
            const uint32_t k = last ? b : pick(kq);
#else
            const uint32_t k = last ? b : keys[e];
#endif
            if (last || k != b) {
                flush(e);
                if (last) break;
                inf = true;
                b = k;
                run = e;
            }
#ifndef EON_PIECE_SCALAR_PAIRS
            const uint32_t v = pick(vq);
#else
            const uint32_t v = vals[e];
#endif
#ifdef EON_PIECE_PROBE_MASK
            // memory-sensitivity probe (tuning builds only, wrong results): every gather from a
            // cache-resident slice of the table
            G1Affine a = ld_affine(pts29 + (v & EON_PIECE_PROBE_MASK));
#else
            G1Affine a = ld_affine(pts29 + (v & 0x7fffffffu));
#endif
            if (a.y.is_zero()) continue;
#if EON_PIECE_NEGSUM
            // the digit's sign and the accumulator's are applied together, as one lazy negation of
            // the base's y in radix 2^29 (9 subtractions and 9 selects instead of a borrow chain)
            const bool neg_digit = v >> 31;
            const F29 ax = unpack29(a.x), ay = unpack29(a.y);
            if (inf) {
                acc.X = ax;
                acc.Y = ay;
                acc.ZZ = const29<FqP>(R29<FqP>::ONE);
                acc.ZZZ = acc.ZZ;
                flip = neg_digit;
                inf = false;
            } else {
                const F29 ayn = neg29_lazy<2>(ay);
                const bool ng = neg_digit != flip;
                F29 ys;
#pragma unroll
                for (int i = 0; i < 9; i++) ys.l[i] = ng ? ayn.l[i] : ay.l[i];
                madd29_negsum(acc, ax, ys);
                flip = !flip;
            }
#else
            if (v >> 31) a.y = neg(a.y);
            const F29 ax = unpack29(a.x), ay = unpack29(a.y);
            if (inf) {
                acc.X = ax;
                acc.Y = ay;
                acc.ZZ = const29<FqP>(R29<FqP>::ONE);
                acc.ZZZ = acc.ZZ;
                inf = false;
            } else {
                madd29_unchecked(acc, ax, ay);
            }
#endif
        }
#if EON_PIECE_MERGE == 2
        // acc holds the chunk's last piece as stored.  When its bucket goes on into the next chunk
        // and ends there (two pieces), lane t + 1 of this wave stored the bucket's second piece
        // at its first flush -- earlier in this wave's instruction stream, every lane's pair loop
        // having ended -- so lane t sums it in here (k_piece_merge29 covers lane 63's boundary)
        if (e1 < n_pairs && ((t + 1) & 63u) != 0 && keys[e1] == b) {
            const uint32_t bb = bucket_of(b, c, groups, nb);
            const uint32_t p0 = piece_off[bb];
            if (piece_off[bb + 1] - p0 == 2) {
                __threadfence_block();
                G1X29 x;
                const bool x_inf = ld_raw29(piece_raw + p0 + 1, x);
                acc29(acc, inf, x, x_inf);
                if (inf) acc.ZZ = F29{};
                st_raw29(piece_raw + p0, acc);
                // the second piece becomes the identity, for the reductions that read every piece
                st_raw29_inf(piece_raw + p0 + 1);
            }
        }
#endif
    }
}

__global__ void k_raw29_to_xyzz(const G1Raw29* in, uint32_t n, G1Xyzz* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    st_xyzz(out + i, raw29_to_xyzz(in + i));
}

// affine points (canonical radix-2^32 Montgomery) -> 29-Montgomery in place; (0, 0) stays
__global__ void k_table_to29(G1Affine* pts, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    G1Affine a = ld_affine(pts + i);
    a.x = to_fq261(a.x);
    a.y = to_fq261(a.y);
    st_affine(pts + i, a);
}

// One combine level: new partial p of bucket b sums old partials
// [off_old[b] + PIECE*j, min(+PIECE, off_old[b+1])), j = p - off_new[b].
// The launch covers an upper bound of the new partial count; the count itself is off_new[nb].
__global__ void k_partial_combine(const uint32_t* off_old, const uint32_t* off_new,
                                  const uint32_t* owner, uint32_t nb, const G1Xyzz* in,
                                  G1Xyzz* out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= off_new[nb]) return;
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
__global__ void k_bucket_final(const uint32_t* off, uint32_t B, uint32_t groups,
                               const G1Xyzz* partials, G1Xyzz* bucket_sums) {
    // bucket_sums is column-major (group * B + m) for the reduction; partials follow b' order
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B * groups) return;
    const uint32_t bp = (b % B) * groups + b / B;
    st_xyzz(bucket_sums + b, off[bp + 1] > off[bp] ? ld_xyzz(partials + off[bp]) : xyzz_inf());
}

// Segment s of group g covers buckets [lo, lo + SEG) (bucket b holds digit b + 1):
// out = sum_b (b + 1) * S_b = (running-sum form) + lo * (sum_b S_b).  The latency-optimal form
// for few groups (one short chain per segment, one tree): used when a batch has < 64 groups.
__global__ void __launch_bounds__(64) k_segment_sum(const G1Xyzz* bucket_sums, uint32_t B,
                                                    uint32_t groups, G1Xyzz* seg_out) {
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

// One level of the weighted bucket sum: segment j of group g covers x = X[g L + j seg ..+ seg);
// T = sum_k x_k and U = sum_k k x_k, by running sums from the top (2 (seg - 1) + 1 additions).
__global__ void __launch_bounds__(64) k_seg_level(const G1Xyzz* X, uint32_t L, uint32_t seg, uint32_t groups, G1Xyzz* T,
                            G1Xyzz* U) {
    const uint32_t nseg = L / seg;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg * groups) return;
    const G1Xyzz* x = X + (uint64_t)(t / nseg) * L + (uint64_t)(t % nseg) * seg;
    G1Xyzz run = xyzz_inf(), acc = xyzz_inf();
    for (uint32_t k = seg - 1; k >= 1; k--) {
        run = xyzz_add(run, ld_xyzz(x + k));
        acc = xyzz_add(acc, run);
    }
    run = xyzz_add(run, ld_xyzz(x));
    st_xyzz(T + t, run);
    st_xyzz(U + t, acc);
}

// The first level of the weighted bucket sum fused with the bucket sums, straight from
// k_piece_sum29's raw partials (radix 2^29, lazy): segment s of group g covers magnitudes
// [s seg, s seg + seg); bucket m is the sum of its pieces [piece_off[b'], piece_off[b' + 1]),
// b' = m groups + g (<= PIECE of them: used when no combine level is needed).  Same T / U as
// k_seg_level over the bucket sums, at T[g nseg + s] / U[g nseg + s]; a wave covers consecutive
// groups of one segment, so its piece reads are adjacent.
// OutT = G1Xyzz (radix-2^32, canonical: the per-batch k_group_finish) or G1Raw29 (the raw lazy
// accumulator, ZZ = 0 for the identity: the call-wide k_group_finish29)
__device__ __forceinline__ void st_point(G1Xyzz* p, const G1X29& a, bool inf) { st_xyzz(p, x29_to_xyzz(a, inf)); }
__device__ __forceinline__ void st_point(G1Raw29* p, const G1X29& a, bool inf) {
    if (inf)
        st_raw29_inf(p);
    else
        st_raw29(p, a);
}

// Buckets whose pairs straddle exactly one chunk boundary hold two pieces (k_piece_sum29's thread
// t - 1 ends the bucket's first run, thread t starts its second): here they are summed into the
// first, one thread per chunk boundary, so that k_bucket_reduce29<.., true> reads one piece for
// every such bucket.  In the reduction a wave walks the buckets of a segment in step, one lane
// per group, and pays the most pieces any lane has per bucket -- two almost always (a bucket of
// ~64 sorted pairs straddles a 128-pair chunk boundary half of the time), so its three additions
// per bucket become two there, and this kernel's half addition per bucket runs with every lane
// busy.  Buckets spanning three or more chunks (rare) keep all their pieces.
// Thread i takes the boundary before chunk (i + 1) 2^log_step (log_step 6: the boundaries between
// k_piece_sum29's waves, the rest merged there).
__global__ void __launch_bounds__(64) k_piece_merge29(const uint32_t* keys, const uint32_t* start,
                                                      const uint32_t* piece_off, uint32_t log_chunk,
                                                      uint32_t log_step, uint32_t c, uint32_t groups, uint32_t nb,
                                                      G1Raw29* pieces) {
    const uint32_t n_pairs = start[nb];
    const uint64_t e0 = (uint64_t)(blockIdx.x * blockDim.x + threadIdx.x + 1) << (log_chunk + log_step);
    if (e0 >= n_pairs) return;
    const uint32_t k = keys[e0];
    if (keys[e0 - 1] != k) return;
    const uint32_t bb = bucket_of(k, c, groups, nb);
    const uint32_t p0 = piece_off[bb];
    if (piece_off[bb + 1] - p0 != 2) return;
    G1X29 a, x;
    bool a_inf = ld_raw29(pieces + p0, a);
    const bool x_inf = ld_raw29(pieces + p0 + 1, x);
    acc29(a, a_inf, x, x_inf);
    if (a_inf)
        st_raw29_inf(pieces + p0);
    else
        st_raw29(pieces + p0, a);
}

template <class OutT, bool MERGED = false>
__global__ void __launch_bounds__(64) k_bucket_reduce29(const G1Raw29* pieces, const uint32_t* piece_off,
                                                        uint32_t B, uint32_t seg, uint32_t groups, OutT* T,
                                                        OutT* U) {
    const uint32_t nseg = B / seg;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg * groups) return;
    const uint32_t g = t % groups, s = t / groups;
    G1X29 run, acc, x;
    bool run_inf = true, acc_inf = true;
    for (int k = (int)seg - 1; k >= 0; k--) {
        const uint32_t bp = (s * seg + (uint32_t)k) * groups + g;
        const uint32_t e0 = piece_off[bp];
        uint32_t e1 = piece_off[bp + 1];
        if (MERGED && e1 - e0 == 2) e1 = e0 + 1;  // k_piece_merge29 summed the two into the first
        for (uint32_t e = e0; e < e1; e++) {
            const bool inf = ld_raw29(pieces + e, x);
            acc29(run, run_inf, x, inf);
        }
        if (k >= 1) acc29(acc, acc_inf, run, run_inf);
    }
    st_point(T + (uint64_t)g * nseg + s, run, run_inf);
    st_point(U + (uint64_t)g * nseg + s, acc, acc_inf);
}

// k_group_finish in radix 2^29 over raw segment sums (k_bucket_reduce29<G1Raw29>): the same
// out[g] = sum_j U_j + 2^log_seg sum_j j T_j + sum_j T_j, with the 1.4x faster carry-free product
// and no radix conversion of the inputs; the LDS tree holds raw accumulators (144 B per thread).
template <uint32_t GF_THREADS>
__global__ void __launch_bounds__(GF_THREADS) k_group_finish29(const G1Raw29* T, const G1Raw29* U, uint32_t S,
                                                              uint32_t log_seg, G1Xyzz* out) {
    __shared__ G1Raw29 sh[GF_THREADS];
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    const uint32_t nt = S < GF_THREADS ? S : GF_THREADS;
    const uint32_t Q = S / nt;
    G1X29 c, x;
    bool c_inf = true;
    if (t < nt) {
        const G1Raw29* Tg = T + (uint64_t)g * S + (uint64_t)t * Q;
        const G1Raw29* Ug = U + (uint64_t)g * S + (uint64_t)t * Q;
        G1X29 run, acc, us;
        bool run_inf = true, acc_inf = true, us_inf = true;
        for (uint32_t k = Q - 1; k >= 1; k--) {
            const bool inf = ld_raw29(Tg + k, x);
            acc29(run, run_inf, x, inf);
            acc29(acc, acc_inf, run, run_inf);
        }
        {
            const bool inf = ld_raw29(Tg, x);
            acc29(run, run_inf, x, inf);
        }
        for (uint32_t k = 0; k < Q; k++) {
            const bool inf = ld_raw29(Ug + k, x);
            acc29(us, us_inf, x, inf);
        }
        const uint32_t lo = t * Q;
        if (lo && !run_inf) {  // acc += lo * run (double-and-add, MSB first)
            G1X29 m;
            bool m_inf = true;
            for (int bit = 31 - __builtin_clz(lo); bit >= 0; bit--) {
                if (!m_inf) dbl29(m);
                if ((lo >> bit) & 1) acc29(m, m_inf, run, false);
            }
            acc29(acc, acc_inf, m, m_inf);
        }
        if (!acc_inf)
            for (uint32_t d = 0; d < log_seg; d++) dbl29(acc);
        acc29(us, us_inf, acc, acc_inf);
        acc29(us, us_inf, run, run_inf);
        c = us;
        c_inf = us_inf;
    }
    st_point(sh + t, c, c_inf);
    __syncthreads();
    for (uint32_t w = GF_THREADS / 2; w > 0; w >>= 1) {
        if (t < w) {
            const bool inf = ld_raw29(sh + t + w, x);
            acc29(c, c_inf, x, inf);
            st_point(sh + t, c, c_inf);
        }
        __syncthreads();
    }
    if (t == 0) st_xyzz(out + g, x29_to_xyzz(c, c_inf));
}

// After the first level (T_j, U_j of the S segments of each group): one block per group does
// the rest, out[g] = sum_j U_j + 2^log_seg sum_j j T_j + sum_j T_j (= sum_b (b + 1) B_b).
// Thread t takes segments [t Q, (t + 1) Q): running sums give its total and locally weighted sum,
// (t Q) times its total by double-and-add, then an LDS tree over the block.  One launch instead
// of the seg-level / tree / final chain (~12 latency-bound launches per batch).
template <uint32_t GF_THREADS>
__global__ void __launch_bounds__(GF_THREADS) k_group_finish(const G1Xyzz* T, const G1Xyzz* U, uint32_t S,
                                                            uint32_t log_seg, G1Xyzz* out) {
    __shared__ G1Xyzz sh[GF_THREADS];
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    const uint32_t nt = S < GF_THREADS ? S : GF_THREADS;
    const uint32_t Q = S / nt;
    G1Xyzz c = xyzz_inf();
    if (t < nt) {
        const G1Xyzz* Tg = T + (uint64_t)g * S + (uint64_t)t * Q;
        const G1Xyzz* Ug = U + (uint64_t)g * S + (uint64_t)t * Q;
        G1Xyzz run = xyzz_inf(), acc = xyzz_inf(), us = xyzz_inf();
        for (uint32_t k = Q - 1; k >= 1; k--) {
            run = xyzz_add(run, ld_xyzz(Tg + k));
            acc = xyzz_add(acc, run);
        }
        run = xyzz_add(run, ld_xyzz(Tg));
        for (uint32_t k = 0; k < Q; k++) us = xyzz_add(us, ld_xyzz(Ug + k));
        if (t) acc = xyzz_add(acc, xyzz_mul_small(run, t * Q));
        for (uint32_t d = 0; d < log_seg; d++) acc = xyzz_dbl(acc);
        c = xyzz_add(xyzz_add(us, acc), run);
    }
    sh[t] = c;
    __syncthreads();
    for (uint32_t w = GF_THREADS / 2; w > 0; w >>= 1) {
        if (t < w) {
            G1Xyzz o = sh[t + w];
            pin(o);
            c = xyzz_add(c, o);
            sh[t] = c;
        }
        __syncthreads();
    }
    if (t == 0) st_xyzz(out + g, c);
}

// Few-groups form of k_bucket_reduce29 (a single MSM, the quotient chunks): segment s of group g
// (buckets [lo, lo + SEG), lo = s SEG; bucket b holds digit b + 1) sums its buckets' raw
// radix-2^29 pieces and returns sum_b (b + 1) B_b = running-sum form + lo * (sum_b B_b) -- the
// value of k_segment_sum over the bucket sums, without the combine / bucket-final passes.
__global__ void __launch_bounds__(64) k_segment_reduce29(const G1Raw29* pieces, const uint32_t* piece_off,
                                                         uint32_t B, uint32_t groups, G1Xyzz* seg_out) {
    const uint32_t nseg = B / SEG;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg * groups) return;
    const uint32_t g = t / nseg, s = t % nseg;
    const uint32_t lo = s * SEG;
    G1X29 run, acc, x;
    bool run_inf = true, acc_inf = true;
    for (int k = (int)SEG - 1; k >= 0; k--) {
        const uint32_t bp = (lo + (uint32_t)k) * groups + g;
        const uint32_t e1 = piece_off[bp + 1];
        for (uint32_t e = piece_off[bp]; e < e1; e++) {
            const bool inf = ld_raw29(pieces + e, x);
            acc29(run, run_inf, x, inf);
        }
        acc29(acc, acc_inf, run, run_inf);
    }
    if (lo && !run_inf) {  // acc += lo * run (double-and-add, MSB first)
        G1X29 m;
        bool m_inf = true;
        for (int bit = 31 - __builtin_clz(lo); bit >= 0; bit--) {
            if (!m_inf) dbl29(m);
            if ((lo >> bit) & 1) acc29(m, m_inf, run, false);
        }
        acc29(acc, acc_inf, m, m_inf);
    }
    st_xyzz(seg_out + t, x29_to_xyzz(acc, acc_inf));
}

// Few groups with several pieces per bucket (a single 2^20 MSM: ~4.5), round 5.  Two short,
// wide kernels instead of combine level + bucket final + k_segment_sum in radix 2^32:
//   k_bucket_sums29   one thread per bucket (the whole MSM's buckets: 4 waves per SIMD at 2^18)
//                     sums its raw pieces -> raw bucket sum, group-major (g B + m)
//   k_segment_sum29   one thread per segment of SEG buckets: running sums of the bucket sums
//                     plus lo times their total by double-and-add, in radix 2^29 -> XYZZ
// then the k_tree_sum levels as before.  The sums are the same group elements as the combine path
// (exact EC arithmetic; only the order of additions differs).
__global__ void __launch_bounds__(256) k_bucket_sums29(const G1Raw29* pieces, const uint32_t* piece_off, uint32_t B,
                                                      uint32_t groups, G1Raw29* sums) {
    const uint32_t bp = blockIdx.x * blockDim.x + threadIdx.x;  // b' = m groups + g
    if (bp >= B * groups) return;
    G1X29 run, x;
    bool run_inf = true;
    const uint32_t e1 = piece_off[bp + 1];
    for (uint32_t e = piece_off[bp]; e < e1; e++) {
        const bool inf = ld_raw29(pieces + e, x);
        acc29(run, run_inf, x, inf);
    }
    const uint32_t g = bp % groups, m = bp / groups;
    st_point(sums + (uint64_t)g * B + m, run, run_inf);
}

// One thread per segment of `seg` bucket sums (seg29_for), 256 segments of one group per block
// (segments past the group's last are the identity): running sums and lo times their total, then
// the block's LDS tree -> one raw partial per block (part[g bpg + blk]).  Latency-bound (a 2^20
// MSM has 65536 segments: one wave per SIMD), so every addition / doubling issues its independent
// products together (add29_ilp / dbl29_ilp).
constexpr uint32_t SEG_BLOCK = 256;
__device__ __forceinline__ void st_raw_point(G1Raw29* p, const G1X29& a, bool inf) {
    if (inf)
        st_raw29_inf(p);
    else
        st_raw29(p, a);
}

// Buckets per k_segment_sum29 thread (seg29): the fewest (>= 4) that keep the threads within one
// wave per SIMD -- below that the waves are issue-bound alone and a shorter chain per wave is the
// gain (2^18 buckets: 4 per thread, 0.31 ms, against 8: 0.36 ms, half the SIMDs idle); above it
// the SIMDs share waves and the total work counts (2^19 buckets at 4: 0.60 ms, at 8: 0.43 ms).
// profiles/r05/s17.
static uint32_t seg29_for(uint64_t buckets) {
    uint32_t seg = 4;
    while (seg < 64 && buckets / seg > (1u << 16)) seg <<= 1;
    return seg;
}
__global__ void __launch_bounds__(SEG_BLOCK) k_segment_sum29(const G1Raw29* sums, uint32_t B, uint32_t seg,
                                                             uint32_t bpg, G1Raw29* part) {
    __shared__ G1Raw29 sh[SEG_BLOCK];
    const uint32_t nseg = B / seg;
    const uint32_t g = blockIdx.x / bpg, blk = blockIdx.x % bpg;
    const uint32_t s = blk * SEG_BLOCK + threadIdx.x;
    G1X29 acc, x;
    bool acc_inf = true;
    if (s < nseg) {
        const uint32_t lo = s * seg;
        const G1Raw29* sb = sums + (uint64_t)g * B + lo;
        G1X29 run;
        bool run_inf = true;
        for (int k = (int)seg - 1; k >= 0; k--) {  // bucket lo + k holds digit lo + k + 1
            const bool inf = ld_raw29(sb + k, x);
            acc29_ilp(run, run_inf, x, inf);
            acc29_ilp(acc, acc_inf, run, run_inf);
        }
        if (lo && !run_inf) {  // acc += lo * run (double-and-add, MSB first)
            G1X29 m;
            bool m_inf = true;
            for (int bit = 31 - __builtin_clz(lo); bit >= 0; bit--) {
                if (!m_inf) dbl29_ilp(m);
                if ((lo >> bit) & 1) acc29_ilp(m, m_inf, run, false);
            }
            acc29_ilp(acc, acc_inf, m, m_inf);
        }
    }
    st_raw_point(sh + threadIdx.x, acc, acc_inf);
    __syncthreads();
    for (uint32_t w = SEG_BLOCK / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const bool inf = ld_raw29(sh + threadIdx.x + w, x);
            acc29_ilp(acc, acc_inf, x, inf);
            st_raw_point(sh + threadIdx.x, acc, acc_inf);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) st_raw_point(part + blockIdx.x, acc, acc_inf);
}

// out[g] = sum of part[g bpg .. (g + 1) bpg), one block per group (LDS tree, radix 2^29)
__global__ void __launch_bounds__(SEG_BLOCK) k_tree_sum29(const G1Raw29* part, uint32_t bpg, G1Xyzz* out) {
    __shared__ G1Raw29 sh[SEG_BLOCK];
    G1X29 acc, x;
    bool acc_inf = true;
    for (uint32_t i = threadIdx.x; i < bpg; i += SEG_BLOCK) {
        const bool inf = ld_raw29(part + (uint64_t)blockIdx.x * bpg + i, x);
        acc29_ilp(acc, acc_inf, x, inf);
    }
    st_raw_point(sh + threadIdx.x, acc, acc_inf);
    __syncthreads();
    for (uint32_t w = SEG_BLOCK / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const bool inf = ld_raw29(sh + threadIdx.x + w, x);
            acc29_ilp(acc, acc_inf, x, inf);
            st_raw_point(sh + threadIdx.x, acc, acc_inf);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) st_xyzz(out + blockIdx.x, x29_to_xyzz(acc, acc_inf));
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
template <uint32_t CHUNK>
__global__ void k_batch_to_affine(const G1Xyzz* in, uint64_t m, G1Affine* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * CHUNK;
    if (i0 >= m) return;
    const uint64_t i1 = min(i0 + CHUNK, m);
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
    // one inversion (~380 dependent products) per BATCH points: a smaller chunk spends more
    // products, a larger one leaves the SIMDs idle behind the latency of too few waves
    const unsigned threads = 128;
    hipLaunchKernelGGL(k_batch_to_affine<BATCH>, dim3(blocks_for((m + BATCH - 1) / BATCH, threads)), dim3(threads), 0,
                       st, in, m, out);
    return hipGetLastError();
}

Status bases_create(eon_ctx* ctx, const eon_g1_affine* bases, uint64_t n, uint32_t flags,
                    bool device_ptr, eon_msm_bases** out, uint32_t force_c, hipStream_t stream,
                    DevBuf* async_tmp) {
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
    // async_tmp: enqueue on `stream` and return without a sync, the precompute scratch parked in
    // *async_tmp until the caller has synchronised the stream
    hipStream_t st = async_tmp ? stream : ctx->stream;
    auto fail = [&](Status s) {
        b->points.release();
        b->table.release();
        b->points29.release();
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
    // EON_MSM_FORCE_C (tests): the window width of a fixed-base table, e.g. c = 16 at sizes whose
    // own choice is narrower, so the fused digit sort (batch_sort) runs at test sizes
    if (!force_c && b->precomputed) {
        const char* fc = getenv("EON_MSM_FORCE_C");
        const int v = fc ? atoi(fc) : 0;
        if (v >= 4 && v <= 20) force_c = (uint32_t)v;
    }
    b->c = force_c ? force_c : choose_c(n ? n : 1, b->precomputed);
    b->windows = (255 + b->c - 1) / b->c;
    if (b->precomputed) {
        const uint64_t m = n * b->windows;
        DevBuf tmp_local;
        DevBuf& tmp = async_tmp ? *async_tmp : tmp_local;
        if (tmp.ensure(m * sizeof(G1Xyzz)) != hipSuccess ||
            b->table.ensure(m * sizeof(G1Affine)) != hipSuccess) {
            tmp.release();
            return fail(Status::err(EON_E_OOM, "precomputed table allocation failed"));
        }
        hipLaunchKernelGGL(k_precompute_windows, dim3(blocks_for(n, 128)), dim3(128), 0, st,
                           b->points.as<G1Affine>(), n, b->c, b->windows, tmp.as<G1Xyzz>());
        e = launch_batch_to_affine(tmp.as<G1Xyzz>(), m, b->table.as<G1Affine>(), st);
        if (!async_tmp) {
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            tmp.release();
        }
        if (e != hipSuccess) return fail(Status::err(EON_E_DEVICE, hipGetErrorString(e)));
    }
    if (n) {
        const uint64_t m = b->precomputed ? n * b->windows : n;
        if (!b->precomputed) {
            e = b->points29.ensure(n * sizeof(G1Affine));
            if (e == hipSuccess)
                e = hipMemcpyAsync(b->points29.p, b->points.p, n * sizeof(G1Affine), hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return fail(Status::err(EON_E_OOM, "bases allocation failed"));
        }
        G1Affine* src = b->precomputed ? b->table.as<G1Affine>() : b->points29.as<G1Affine>();
        hipLaunchKernelGGL(k_table_to29, dim3(blocks_for(m, 256)), dim3(256), 0, st, src, m);
        e = hipGetLastError();
        if (e != hipSuccess) return fail(Status::err(EON_E_DEVICE, hipGetErrorString(e)));
    }
    if (!async_tmp) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(Status::err(EON_E_DEVICE, hipGetErrorString(e)));
    *out = b;
    return Status::ok();
}

// One batch of `cols` MSMs of length n over bases[0..n): MSM j uses scalars[i * ld + j].  A batch
// runs in three steps on one stream with its own workspace, so that consecutive batches on two
// streams overlap the memory-bound digit sort of one with the VALU-bound piece sums of the other:
//   batch_sort    digits, radix sort, bucket starts, piece offsets; reads back the pair / piece
//                 counts (synchronises its stream)
//   batch_pieces  k_piece_sum (asynchronous)
//   batch_reduce  combine levels (count read-backs), bucket sums, weighted bucket reduction;
//                 leaves one XYZZ point per column in `out_dev`
struct Batch {
    const Fr* scalars = nullptr;
    uint32_t cols = 0, col0 = 0;
    G1Xyzz* out = nullptr;
    uint32_t c = 0, W = 0, B = 0, groups = 0, nb = 0, key_bits = 0, log_chunk = 0;
    uint64_t E = 0, max_pieces = 0;
    size_t sort_bytes = 0, scan_bytes = 0;
    uint32_t n_pieces = 0, n_pairs = 0;
    uint32_t levels = 0;  // PIECE-way combine levels until every bucket holds <= 1 partial
    bool counted = false;  // n_pieces / n_pairs / levels read back (batch_counts)
    size_t prof_rec = SIZE_MAX;  // the k_piece_sum profiler record to complete with the counts
    uint32_t w_act = 0;   // windows that can hold a nonzero digit (0: all of the layout's)
};

struct SortedRef {
    const uint32_t *keys, *vals, *start, *piece_off;
};

static bool msm_debug() {
    static const bool d = getenv("EON_MSM_DEBUG") != nullptr;
    return d;
}

// Layout of a batched column MSM of n-row columns against bases with this window layout: the
// window size, window count and columns per batch (<= 2^28 digit pairs per batch).
struct MsmLayout {
    uint32_t c = 0, W = 0;
    bool precomputed = false;
    uint64_t cpb = 1;
};

// digit pairs per column batch: 2^29 (the prove's 1312 columns in 6 batches of <= 256, a rank's
// 164 of the 8-way sharded prove in one): fewer, larger piece-sum launches than 2^28 -- prove
// -0.5 %, emulated 8-rank prove -1 % (profiles/r05/s23, s24; 2^30 measured the same)
#ifndef EON_MSM_BATCH_LOG_PAIRS
#define EON_MSM_BATCH_LOG_PAIRS 29
#endif
static MsmLayout msm_layout(const eon_msm_bases* b, uint64_t n, uint32_t width) {
    MsmLayout L;
    L.precomputed = b->precomputed;
    L.c = b->precomputed ? b->c : choose_c(n, false);
    L.W = (255 + L.c - 1) / L.c;
    // columns per batch: keep the digit pairs of one batch at <= 2^EON_MSM_BATCH_LOG_PAIRS (8 GiB of
    // sort buffers at 2^29)
    uint64_t cpb = (1ull << EON_MSM_BATCH_LOG_PAIRS) / (n * L.W);
    if (cpb < 1) cpb = 1;
    const uint64_t max_groups = b->precomputed ? cpb : cpb * L.W;
    if (max_groups > 65535) cpb = b->precomputed ? 65535 : 65535 / L.W;
    // equal batches (164 columns -> 82 + 82, not 128 + 36): the two streams overlap evenly
    const uint64_t n_batches = (width + cpb - 1) / cpb;
    L.cpb = (width + n_batches - 1) / n_batches;
    return L;
}

static std::vector<Batch> make_batches(const Fr* scalars, uint32_t width, uint64_t cpb) {
    std::vector<Batch> batches;
    for (uint32_t j0 = 0; j0 < width; j0 += (uint32_t)cpb) {
        Batch bt;
        bt.scalars = scalars + j0;
        bt.col0 = j0;
        bt.cols = (uint32_t)std::min<uint64_t>(cpb, width - j0);
        batches.push_back(bt);
    }
    return batches;
}

// EON_MSM_FUSED_SORT (default 1): the digit sort's first pass ranks the digits as k_digit_sort_pass
// computes them (batch_sort); 0 restores k_msm_digits4 + two k_sort_pass passes
#ifndef EON_MSM_FUSED_SORT
#define EON_MSM_FUSED_SORT 1
#endif

// The digit sort: sort.hip's stable LSD radix sort (two 8-bit passes for c = 16)
static hipError_t sort_pairs(void* temp, const uint32_t* k_in, uint32_t* k_out, const uint32_t* v_in,
                             uint32_t* v_out, uint64_t n, uint32_t bits, hipStream_t st, bool hist_ready) {
    return radix_sort_pairs(temp, k_in, k_out, v_in, v_out, n, bits, st, hist_ready);
}

// digits + radix sort + bucket starts + piece offsets of one batch into `out`; `wk` supplies the
// unsorted pairs, the sort / scan scratch and the count read-back slots
static Status batch_sort(eon_ctx* ctx, const MsmLayout& L, uint64_t n, uint64_t ld, Batch& bt,
                         MsmWork& wk, SortedBufs& out, hipStream_t st, hipEvent_t sorted_ev) {
    bt.c = L.c;
    bt.W = bt.w_act ? std::min(bt.w_act, L.W) : L.W;
    bt.B = 1u << (bt.c - 1);
    bt.groups = L.precomputed ? bt.cols : bt.cols * bt.W;
    bt.nb = bt.groups * bt.B;
    bt.E = n * bt.W * bt.cols;
    if (bt.E > RADIX_SORT_MAX_PAIRS) return Status::err(EON_E_SHAPE, "MSM batch too large for 32-bit pair indices");
    // keys are (group << c) | (|digit| - 1); only the low c bits are sorted
    if (((uint64_t)bt.groups << bt.c) > 0xFFFFFFFFull)
        return Status::err(EON_E_SHAPE, "too many MSM groups for 32-bit digit keys");
    bt.key_bits = bt.c;
    const uint64_t E = bt.E;
    const uint32_t nb = bt.nb;

    EON_HIP(ctx_ensure(ctx, wk.keys, E * 4));
    EON_HIP(ctx_ensure(ctx, wk.vals, E * 4));
    EON_HIP(ctx_ensure(ctx, out.keys2, E * 4));
    EON_HIP(ctx_ensure(ctx, out.vals2, E * 4));
    EON_HIP(ctx_ensure(ctx, out.start, (nb + 1) * 4ull));
    EON_HIP(ctx_ensure(ctx, out.piece_off, (nb + 1) * 4ull));
    bt.sort_bytes = radix_sort_temp_bytes(E, bt.key_bits);
    bt.scan_bytes = exclusive_scan_temp_bytes(nb + 1);
    EON_HIP(ctx_ensure(ctx, wk.temp, std::max(bt.sort_bytes, bt.scan_bytes)));
    bt.log_chunk = LOG_CHUNK_MIN;
    while (bt.log_chunk < LOG_CHUNK_MAX && (E >> (bt.log_chunk + 1)) >= (1ull << EON_PIECE_THREADS_LOG)) bt.log_chunk++;
    // few buckets for many pairs (a bucket would collect more than ~8 pieces): longer chunks while
    // the piece sums keep 2^18 threads (4 waves per SIMD)
    while (bt.log_chunk < LOG_CHUNK_MAX && (E >> bt.log_chunk) > 8ull * nb && (E >> (bt.log_chunk + 1)) >= (1ull << 18))
        bt.log_chunk++;
    bt.max_pieces = (E >> bt.log_chunk) + nb + 1;  // >= the real piece count
    if (!wk.host_counts) EON_HIP(hipHostMalloc(reinterpret_cast<void**>(&wk.host_counts), 64));

    Profiler* prof = &ctx->prof;
    uint32_t* hist = radix_sort_histograms(wk.temp.p, E);
    EON_HIP(hipMemsetAsync(hist, 0, RADIX_SORT_MAX_PASSES * 256 * 4, st));
    const uint32_t tile_cols = bt.cols >= DIGIT_COLS ? DIGIT_COLS : (bt.cols >= 2 ? 2 : 1);
    // four rows per thread (16-byte stores) when n allows it, k_msm_digits otherwise: 6.2 vs 10.4 ms
    // of digits per prove (round 4, profiles/r04/s19)
    const bool quad = (n & 3) == 0;
    const uint32_t tile_rows = (quad ? 1024 : 256) / tile_cols;
    const uint32_t grid_y = (bt.cols + tile_cols - 1) / tile_cols;
    const uint64_t tiles = (n + tile_rows - 1) / tile_rows;
    const uint32_t grid_x = (uint32_t)std::min<uint64_t>(tiles, std::max<uint32_t>(1, DIGIT_BLOCKS / grid_y));
    // the first sort pass fused with the digits (DigitSource): fixed-base tables, c = 16, all 16
    // windows, whole 1024-row tiles, two passes
    const bool fused = EON_MSM_FUSED_SORT && L.precomputed && bt.c == 16 && bt.W == 16 && L.W == 16 &&
                       n % (EON_SORT_LEAN ? sortpass::LEAN_THREADS / 8 : sortpass::SORT_THREADS) == 0 &&
                       radix_sort_passes(bt.key_bits).passes == 2;
    if (fused) {
        EON_HIP(ctx_ensure(ctx, wk.canon, n * bt.cols * sizeof(Fr)));
        prof->begin("k_msm_digit_hist", n * bt.cols * 64, st);
        hipLaunchKernelGGL(k_msm_digits4<false>, dim3(grid_x, grid_y), dim3(256), 0, st, bt.scalars, n, ld, bt.cols,
                           bt.c, bt.W, L.W, 1u, tile_cols, nullptr, nullptr, radix_sort_passes(bt.key_bits), hist,
                           wk.canon.as<Fr>());
        prof->end(st);
        EON_HIP(hipGetLastError());
        EON_HIP(radix_sort_prepare(wk.temp.p, E, bt.key_bits, st));
        const RadixPassArgs a0 = radix_sort_pass_args(wk.temp.p, E, bt.key_bits, 0);
        // per call: the attribute is per device (another context may run on another GPU)
        // the pass's own traffic: 32 bytes of scalar per 16 pairs read, 8 bytes per pair written
        prof->begin("k_digit_sort_pass", n * bt.cols * 32 + E * 8, st);
#if EON_SORT_LEAN
        const DigitSourceLean src{wk.canon.as<Fr>(), n, (uint32_t)(n / (sortpass::LEAN_THREADS / 8)), L.W};
        hipLaunchKernelGGL(k_digit_sort_pass_lean, dim3(a0.tiles), dim3(sortpass::LEAN_THREADS), sortpass::LEAN_LDS, st,
                           src, wk.keys.as<uint32_t>(), wk.vals.as<uint32_t>(), (uint32_t)E, a0.shift, a0.base,
                           a0.status, a0.tile_ctr);
#else
        // per call: the attribute is per device (another context may run on another GPU)
        EON_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_digit_sort_pass),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)sortpass::SORT_LDS));
        const DigitSource src{wk.canon.as<Fr>(), n, (uint32_t)(n / sortpass::SORT_THREADS), L.W};
        hipLaunchKernelGGL(k_digit_sort_pass, dim3(a0.tiles), dim3(sortpass::SORT_THREADS), sortpass::SORT_LDS, st, src,
                           wk.keys.as<uint32_t>(), wk.vals.as<uint32_t>(), (uint32_t)E, a0.shift, a0.base, a0.status,
                           a0.tile_ctr);
#endif
        prof->end(st);
        EON_HIP(hipGetLastError());
        prof->begin("radix_sort_pairs", E * 16, st);  // the second pass
        EON_HIP(radix_sort_tail(wk.temp.p, wk.keys.as<uint32_t>(), wk.vals.as<uint32_t>(), out.keys2.as<uint32_t>(),
                                out.vals2.as<uint32_t>(), E, bt.key_bits, st));
        prof->end(st);
    } else {
        prof->begin("k_msm_digits", n * bt.cols * 32 + E * 8, st);
        hipLaunchKernelGGL(quad ? k_msm_digits4<true> : k_msm_digits, dim3(grid_x, grid_y),
                           dim3(256), 0, st, bt.scalars, n, ld, bt.cols, bt.c, bt.W, L.W, (uint32_t)L.precomputed,
                           tile_cols, wk.keys.as<uint32_t>(), wk.vals.as<uint32_t>(), radix_sort_passes(bt.key_bits),
                           hist, nullptr);
        prof->end(st);
        EON_HIP(hipGetLastError());
        // every pass reads and writes each (key, value) pair once: 16 bytes per pair and pass
        prof->begin("radix_sort_pairs", E * 16 * radix_sort_passes(bt.key_bits).passes, st);
        EON_HIP(sort_pairs(wk.temp.p, wk.keys.as<uint32_t>(), out.keys2.as<uint32_t>(), wk.vals.as<uint32_t>(),
                           out.vals2.as<uint32_t>(), E, bt.key_bits, st, true));
        prof->end(st);
    }
    prof->begin("k_bucket_start", E * 4, st);
    hipLaunchKernelGGL(k_bucket_start, dim3(blocks_for(E / BS_KEYS + 1, 256)), dim3(256), 0, st,
                       out.keys2.as<uint32_t>(), E, bt.c, bt.groups, nb, out.start.as<uint32_t>());
    prof->end(st);
    // the most pieces one bucket holds fixes the combine levels (no read-backs in the reduction)
    EON_HIP(ctx_ensure(ctx, wk.stat, 16));
    EON_HIP(hipMemsetAsync(wk.stat.p, 0, 16, st));
    EON_HIP(exclusive_scan_chunk_counts(wk.temp.p, out.start.as<uint32_t>(), nb, bt.log_chunk,
                                        out.piece_off.as<uint32_t>(), wk.stat.as<uint32_t>(), st));
    // the sorted pairs are ready for the piece sums (sorted_ev), ahead of the count read-back
    EON_HIP(hipEventRecord(sorted_ev, st));
    // the reduction's launches are sized by the real counts (12-byte read-back: pieces, nonzero
    // digits, max pieces); batch_counts waits for them
    EON_HIP(hipMemcpyAsync(wk.host_counts, out.piece_off.as<uint32_t>() + nb, 4, hipMemcpyDeviceToHost, st));
    EON_HIP(hipMemcpyAsync(wk.host_counts + 1, out.start.as<uint32_t>() + nb, 4, hipMemcpyDeviceToHost, st));
    EON_HIP(hipMemcpyAsync(wk.host_counts + 3, wk.stat.p, 4, hipMemcpyDeviceToHost, st));
    if (!wk.counts_ev) EON_HIP(hipEventCreateWithFlags(&wk.counts_ev, hipEventDisableTiming));
    EON_HIP(hipEventRecord(wk.counts_ev, st));
    bt.counted = false;
    return Status::ok();
}

static Status batch_counts(eon_ctx* ctx, Batch& bt, MsmWork& wk, uint64_t n) {
    EON_HIP(hipEventSynchronize(wk.counts_ev));
    bt.n_pieces = wk.host_counts[0];
    bt.n_pairs = wk.host_counts[1];
    bt.levels = 0;
    for (uint64_t m = wk.host_counts[3]; m > 1; m = (m + PIECE - 1) / PIECE) bt.levels++;
    if (msm_debug())
        fprintf(stderr, "msm_batch n=%llu cols=%u c=%u W=%u nb=%u E=%llu pairs=%u pieces=%u\n",
                (unsigned long long)n, bt.cols, bt.c, bt.W, bt.nb, (unsigned long long)bt.E, bt.n_pairs,
                bt.n_pieces);
    bt.counted = true;
    if (bt.prof_rec < ctx->prof.recs.size()) {  // k_piece_sum was launched before the counts
        ctx->prof.recs[bt.prof_rec].alg_mulmods = (uint64_t)bt.n_pairs * 10;
        ctx->prof.recs[bt.prof_rec].design_bytes = (uint64_t)bt.n_pairs * 72 + (uint64_t)bt.n_pieces * 144;
        bt.prof_rec = SIZE_MAX;
    }
    return Status::ok();
}

static SortedRef sorted_ref(const SortedBufs& s) {
    return SortedRef{s.keys2.as<uint32_t>(), s.vals2.as<uint32_t>(), s.start.as<uint32_t>(),
                     s.piece_off.as<uint32_t>()};
}

// the reduction reads k_piece_sum29's raw partials directly (k_bucket_reduce29 /
// k_segment_reduce29): radix-2^29 pieces, no combine level needed, and either many groups or few
// pieces per bucket -- with few groups and several pieces per bucket (a single 2^20 MSM: ~4.5)
// the one-thread-per-segment chain is longer than combine + bucket-final + k_segment_sum
// (3.23 vs 3.00 ms for the 2^20 MSM)
static bool fused_reduce(const Batch& bt) {
    return bt.levels <= 1 && bt.B >= SEG &&
           (bt.groups >= 64 || (uint64_t)bt.n_pieces <= 2ull * bt.nb);
}

// few groups, several pieces per bucket, none above PIECE: k_bucket_sums29 + k_segment_sum29
// (round 5; the combine-level path stays for skewed inputs, whose buckets hold more pieces)
#ifndef EON_MSM_SUMS29
#define EON_MSM_SUMS29 1
#endif
static bool sums_reduce(const Batch& bt) {
    return EON_MSM_SUMS29 && bt.levels <= 1 && bt.B >= SEG && bt.groups < 64 && !fused_reduce(bt);
}

// piece sums of one sorted batch against bases `b` (asynchronous); wk supplies the piece buffers
static Status batch_pieces(eon_ctx* ctx, const eon_msm_bases* b, Batch& bt, const SortedRef& sr,
                           MsmWork& wk, hipStream_t st) {
    EON_HIP(ctx_ensure(ctx, wk.piece_sums, std::max<uint64_t>(bt.max_pieces * sizeof(G1Xyzz), (uint64_t)bt.nb * sizeof(G1Raw29))));
    EON_HIP(ctx_ensure(ctx, wk.piece_sums2, bt.max_pieces * sizeof(G1Xyzz)));
    EON_HIP(ctx_ensure(ctx, wk.owner, bt.max_pieces * 4));
    EON_HIP(ctx_ensure(ctx, wk.bucket_sums, (uint64_t)bt.nb * sizeof(G1Xyzz)));
    EON_HIP(ctx_ensure(ctx, wk.off2, (bt.nb + 1) * 4ull));
    EON_HIP(ctx_ensure(ctx, wk.off3, (bt.nb + 1) * 4ull));
    EON_HIP(ctx_ensure(ctx, wk.count, (bt.nb + 1) * 4ull));
    EON_HIP(ctx_ensure(ctx, wk.temp, bt.scan_bytes));
    EON_HIP(ctx_ensure(ctx, wk.piece_raw, bt.max_pieces * sizeof(G1Raw29)));
    if (!wk.host_counts) EON_HIP(hipHostMalloc(reinterpret_cast<void**>(&wk.host_counts), 64));
    const G1Affine* pts = b->piece_source();
    // algorithmic bytes: n (64 + 32) B per MSM of n terms -- each
    // base and scalar read once; design bytes: what this kernel's access pattern moves instead,
    // a 4-byte key, a 4-byte reference and a 64-byte table entry per nonzero digit plus one
    // 144-byte partial per piece
    // mulmods: one XYZZ mixed addition (madd-2008-s, 8M + 2S) per nonzero digit
    const uint64_t msm_n = bt.E / ((uint64_t)bt.W * bt.cols);
    // launched before the count read-back (batch_counts), the grid covers all E pairs and the
    // profiler record gets its counts later
    const uint64_t pairs_max = bt.counted ? bt.n_pairs : bt.E;
    if (!bt.counted && ctx->prof.enabled) bt.prof_rec = ctx->prof.recs.size();
    ctx->prof.begin("k_piece_sum", (uint64_t)bt.cols * msm_n * 96, st, (uint64_t)bt.n_pairs * 10,
                    (uint64_t)bt.n_pairs * 72 + (uint64_t)bt.n_pieces * 144);
    const uint32_t blocks = blocks_for((pairs_max + (1u << bt.log_chunk) - 1) >> bt.log_chunk, 64);
    if (pairs_max)
        hipLaunchKernelGGL(k_piece_sum29, dim3(blocks), dim3(64), 0, st, sr.keys, sr.vals, sr.start, sr.piece_off,
                           bt.log_chunk, bt.c, bt.groups, bt.nb, pts, wk.piece_raw.as<G1Raw29>());
    ctx->prof.end(st);
    if (!bt.counted) EON_TRY(batch_counts(ctx, bt, wk, msm_n));
    if (bt.n_pieces && !fused_reduce(bt) && !sums_reduce(bt))
        hipLaunchKernelGGL(k_raw29_to_xyzz, dim3(blocks_for(bt.n_pieces, 128)), dim3(128), 0, st,
                           wk.piece_raw.as<G1Raw29>(), bt.n_pieces, wk.piece_sums.as<G1Xyzz>());
    EON_HIP(hipGetLastError());
    return Status::ok();
}

// per-column output step shared by both bucket reductions
static Status write_columns(const MsmLayout& L, const Batch& bt, const G1Xyzz* per_group,
                            hipStream_t st) {
    // one point per group; per column: the group itself (fixed base) or the Horner combination of
    // its windows
    if (!L.precomputed) {
        hipLaunchKernelGGL(k_window_horner, dim3(blocks_for(bt.cols, 64)), dim3(64), 0, st, per_group,
                           bt.cols, bt.W, bt.c, bt.out);
        EON_HIP(hipGetLastError());
    } else {
        EON_HIP(hipMemcpyAsync(bt.out, per_group, bt.cols * sizeof(G1Xyzz), hipMemcpyDeviceToDevice, st));
    }
    return Status::ok();
}

// sum_d d * B_d per group, few-groups form: k_segment_sum + LDS trees (short dependency chains)
static Status reduce_segments(eon_ctx* ctx, const MsmLayout& L, const Batch& bt, const SortedRef& sr,
                              MsmWork& wk, hipStream_t st, bool fused, bool sums29 = false) {
    const uint32_t nseg = bt.B / SEG;  // c >= 4, so B >= SEG
    const uint32_t groups = bt.groups;
    EON_HIP(ctx_ensure(ctx, wk.red_a, (uint64_t)groups * nseg * sizeof(G1Xyzz)));
    EON_HIP(ctx_ensure(ctx, wk.red_b, (uint64_t)groups * nseg * sizeof(G1Xyzz)));
    ctx->prof.begin("k_segment_sum", (uint64_t)bt.nb * 128 + (uint64_t)groups * nseg * 128, st);
    if (sums29) {
        // raw bucket sums (k_bucket_sums29, in wk.piece_sums as G1Raw29) -> one raw partial per
        // 256 segments -> one point per group, all in radix 2^29
        const uint32_t seg = std::min(bt.B, seg29_for((uint64_t)bt.B * groups));
        const uint32_t bpg = (bt.B / seg + SEG_BLOCK - 1) / SEG_BLOCK;
        EON_HIP(ctx_ensure(ctx, wk.red_b, (uint64_t)groups * bpg * sizeof(G1Raw29)));
        hipLaunchKernelGGL(k_segment_sum29, dim3(groups * bpg), dim3(SEG_BLOCK), 0, st, wk.piece_sums.as<G1Raw29>(),
                           bt.B, seg, bpg, wk.red_b.as<G1Raw29>());
        hipLaunchKernelGGL(k_tree_sum29, dim3(groups), dim3(SEG_BLOCK), 0, st, wk.red_b.as<G1Raw29>(), bpg,
                           wk.red_a.as<G1Xyzz>());
        ctx->prof.end(st);
        EON_HIP(hipGetLastError());
        return write_columns(L, bt, wk.red_a.as<G1Xyzz>(), st);
    } else if (fused)
        hipLaunchKernelGGL(k_segment_reduce29, dim3(blocks_for((uint64_t)nseg * groups, 64)), dim3(64), 0, st,
                           wk.piece_raw.as<G1Raw29>(), sr.piece_off, bt.B, groups, wk.red_a.as<G1Xyzz>());
    else
        hipLaunchKernelGGL(k_segment_sum, dim3(blocks_for((uint64_t)nseg * groups, 64)), dim3(64), 0, st,
                           wk.bucket_sums.as<G1Xyzz>(), bt.B, groups, wk.red_a.as<G1Xyzz>());
    ctx->prof.end(st);
    G1Xyzz* cur = wk.red_a.as<G1Xyzz>();
    G1Xyzz* nxt = wk.red_b.as<G1Xyzz>();
    uint32_t len = nseg;
    while (len > 1) {
        const uint32_t blk = (len + TREE - 1) / TREE;
        hipLaunchKernelGGL(k_tree_sum, dim3(blk, groups), dim3(TREE), 0, st, cur, len, nxt);
        std::swap(cur, nxt);
        len = blk;
    }
    EON_HIP(hipGetLastError());
    return write_columns(L, bt, cur, st);
}

// Deferred group finish: the batches of one call leave their first-level segment sums (T, U of
// k_bucket_reduce29) in call-wide arrays, row = the group's output index, and ONE k_group_finish
// launch over every row runs after the last batch.  Per batch, that finish was 120 groups x 256
// threads -- under one wave per SIMD, a chain of ~75 dependent additions (1.1 ms per batch,
// latency-bound); over the whole call (1312 or 2624 groups) it is throughput-bound.
struct DeferredFinish {
    G1Raw29* T = nullptr;
    G1Raw29* U = nullptr;
    G1Xyzz* out_base = nullptr;  // row r's result goes to out_base[r]
    uint32_t nseg = 0, log_seg = 0;
    std::vector<std::pair<uint64_t, uint64_t>> rows;  // deferred [row0, row0 + n)
};

// k_group_finish over the deferred rows (merged into maximal runs) on `st`
static hipError_t launch_group_finish29(const G1Raw29* T, const G1Raw29* U, uint32_t nseg, uint32_t lsg,
                                        G1Xyzz* out, uint32_t groups, hipStream_t st);

static Status run_deferred_finish(eon_ctx* ctx, DeferredFinish& df, hipStream_t st) {
    if (df.rows.empty()) return Status::ok();
    std::sort(df.rows.begin(), df.rows.end());
    std::vector<std::pair<uint64_t, uint64_t>> runs;
    for (auto& r : df.rows) {
        if (!runs.empty() && runs.back().first + runs.back().second == r.first)
            runs.back().second += r.second;
        else
            runs.push_back(r);
    }
    for (auto& r : runs) {
        ctx->prof.begin("k_group_finish", r.second * df.nseg * 256ull, st, r.second * df.nseg * 3ull * 14);
        EON_HIP(launch_group_finish29(df.T + r.first * df.nseg, df.U + r.first * df.nseg, df.nseg, df.log_seg,
                                      df.out_base + r.first, (uint32_t)r.second, st));
        ctx->prof.end(st);
    }
    df.rows.clear();
    return Status::ok();
}

static Status prepare_deferred(eon_ctx* ctx, const MsmLayout& L, uint64_t rows, G1Xyzz* out_base,
                               DeferredFinish& df) {
    df = DeferredFinish{};
    if (!L.precomputed) return Status::ok();
    const uint32_t B = 1u << (L.c - 1);
    if (B < RED_SEG) return Status::ok();
    df.nseg = B / RED_SEG;
    df.log_seg = 31 - __builtin_clz(RED_SEG);
    EON_HIP(ctx_ensure(ctx, ctx->fin_T, rows * df.nseg * sizeof(G1Raw29)));
    EON_HIP(ctx_ensure(ctx, ctx->fin_U, rows * df.nseg * sizeof(G1Raw29)));
    df.T = ctx->fin_T.as<G1Raw29>();
    df.U = ctx->fin_U.as<G1Raw29>();
    df.out_base = out_base;
    return Status::ok();
}

static Status piece_merge(eon_ctx* ctx, const Batch& bt, const SortedRef& sr, MsmWork& wk, hipStream_t st) {
    if (!EON_PIECE_MERGE) return Status::ok();
    const uint64_t chunks = ((uint64_t)bt.n_pairs + (1u << bt.log_chunk) - 1) >> bt.log_chunk;
    const uint32_t log_step = EON_PIECE_MERGE == 2 ? 6 : 0;
    const uint64_t boundaries = (chunks - 1) >> log_step;
    if (chunks < 2 || boundaries == 0) return Status::ok();
    // ~one addition per boundary: 2 x 144 B read, 144 B written
    ctx->prof.begin("k_piece_merge29", boundaries * 432, st, boundaries * 14);
    hipLaunchKernelGGL(k_piece_merge29, dim3(blocks_for(boundaries, 64)), dim3(64), 0, st, sr.keys, sr.start,
                       sr.piece_off, bt.log_chunk, log_step, bt.c, bt.groups, bt.nb, wk.piece_raw.as<G1Raw29>());
    ctx->prof.end(st);
    EON_HIP(hipGetLastError());
    return Status::ok();
}

// combine levels, bucket sums and the weighted bucket reduction of one batch's pieces (read-back
// of each level's count synchronises `st`); leaves one XYZZ point per column at bt.out.  The
// sorted piece offsets are only read (a prepared batch is reduced once per bases object).
static Status batch_reduce(eon_ctx* ctx, const MsmLayout& L, const Batch& bt, const SortedRef& sr,
                           MsmWork& wk, hipStream_t st, bool fused, DeferredFinish* df = nullptr) {
    Profiler* prof = &ctx->prof;
    const uint32_t nb = bt.nb, groups = bt.groups, B = bt.B;
    if (df && df->T && fused && groups >= 64 && B >= RED_SEG && L.precomputed) {
        // first level only; the finish runs once per call (run_deferred_finish)
        const uint64_t row0 = (uint64_t)(bt.out - df->out_base);
        EON_TRY(piece_merge(ctx, bt, sr, wk, st));
        prof->begin("bucket_reduce", (uint64_t)nb * 128 + (uint64_t)nb / SEG * 256, st);
        hipLaunchKernelGGL((k_bucket_reduce29<G1Raw29, EON_PIECE_MERGE != 0>),
                           dim3(blocks_for((uint64_t)df->nseg * groups, 64)), dim3(64), 0, st,
                           wk.piece_raw.as<G1Raw29>(), sr.piece_off, B, RED_SEG, groups, df->T + row0 * df->nseg,
                           df->U + row0 * df->nseg);
        prof->end(st);
        EON_HIP(hipGetLastError());
        df->rows.emplace_back(row0, groups);
        return Status::ok();
    }
    if (!fused && sums_reduce(bt)) {
        prof->begin("k_bucket_sums29", (uint64_t)bt.n_pieces * 144 + (uint64_t)nb * 144, st);
        hipLaunchKernelGGL(k_bucket_sums29, dim3(blocks_for(nb, 256)), dim3(256), 0, st, wk.piece_raw.as<G1Raw29>(),
                           sr.piece_off, B, groups, wk.piece_sums.as<G1Raw29>());
        prof->end(st);
        EON_HIP(hipGetLastError());
        return reduce_segments(ctx, L, bt, sr, wk, st, false, true);
    }
    // combine levels until every bucket holds one partial (skewed scalars put many pieces in a
    // bucket: all-equal scalars put n pieces in one bucket per window)
    const uint32_t* off_cur = sr.piece_off;
    uint32_t* off_bufs[2] = {wk.off2.as<uint32_t>(), wk.off3.as<uint32_t>()};
    int next_off = 0;
    G1Xyzz* part_cur = wk.piece_sums.as<G1Xyzz>();
    G1Xyzz* part_nxt = wk.piece_sums2.as<G1Xyzz>();
    uint64_t bound = bt.n_pieces;  // >= the partials of the current level
    for (uint32_t level = 0; level < (fused ? 0u : bt.levels); level++) {
        uint32_t* off_nxt = off_bufs[next_off];
        hipLaunchKernelGGL(k_level_count, dim3(blocks_for(nb + 1, 256)), dim3(256), 0, st, off_cur,
                           nb, wk.count.as<uint32_t>());
        EON_HIP(exclusive_scan_u32(wk.temp.p, wk.count.as<uint32_t>(), off_nxt, nb + 1, st));
        hipLaunchKernelGGL(k_piece_owner, dim3(blocks_for(nb, 256)), dim3(256), 0, st, off_nxt, nb,
                           wk.owner.as<uint32_t>());
        // sum_b ceil(p_b / PIECE) <= min(bound, nb + bound / PIECE)
        const uint64_t nxt = std::min<uint64_t>(bound, nb + bound / PIECE);
        prof->begin("k_partial_combine", (bound + nxt) * 128, st, (bound - std::min(bound, nxt)) * 14);
        hipLaunchKernelGGL(k_partial_combine, dim3(blocks_for(nxt, 64)), dim3(64), 0, st, off_cur, off_nxt,
                           wk.owner.as<uint32_t>(), nb, part_cur, part_nxt);
        prof->end(st);
        off_cur = off_nxt;
        next_off ^= 1;
        std::swap(part_cur, part_nxt);
        bound = nxt;
    }
    if (!fused)
        hipLaunchKernelGGL(k_bucket_final, dim3(blocks_for(nb, 256)), dim3(256), 0, st, off_cur, B, groups,
                           part_cur, wk.bucket_sums.as<G1Xyzz>());
    if (groups < 64) return reduce_segments(ctx, L, bt, sr, wk, st, fused);
    // sum_d d * B_d per group (bucket b holds digit b + 1): segment sums T, U of SEG buckets
    // (k_bucket_reduce29 from the raw pieces, or k_seg_level from bucket sums), then k_group_finish
    G1Xyzz* T = wk.piece_sums.as<G1Xyzz>();
    G1Xyzz* u_buf = wk.piece_sums2.as<G1Xyzz>();
    EON_HIP(wk.red_a.ensure((uint64_t)groups * sizeof(G1Xyzz)));
    prof->begin("bucket_reduce", (uint64_t)nb * 128 + (uint64_t)nb / SEG * 256, st);
    const uint32_t seg = B < SEG ? B : SEG;
    const uint32_t nseg = B / seg;
    if (fused) {
        EON_TRY(piece_merge(ctx, bt, sr, wk, st));
        hipLaunchKernelGGL((k_bucket_reduce29<G1Xyzz, EON_PIECE_MERGE != 0>), dim3(blocks_for((uint64_t)nseg * groups, 64)),
                           dim3(64), 0, st, wk.piece_raw.as<G1Raw29>(), sr.piece_off, B, seg, groups, T, u_buf);
    } else
        hipLaunchKernelGGL(k_seg_level, dim3(blocks_for((uint64_t)nseg * groups, 64)), dim3(64), 0, st,
                           wk.bucket_sums.as<G1Xyzz>(), B, seg, groups, T, u_buf);
    G1Xyzz* per_group = wk.red_a.as<G1Xyzz>();
    hipLaunchKernelGGL(k_group_finish<FINISH_THREADS>, dim3(groups), dim3(FINISH_THREADS), 0, st, T, u_buf, nseg,
                       31 - __builtin_clz(seg), per_group);
    prof->end(st);
    EON_HIP(hipGetLastError());
    return write_columns(L, bt, per_group, st);
}

static hipError_t launch_group_finish29(const G1Raw29* T, const G1Raw29* U, uint32_t nseg, uint32_t lsg,
                                        G1Xyzz* out, uint32_t groups, hipStream_t st) {
    hipLaunchKernelGGL(k_group_finish29<FINISH_THREADS>, dim3(groups), dim3(FINISH_THREADS), 0, st, T, U, nseg, lsg,
                       out);
    return hipGetLastError();
}

}  // namespace eon

// Prepared scalars: every batch's digit pairs sorted once and kept on device, so that MSMs of the
// same scalar columns against other bases objects of the same window layout skip the digit
// extraction and the sort (KzgPcs: the SRS for the commitment, then the opening bases H(z) of
// every opening point, kzg/src/pcs.rs:244-251,297-330).  The scalars themselves are not retained.
struct eon_msm_scalars {
    eon_ctx* ctx = nullptr;
    uint64_t n = 0;
    uint32_t width = 0;
    eon::MsmLayout layout;
    std::vector<eon::Batch> batches;
    std::vector<eon::SortedBufs> sorted;
    // buffers go back to the context's cache (caller holds ctx->mu)
    ~eon_msm_scalars() {
        constexpr size_t CAP = 48ull << 30;  // MSM_SORTED_CACHE_CAP
        size_t cached = 0;
        if (ctx)
            for (const auto& sb : ctx->sorted_cache) cached += sb.bytes();
        for (auto& sb : sorted) {
            if (ctx && cached + sb.bytes() <= CAP) {
                cached += sb.bytes();
                ctx->sorted_cache.push_back(std::move(sb));
                sb = eon::SortedBufs{};
            } else {
                sb.release();
            }
        }
    }
};

namespace eon {

const G1Affine* bases_points(const eon_msm_bases* b) { return b->points.as<G1Affine>(); }

// out[e] = 3 tab[e] (tab: 29-form canonical affine; out radix-2^32 XYZZ for the batched affine
// conversion)
__global__ void k_triple29(const G1Affine* tab, uint64_t m, G1Xyzz* out) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const G1Affine a = ld_affine(tab + e);
    if (is_inf(a)) {
        st_xyzz(out + e, xyzz_inf());
        return;
    }
    const F29 x = unpack29(a.x), y = unpack29(a.y);
    G1X29 acc = dbl29_affine(x, y);  // 2T (T has odd order r: 2T != -T, != O)
    bool inf = false;
    if (!madd29(acc, x, y)) inf = madd29_exceptional(acc, x, y);
    st_xyzz(out + e, x29_to_xyzz(acc, inf));
}

const G1Affine* bases_table3_29(const eon_msm_bases* cb, hipStream_t st) {
    eon_msm_bases* b = const_cast<eon_msm_bases*>(cb);  // a cache filled once
    if (!b->precomputed || b->n == 0) return nullptr;
    if (b->table3.p) return b->table3.as<G1Affine>();
    const uint64_t m = b->n * b->windows;
    DevBuf tmp;
    if (tmp.ensure(m * sizeof(G1Xyzz)) != hipSuccess || b->table3.ensure(m * sizeof(G1Affine)) != hipSuccess) {
        tmp.release();
        b->table3.release();
        return nullptr;
    }
    hipLaunchKernelGGL(k_triple29, dim3(blocks_for(m, 128)), dim3(128), 0, st, b->table.as<G1Affine>(), m,
                       tmp.as<G1Xyzz>());
    hipError_t e = launch_batch_to_affine(tmp.as<G1Xyzz>(), m, b->table3.as<G1Affine>(), st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_table_to29, dim3(blocks_for(m, 256)), dim3(256), 0, st, b->table3.as<G1Affine>(), m);
        e = hipStreamSynchronize(st);  // tmp is released below
    }
    tmp.release();
    if (e != hipSuccess) {
        b->table3.release();
        return nullptr;
    }
    return b->table3.as<G1Affine>();
}

const G1Affine* bases_table29(const eon_msm_bases* b) {
    return b->precomputed ? b->table.as<G1Affine>() : nullptr;
}

uint32_t bases_windows(const eon_msm_bases* b) { return b->windows; }

Status bases_alloc_table(eon_ctx* ctx, uint64_t n, uint32_t c, eon_msm_bases** out) {
    if (n == 0 || n > (1ull << 27)) return Status::err(EON_E_SHAPE, "table bases need 1 <= n <= 2^27");
    auto* b = new eon_msm_bases();
    b->ctx = ctx;
    b->n = n;
    b->precomputed = true;
    b->c = c;
    b->windows = (255 + c - 1) / c;
    b->pooled = true;
    if (ctx->pool.take(b->points, n * sizeof(G1Affine)) != hipSuccess ||
        ctx->pool.take(b->table, n * b->windows * sizeof(G1Affine)) != hipSuccess) {
        bases_free(b);
        return Status::err(EON_E_OOM, "bases allocation failed");
    }
    *out = b;
    return Status::ok();
}

G1Affine* bases_table_mut(eon_msm_bases* b) { return b->table.as<G1Affine>(); }

Status bases_seal_table(eon_msm_bases* b, hipStream_t st) {
    // points = the w = 0 entries (radix-2^32 ABI form), then the table to 29-Montgomery
    EON_HIP(hipMemcpy2DAsync(b->points.p, sizeof(G1Affine), b->table.p, sizeof(G1Affine) * b->windows,
                             sizeof(G1Affine), b->n, hipMemcpyDeviceToDevice, st));
    const uint64_t m = b->n * b->windows;
    hipLaunchKernelGGL(k_table_to29, dim3(blocks_for(m, 256)), dim3(256), 0, st, b->table.as<G1Affine>(), m);
    EON_HIP(hipGetLastError());
    return Status::ok();
}

void bases_free(eon_msm_bases* b) {
    if (b->pooled) {  // the caller has synchronised the context's streams
        b->ctx->pool.give(b->points);
        b->ctx->pool.give(b->table);
    }
    b->points.release();
    b->table.release();
    b->table3.release();
    b->points29.release();
    delete b;
}

uint32_t bases_window(const eon_msm_bases* b) { return b->c; }

bool bases_precomputed(const eon_msm_bases* b) { return b->precomputed; }

static SortedBufs& wks_sorted(eon_ctx* ctx, size_t w) {
    MsmWork* wks[3] = {&ctx->msm, &ctx->msm_b, &ctx->msm_c};
    return wks[w]->sorted;
}

// ---- host-side XYZZ -> affine for a call's few results ------------------------------------------
// A device conversion of a handful of points is one thread's Fermat inversion: ~380 dependent
// products, ~0.5 ms of latency per call (0.7 ms of a 2^20 MSM's 3.5).  The results travel to the
// host anyway, so they are converted there: Montgomery batch inversion with 64-bit limbs (the same
// R = 2^256 residues, so the bytes equal the device conversion's).
namespace hostq {

static F from_dev(const Fq& a) {
    F r;
    for (int i = 0; i < 4; i++) r.l[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
    return r;
}

static Fq to_dev(const F& a) {
    Fq r;
    for (int i = 0; i < 4; i++) {
        r.v[2 * i] = (uint32_t)a.l[i];
        r.v[2 * i + 1] = (uint32_t)(a.l[i] >> 32);
    }
    return r;
}

// out[i] = affine(in[i]) (x = X / ZZ, y = Y / ZZZ; the identity -> (0, 0))
static void batch_to_affine(const G1Xyzz* in, uint64_t m, G1Affine* out) {
    std::vector<F> pre(m);
    F acc{{0, 0, 0, 0}};
    bool any = false;
    for (uint64_t i = 0; i < m; i++) {
        pre[i] = acc;
        const F zzz = from_dev(in[i].ZZZ);
        if (is_zero(from_dev(in[i].ZZ))) continue;
        acc = any ? mul(acc, zzz) : zzz;
        any = true;
    }
    if (!any) {
        for (uint64_t i = 0; i < m; i++) out[i] = G1Affine{Fq::zero(), Fq::zero()};
        return;
    }
    F inv = inverse(acc);  // 1 / prod ZZZ over the non-identity points
    for (uint64_t i = m; i-- > 0;) {
        if (is_zero(from_dev(in[i].ZZ))) {
            out[i] = G1Affine{Fq::zero(), Fq::zero()};
            continue;
        }
        const F zzz = from_dev(in[i].ZZZ);
        // pre[i] = product of the earlier non-identity ZZZ (zero when there is none)
        const bool first_live = is_zero(pre[i]);
        const F inv_zzz = first_live ? inv : mul(inv, pre[i]);
        if (!first_live) inv = mul(inv, zzz);
        const F inv_z = mul(from_dev(in[i].ZZ), inv_zzz);  // ZZ / ZZZ = 1 / Z
        out[i].x = to_dev(mul(from_dev(in[i].X), mul(inv_z, inv_z)));
        out[i].y = to_dev(mul(from_dev(in[i].Y), inv_zzz));
    }
}

}  // namespace hostq

// device XYZZ results -> affine on the host (synchronises `st`)
static Status results_to_host_affine(const G1Xyzz* dev, uint64_t m, G1Affine* out_host, hipStream_t st) {
    std::vector<G1Xyzz> h(m);
    EON_HIP(hipMemcpyAsync(h.data(), dev, m * sizeof(G1Xyzz), hipMemcpyDeviceToHost, st));
    EON_HIP(hipStreamSynchronize(st));
    hostq::batch_to_affine(h.data(), m, out_host);
    return Status::ok();
}

void host_xyzz_to_affine(const G1Xyzz* in, uint64_t m, G1Affine* out) { hostq::batch_to_affine(in, m, out); }

static Status identity_columns(uint32_t width, G1Affine* out_host) {
    // G1::multi_exp returns the identity for empty input (curve.rs:163-165)
    for (uint32_t j = 0; j < width; j++) {
        out_host[j].x = Fq::zero();
        out_host[j].y = Fq::zero();
    }
    return Status::ok();
}

Status msm_run_columns(eon_ctx* ctx, const eon_msm_bases* b, const Fr* scalars, uint64_t n,
                       uint32_t width, G1Affine* out_host, eon_msm_scalars* keep) {
    if (n > b->n) return Status::err(EON_E_SHAPE, "more scalars than bases");
    if (keep) {
        keep->ctx = ctx;
        keep->n = n;
        keep->width = width;
        keep->layout = msm_layout(b, n ? n : 1, width ? width : 1);
    }
    if (width == 0) return Status::ok();
    if (n == 0) return out_host ? identity_columns(width, out_host) : Status::ok();
    const MsmLayout L = msm_layout(b, n, width);
    // every batch leaves XYZZ results; one batched XYZZ -> affine conversion at the end (the
    // conversion is an inversion-latency-bound launch, so it is paid once per call)
    EON_HIP(ctx->msm.results.ensure(width * (sizeof(G1Affine) + sizeof(G1Xyzz))));
    G1Affine* res = ctx->msm.results.as<G1Affine>();
    G1Xyzz* res_xyzz = reinterpret_cast<G1Xyzz*>(res + width);
    std::vector<Batch> batches = make_batches(scalars, width, L.cpb);
    for (Batch& bt : batches) bt.out = res_xyzz + bt.col0;
    // a single MSM digitises only the windows its largest scalar reaches (the signed recoding
    // carries at most one bit past it): scalars < 2^64, as in kzg/benches, need 5 of 16 windows
    // of 16 bits.  One OR-reduction over the scalars and a 32-byte read-back.
    static const bool all_windows = getenv("EON_MSM_ALL_WINDOWS") != nullptr;
    if (width == 1 && !keep && !all_windows) {
        constexpr size_t or_bytes = SCALAR_OR_COPIES * 8 * 4;
        EON_HIP(ctx->msm.stat.ensure(std::max<size_t>(64, or_bytes)));
        EON_HIP(hipMemsetAsync(ctx->msm.stat.p, 0, or_bytes, ctx->stream));
        const unsigned blocks = (unsigned)std::min<uint64_t>(blocks_for(n, 256), 4096);
        hipLaunchKernelGGL(k_scalar_or, dim3(blocks), dim3(256), 0, ctx->stream, scalars, n,
                           ctx->msm.stat.as<uint32_t>());
        EON_HIP(hipGetLastError());
        if (!ctx->msm.or_host) EON_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->msm.or_host), or_bytes));
        EON_HIP(hipMemcpyAsync(ctx->msm.or_host, ctx->msm.stat.p, or_bytes, hipMemcpyDeviceToHost, ctx->stream));
        EON_HIP(hipStreamSynchronize(ctx->stream));
        uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t k = 0; k < SCALAR_OR_COPIES; k++)
            for (int j = 0; j < 8; j++) h[j] |= ctx->msm.or_host[k * 8 + j];
        uint32_t bits = 0;
        for (int j = 7; j >= 0 && !bits; j--)
            if (h[j]) bits = 32 * j + 32 - __builtin_clz(h[j]);
        batches[0].w_act = std::max<uint32_t>(1, std::min<uint32_t>(L.W, (bits + 1 + L.c - 1) / L.c));
    }
    // sorted pairs land in the workspace of batch k % 3, or, when kept, in buffers of their own
    if (keep) {
        keep->sorted.resize(batches.size());
        for (auto& sb : keep->sorted) {
            if (ctx->sorted_cache.empty()) break;
            sb = std::move(ctx->sorted_cache.back());
            ctx->sorted_cache.back() = SortedBufs{};
            ctx->sorted_cache.pop_back();
        }
    }
    auto sorted_of = [&](size_t k) -> SortedBufs& { return keep ? keep->sorted[k] : wks_sorted(ctx, k % 3); };
    // Three streams: every digit sort on the high-priority sort stream, piece sums + reductions
    // alternating between the context stream and the side stream.  Three workspaces (batch k uses
    // k % 3): sort(k+1) only waits for reduce(k-2).  Events order sort(k) after reduce(k - 3)
    // and pieces(k) after sort(k).
    hipStream_t comp[2] = {ctx->stream, ctx->side(ctx->msm_side)};
    hipStream_t sort_st = ctx->side(ctx->msm_sort);
    MsmWork* wks[3] = {&ctx->msm, &ctx->msm_b, &ctx->msm_c};
    EON_HIP(hipEventRecord(ctx->msm_ev[0], ctx->stream));  // scalars and earlier work are ready
    EON_HIP(hipStreamWaitEvent(sort_st, ctx->msm_ev[0], 0));
    for (hipStream_t st : comp)
        if (st != ctx->stream) EON_HIP(hipStreamWaitEvent(st, ctx->msm_ev[0], 0));
    // wait: read the batch's counts back before returning (otherwise batch_pieces does, after
    // launching its piece sums over all pairs: the first batch's read-back then overlaps them)
    auto sort_batch = [&](size_t k, bool wait) -> Status {
        const int w = (int)(k % 3);
        if (k >= 3) EON_HIP(hipStreamWaitEvent(sort_st, ctx->msm_reduced[w], 0));
        EON_TRY(batch_sort(ctx, L, n, width, batches[k], *wks[w], sorted_of(k), sort_st, ctx->msm_sorted[w]));
        if (wait) EON_TRY(batch_counts(ctx, batches[k], *wks[w], n));
        return Status::ok();
    };
    auto pieces = [&](size_t k) -> Status {
        const int i = (int)(k & 1), w = (int)(k % 3);
        EON_HIP(hipStreamWaitEvent(comp[i], ctx->msm_sorted[w], 0));
        return batch_pieces(ctx, b, batches[k], sorted_ref(sorted_of(k)), *wks[w], comp[i]);
    };
    DeferredFinish df;
    EON_TRY(prepare_deferred(ctx, L, width, res_xyzz, df));
    EON_TRY(sort_batch(0, false));
    for (size_t k = 0; k < batches.size(); k++) {
        const int i = (int)(k & 1), w = (int)(k % 3);
        // pieces(k + 1) is enqueued only after reduce(k)'s read-backs: launched earlier it starves
        // the latency-bound reduction (measured +20 ms per prove)
        EON_TRY(pieces(k));
        if (k + 1 < batches.size()) EON_TRY(sort_batch(k + 1, true));
        EON_TRY(batch_reduce(ctx, L, batches[k], sorted_ref(sorted_of(k)), *wks[w], comp[i],
                             fused_reduce(batches[k]), &df));
        EON_HIP(hipEventRecord(ctx->msm_reduced[w], comp[i]));
    }
    // the context stream resumes after both compute streams' last reductions
    for (int i = 0; i < 2; i++) {
        if (comp[i] == ctx->stream) continue;
        EON_HIP(hipEventRecord(ctx->msm_ev[1 + i], comp[i]));
        EON_HIP(hipStreamWaitEvent(ctx->stream, ctx->msm_ev[1 + i], 0));
    }
    EON_TRY(run_deferred_finish(ctx, df, ctx->stream));
    if (keep) {
        keep->batches = batches;
        for (Batch& bt : keep->batches) bt.scalars = nullptr;
    }
    (void)res;
    if (out_host) return results_to_host_affine(res_xyzz, width, out_host, ctx->stream);
    EON_HIP(hipStreamSynchronize(ctx->stream));
    return Status::ok();
}

// out_host[t * width + j] = MSM of column j against bases[t]
Status msm_run_prepared(eon_ctx* ctx, const eon_msm_bases* const* bases, uint32_t nbases,
                        const eon_msm_scalars* s, G1Affine* out_host) {
    const uint32_t width = s->width;
    if (width == 0 || nbases == 0) return Status::ok();
    for (uint32_t t = 0; t < nbases; t++) {
        const eon_msm_bases* b = bases[t];
        if (!b) return Status::err(EON_E_ARG, "null bases");
        if (s->n > b->n) return Status::err(EON_E_SHAPE, "more scalars than bases");
        const MsmLayout L = msm_layout(b, s->n ? s->n : 1, width);
        if (L.c != s->layout.c || L.precomputed != s->layout.precomputed)
            return Status::err(EON_E_SHAPE, "bases window layout differs from the prepared scalars'");
    }
    if (s->n == 0) {
        for (uint32_t t = 0; t < nbases; t++) identity_columns(width, out_host + (uint64_t)t * width);
        return Status::ok();
    }
    const uint64_t total = (uint64_t)width * nbases;
    EON_HIP(ctx->msm.results.ensure(total * (sizeof(G1Affine) + sizeof(G1Xyzz))));
    G1Affine* res = ctx->msm.results.as<G1Affine>();
    G1Xyzz* res_xyzz = reinterpret_cast<G1Xyzz*>(res + total);
    // Jobs (batch k, bases t) round-robin over NS = 3 streams and workspaces, enqueued without a
    // host wait (the reductions have no read-backs); a workspace is reused only by its own
    // stream, NS jobs later.
    constexpr uint32_t NS = 3;
    hipStream_t comp[NS] = {ctx->stream, ctx->side(ctx->msm_side), ctx->side(ctx->msm_side2)};
    MsmWork* wks[NS] = {&ctx->msm, &ctx->msm_b, &ctx->msm_c};
    DeferredFinish df;
    EON_TRY(prepare_deferred(ctx, s->layout, total, res_xyzz, df));
    EON_HIP(hipEventRecord(ctx->msm_ev[0], ctx->stream));
    for (uint32_t i = 1; i < NS; i++) EON_HIP(hipStreamWaitEvent(comp[i], ctx->msm_ev[0], 0));
    for (size_t k = 0; k < s->batches.size(); k++)
        for (uint32_t t = 0; t < nbases; t++) {
            const size_t j = k * nbases + t;
            hipStream_t st = comp[j % NS];
            Batch bt = s->batches[k];
            bt.out = res_xyzz + (uint64_t)t * width + bt.col0;
            const SortedRef sr = sorted_ref(s->sorted[k]);
            EON_TRY(batch_pieces(ctx, bases[t], bt, sr, *wks[j % NS], st));
            EON_TRY(batch_reduce(ctx, s->layout, bt, sr, *wks[j % NS], st, fused_reduce(bt), &df));
        }
    for (uint32_t i = 1; i < NS; i++) {
        EON_HIP(hipEventRecord(ctx->msm_ev[1], comp[i]));
        EON_HIP(hipStreamWaitEvent(ctx->stream, ctx->msm_ev[1], 0));
    }
    EON_TRY(run_deferred_finish(ctx, df, ctx->stream));
    (void)res;
    return results_to_host_affine(res_xyzz, total, out_host, ctx->stream);
}

Status msm_run(eon_ctx* ctx, const eon_msm_bases* b, const Fr* scalars, uint64_t n,
               G1Affine* result) {
    return msm_run_columns(ctx, b, scalars, n, 1, result, nullptr);
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
    eon::bases_free(b);
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
    Status s = msm_run_columns(ctx, bases, reinterpret_cast<const Fr*>(mat), rows, width, r.data(), nullptr);
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
        return msm_run_columns(ctx, bases, ctx->stage_in.as<Fr>(), rows, width, r.data(), nullptr);
    }();
    if (!s.bad())
        for (uint32_t j = 0; j < width; j++) out[j] = g1_to_abi(r[j]);
    return finish(ctx, s);
}

int eon_msm_g1_columns_prepare_dev(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* mat,
                                   uint64_t rows, uint32_t width, eon_g1_affine* out,
                                   eon_msm_scalars** prepared) {
    if (!ctx) return EON_E_ARG;
    if (!bases || !prepared || (rows && width && !mat)) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    auto* keep = new eon_msm_scalars();
    std::vector<G1Affine> r(width);
    Status s = msm_run_columns(ctx, bases, reinterpret_cast<const Fr*>(mat), rows, width,
                               out ? r.data() : nullptr, keep);
    if (s.bad()) {
        delete keep;
        return finish(ctx, s);
    }
    if (out)
        for (uint32_t j = 0; j < width; j++) out[j] = g1_to_abi(r[j]);
    *prepared = keep;
    return EON_OK;
}

void eon_msm_scalars_destroy(eon_msm_scalars* s) {
    if (!s) return;
    if (s->ctx) {
        std::lock_guard<std::mutex> lk(s->ctx->mu);
        (void)hipSetDevice(s->ctx->device);
        (void)hipStreamSynchronize(s->ctx->stream);
        delete s;
        return;
    }
    delete s;
}

int eon_msm_g1_columns_prepared(eon_ctx* ctx, const eon_msm_bases* const* bases, uint32_t nbases,
                                const eon_msm_scalars* prepared, eon_g1_affine* out) {
    if (!ctx) return EON_E_ARG;
    if (!prepared || (nbases && !bases) || (nbases && prepared->width && !out)) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    if (prepared->ctx && prepared->ctx != ctx) return finish(ctx, Status::err(EON_E_ARG, "prepared scalars of another context"));
    const uint64_t total = (uint64_t)nbases * prepared->width;
    std::vector<G1Affine> r(total);
    Status s = msm_run_prepared(ctx, bases, nbases, prepared, r.data());
    if (!s.bad())
        for (uint64_t j = 0; j < total; j++) out[j] = g1_to_abi(r[j]);
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
