// One onesweep pass of the LSD radix sort (sort.hip) as a device template over the source of its
// pairs, so that a producer can rank the pairs it computes without writing them first: sort.hip
// instantiates it over stored (key, value) arrays, msm.hip over the MSM's digit pairs computed from
// the scalars (the digit extraction fused into the first pass).
//
// A 1024-thread block takes the next tile of 16384 pairs (a virtual tile index from an atomic
// counter, so every earlier tile is already running), each wave ranks its 1024 pairs slot by slot
// -- the lanes holding the same digit found by one ballot per digit bit, the per-wave digit
// counters in LDS -- publishes the tile's digit counts, scatters the pairs into LDS in digit
// order, and then finds the digit's global offset by a decoupled look-back over the preceding
// tiles' published counts (a 2-bit flag and a 62-bit count in one 64-bit word: aggregate or
// inclusive).  The tile's pairs leave LDS in digit runs, so the global writes are contiguous per
// run.  Order: the pairs are ranked in (wave, slot, lane) order and the tiles in tile order, so a
// source whose item (w, j, lane) of tile t is pair t 16384 + w 1024 + j 64 + lane sorts stably.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <type_traits>

#include "sort.h"

namespace eon {
namespace sortpass {

// threads per sort tile (16 pairs each): 1024 -- half the tiles of 512, so half the look-back
// steps, at one 146-KB block of 16 waves per CU instead of two of 8: sort 2^28 x 16 bits 2.77 ->
// 2.47 ms, sort passes 25.6 -> 23.5 ms per prove, prove unchanged (profiles/r05/s26)
#ifndef EON_SORT_THREADS
#define EON_SORT_THREADS 1024
#endif
constexpr uint32_t SORT_THREADS = EON_SORT_THREADS, SORT_WAVES = SORT_THREADS / 64, SORT_ITEMS = 16;
constexpr uint32_t SORT_TILE = SORT_THREADS * SORT_ITEMS;
constexpr uint64_t ST_AGG = 1ull << 62, ST_INC = 2ull << 62, ST_COUNT = (1ull << 62) - 1;
static_assert(SORT_THREADS == 512 || SORT_THREADS == 1024, "tile threads");
static_assert(RADIX_SORT_MAX_PAIRS <= (1ull << 32) - SORT_TILE, "the last tile's indices must not wrap");
constexpr size_t SORT_LDS = (size_t)SORT_TILE * 8 + SORT_WAVES * 256 * 4 + 2 * 256 * 4 + 64;
// LDS bytes of a tile of THREADS x ITEMS pairs
constexpr size_t sort_lds_bytes(uint32_t threads, uint32_t items) {
    return (size_t)threads * items * 8 + threads / 64 * 256 * 4 + 2 * 256 * 4 + 64;
}
// The lean tile (EON_SORT_LEAN): 256 threads x 2 pairs in <= 32 VGPRs, so that a block fits beside
// the piece sums (4 waves x 120 VGPRs per SIMD) and the pass runs under them instead of alone
// EON_SORT_LEAN=1: every pass of the digit sort (and the MSM's fused digit pass) runs in lean tiles
#ifndef EON_SORT_LEAN
#define EON_SORT_LEAN 0
#endif
#ifndef EON_SORT_LEAN_ITEMS
#define EON_SORT_LEAN_ITEMS 2
#endif
constexpr uint32_t LEAN_THREADS = 256, LEAN_ITEMS = EON_SORT_LEAN_ITEMS, LEAN_TILE = LEAN_THREADS * LEAN_ITEMS;
constexpr size_t LEAN_LDS = sort_lds_bytes(LEAN_THREADS, LEAN_ITEMS);

// inclusive scan of one value per lane across a wave64
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// exclusive scan of v over threads [0, 256) of the block (every thread of the block calls it;
// threads >= 256 pass 0 and get garbage); `tot` receives the sum of the 256 values
__device__ __forceinline__ uint32_t scan256(uint32_t v, uint32_t* wsum, uint32_t& tot) {
    const uint32_t incl = wave_incl_scan(v);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63 && w < 4) wsum[w] = incl;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) off += i < w ? wsum[i] : 0;
    tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return off + incl - v;
}

__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_status(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Stored pairs: item (w, j, lane) of tile t is pair t SORT_TILE + w 64 SORT_ITEMS + j 64 + lane
struct PairSource {
    const uint32_t* __restrict__ ks;
    const uint32_t* __restrict__ vs;
    template <bool FULL, uint32_t THREADS = SORT_THREADS, uint32_t ITEMS = SORT_ITEMS>
    __device__ __forceinline__ void load(uint32_t tile, uint32_t w, uint32_t lane, uint32_t n,
                                         uint32_t (&key)[ITEMS], uint32_t (&val)[ITEMS]) const {
        const uint32_t wbase = tile * (THREADS * ITEMS) + w * 64 * ITEMS;
#pragma unroll
        for (uint32_t j = 0; j < ITEMS; j++) {
            const uint32_t i = wbase + j * 64 + lane;
            key[j] = (FULL || i < n) ? ks[i] : 0u;
            val[j] = (FULL || i < n) ? vs[i] : 0u;
        }
    }
};

// One pass over key bits [shift, shift + dbits) of n pairs from `src` into (kd, vd).  DBITS > 0:
// the pass's digit width as a compile-time constant (the MSM's 8-bit passes): the ranking's
// per-bit loop then has no branch on the width (each `b < dbits` test was a VALU compare, wait
// states and a branch per bit and item); DBITS = 0 reads it from `dbits_rt`.  `base`: the digits'
// first output positions (the exclusive scan of the pass's histogram); status / tile_ctr zeroed.
template <uint32_t DBITS, class Src, uint32_t SORT_THREADS = sortpass::SORT_THREADS,
          uint32_t SORT_ITEMS = sortpass::SORT_ITEMS>
__device__ __forceinline__ void sort_pass_tile(const Src& src, uint32_t* __restrict__ kd, uint32_t* __restrict__ vd,
                                               uint32_t n, uint32_t shift, uint32_t dbits_rt,
                                               const uint32_t* __restrict__ base, uint64_t* status,
                                               uint32_t* tile_ctr) {
    constexpr uint32_t SORT_WAVES = SORT_THREADS / 64, SORT_TILE = SORT_THREADS * SORT_ITEMS;
    static_assert(SORT_THREADS >= 256, "the per-digit steps take threads 0..255");
    const uint32_t dbits = DBITS ? DBITS : dbits_rt;
    extern __shared__ uint32_t lds[];
    uint32_t* sk = lds;                                 // SORT_TILE keys in digit order
    uint32_t* sv = sk + SORT_TILE;                      // and their values
    uint32_t(*cnt)[256] = reinterpret_cast<uint32_t(*)[256]>(sv + SORT_TILE);  // per-wave digit counters
    uint32_t* tstart = &cnt[SORT_WAVES][0];             // digit's first slot in the tile
    uint32_t* goff = tstart + 256;                      // digit's first global position
    uint32_t* misc = goff + 256;                        // [0] tile index, [4..8) wave sums
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t dmask = (1u << dbits) - 1;
    for (uint32_t i = tid; i < SORT_WAVES * 256; i += SORT_THREADS) (&cnt[0][0])[i] = 0;
    if (tid == 0) misc[0] = atomicAdd(tile_ctr, 1u);
    __syncthreads();
    const uint32_t tile = misc[0];
    const uint32_t t0 = tile * SORT_TILE;
    const uint32_t wbase = t0 + w * 64 * SORT_ITEMS;
    // every tile but the last is full: its copy of the body has no per-item bounds checks
    auto body = [&](auto full_tag) __attribute__((always_inline)) {
        constexpr bool FULL = decltype(full_tag)::value;
        uint32_t key[SORT_ITEMS], val[SORT_ITEMS], rk[SORT_ITEMS];
        if constexpr (SORT_ITEMS == sortpass::SORT_ITEMS && SORT_THREADS == sortpass::SORT_THREADS)
            src.template load<FULL>(tile, w, lane, n, key, val);
        else
            src.template load<FULL, SORT_THREADS, SORT_ITEMS>(tile, w, lane, n, key, val);
#pragma unroll
        for (uint32_t j = 0; j < SORT_ITEMS; j++) {
            const bool valid = FULL || wbase + j * 64 + lane < n;
            const uint32_t d = (key[j] >> shift) & dmask;
            // the lanes holding the same digit: per digit bit, the ballot m of the bit and this
            // lane's bit as an all-ones / zero word s; eq &= m XNOR s on 32-bit halves (the
            // compiler folds the bits with v_xor / v_or3 / v_bitop3: ~5 VALU per bit, against ~10
            // for the 64-bit select form bit ? m : ~m)
            const uint64_t vm = __ballot(valid);
            uint32_t eq_lo = (uint32_t)vm, eq_hi = (uint32_t)(vm >> 32);
#pragma unroll
            for (uint32_t b = 0; b < 8; b++) {
                if (b < dbits) {
                    const int32_t sb = (int32_t)(d << (31 - b)) >> 31;
                    const uint64_t m = __ballot(sb != 0);
                    eq_lo &= ~((uint32_t)m ^ (uint32_t)sb);
                    eq_hi &= ~((uint32_t)(m >> 32) ^ (uint32_t)sb);
                }
            }
            // lanes below this one in the group (v_mbcnt), and the group's size
            const uint32_t before = __builtin_amdgcn_mbcnt_hi(eq_hi, __builtin_amdgcn_mbcnt_lo(eq_lo, 0u));
            const uint32_t old = valid ? cnt[w][d] : 0u;
            // every lane of the group has read the counter before its lowest lane moves it
            if (valid && before == 0) cnt[w][d] = old + (uint32_t)(__popc(eq_lo) + __popc(eq_hi));
            rk[j] = old + before;
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        // per digit: the waves' counts -> exclusive wave offsets, the tile's count
        uint32_t tcount = 0;
        if (tid < 256) {
#pragma unroll
            for (uint32_t v = 0; v < SORT_WAVES; v++) {
                const uint32_t c = cnt[v][tid];
                cnt[v][tid] = tcount;
                tcount += c;
            }
            // publish this tile's counts before anything else, so the next tiles can look back
            st_status(status + (size_t)tile * 256 + tid, (tile == 0 ? ST_INC : ST_AGG) | (uint64_t)tcount);
        }
        uint32_t tot;
        const uint32_t ts = scan256(tid < 256 ? tcount : 0u, misc + 4, tot);
        if (tid < 256) tstart[tid] = ts;
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < SORT_ITEMS; j++) {
            if (FULL || wbase + j * 64 + lane < n) {
                const uint32_t d = (key[j] >> shift) & dmask;
                const uint32_t pos = tstart[d] + cnt[w][d] + rk[j];
                sk[pos] = key[j];
                sv[pos] = val[j];
            }
        }
        if (tid < 256) {
            uint32_t excl = 0;
            if (tile > 0) {
                for (uint32_t k = tile - 1;; k--) {
                    uint64_t v;
                    while (((v = ld_status(status + (size_t)k * 256 + tid)) >> 62) == 0) __builtin_amdgcn_s_sleep(1);
                    excl += (uint32_t)(v & ST_COUNT);  // a digit's running count is below n < 2^32
                    if (v & ST_INC) break;
                }
                st_status(status + (size_t)tile * 256 + tid, ST_INC | (uint64_t)(excl + tcount));
            }
            goff[tid] = base[tid] + excl;
        }
        __syncthreads();
        const uint32_t valid_n = FULL ? SORT_TILE : min(SORT_TILE, n - t0);
        for (uint32_t i = tid; i < valid_n; i += SORT_THREADS) {
            const uint32_t k = sk[i];
            const uint32_t d = (k >> shift) & dmask;
            const uint32_t dst = goff[d] + i - tstart[d];
            if (dst < n) {  // always, for a consistent ranking: the output is never written out of range
                kd[dst] = k;
                vd[dst] = sv[i];
            }
        }
    };
    if (t0 + SORT_TILE <= n)
        body(std::true_type{});
    else
        body(std::false_type{});
}

}  // namespace sortpass
}  // namespace eon
