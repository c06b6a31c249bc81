// Radix sort and exclusive scan for the MSM digit pipeline (sort.h), hand-written for gfx950.
//
// Radix sort (stable LSD, <= 8-bit digits; the MSM sorts its (bucket key, reference) pairs on the
// c = 16 low key bits in two passes):
//   k_sort_hist   one read of the keys: the digit histogram of every pass (LDS counters, one
//                 global atomic per bin and block)
//   k_sort_base   exclusive scan of each pass's 256 bins -> the digit's first output position
//   k_sort_pass   one launch per pass.  A 1024-thread block takes the next tile of 16384 pairs (a
//                 virtual tile index from an atomic counter, so every earlier tile is already
//                 running), each wave ranks its 1024 pairs slot by slot -- the lanes holding the
//                 same digit found by one ballot per digit bit, the per-wave digit counters in
//                 LDS -- publishes the tile's digit counts, scatters the pairs into LDS in digit
//                 order, and then finds the digit's global offset by a decoupled look-back over the
//                 preceding tiles' published counts (a 2-bit flag and a 62-bit count in one 64-bit
//                 word: aggregate or inclusive).  The tile's pairs leave LDS in digit runs, so the global
//                 writes are contiguous per run.  Stability: the slots are walked in input order
//                 (slot j of a wave covers its pairs j 64 .. j 64 + 63).
// Traffic per pass: 8 B read + 8 B written per pair (plus 4 B per pair once for the histograms).
//
// Exclusive scan (the MSM's piece offsets, <= a few million counts): per-block sums, one block
// scanning the block sums, per-block rescan + offset.
#include "sort.h"

#include <algorithm>
#include <type_traits>

namespace eon {
namespace {

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
constexpr uint32_t MAX_PASSES = RADIX_SORT_MAX_PASSES;
constexpr size_t SORT_LDS = (size_t)SORT_TILE * 8 + SORT_WAVES * 256 * 4 + 2 * 256 * 4 + 64;

using PassBits = RadixPasses;

PassBits split_bits(uint32_t bits) {
    PassBits pb{};
    pb.passes = (bits + 7) / 8;
    uint32_t s = 0;
    for (uint32_t p = 0; p < pb.passes; p++) {
        const uint32_t w = bits / pb.passes + (p < bits % pb.passes ? 1 : 0);
        pb.shift[p] = s;
        pb.bits[p] = w;
        s += w;
    }
    return pb;
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

__global__ void __launch_bounds__(512) k_sort_hist(const uint32_t* __restrict__ keys, uint32_t n, PassBits pb,
                                                   uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[MAX_PASSES][256];
    for (uint32_t i = threadIdx.x; i < MAX_PASSES * 256; i += blockDim.x) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t stride = gridDim.x * blockDim.x;
    auto count = [&](uint32_t k) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t p = 0; p < MAX_PASSES; p++)
            if (p < pb.passes) atomicAdd(&h[p][(k >> pb.shift[p]) & ((1u << pb.bits[p]) - 1)], 1u);
    };
    const uint32_t n4 = n / 4;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += stride) {
        const uint4 k = reinterpret_cast<const uint4*>(keys)[q];
        count(k.x);
        count(k.y);
        count(k.z);
        count(k.w);
    }
    for (uint32_t i = n4 * 4 + blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) count(keys[i]);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < pb.passes * 256; i += blockDim.x) {
        const uint32_t v = (&h[0][0])[i];
        if (v) atomicAdd(hist + i, v);
    }
}

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

__global__ void __launch_bounds__(256) k_sort_base(const uint32_t* __restrict__ hist, uint32_t passes,
                                                   uint32_t* __restrict__ base) {
    __shared__ uint32_t wsum[4];
    for (uint32_t p = 0; p < passes; p++) {
        uint32_t tot;
        const uint32_t e = scan256(hist[p * 256 + threadIdx.x], wsum, tot);
        base[p * 256 + threadIdx.x] = e;
    }
}

__device__ __forceinline__ void st_status(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_status(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// DBITS > 0: the pass's digit width as a compile-time constant (the MSM's 8-bit passes): the
// ranking's per-bit loop then has no branch on the width (each `b < dbits` test was a VALU compare,
// wait states and a branch per bit and item); DBITS = 0 reads it from `dbits`
template <uint32_t DBITS>
__global__ void __launch_bounds__(SORT_THREADS) k_sort_pass(const uint32_t* __restrict__ ks, const uint32_t* __restrict__ vs,
                                                            uint32_t* __restrict__ kd, uint32_t* __restrict__ vd, uint32_t n,
                                                            uint32_t shift, uint32_t dbits_rt,
                                                            const uint32_t* __restrict__ base, uint64_t* status,
                                                            uint32_t* tile_ctr) {
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
#pragma unroll
        for (uint32_t j = 0; j < SORT_ITEMS; j++) {
            const uint32_t i = wbase + j * 64 + lane;
            key[j] = (FULL || i < n) ? ks[i] : 0u;
            val[j] = (FULL || i < n) ? vs[i] : 0u;
        }
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

// ---- exclusive scan ---------------------------------------------------------------------------

constexpr uint32_t SCAN_THREADS = 256, SCAN_ITEMS = 16, SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* wsum, uint32_t& tot) {
    return scan256(v, wsum, tot);
}

// the scanned values: a u32 array, or the MSM's piece counts computed from its bucket starts
struct PlainIn {
    const uint32_t* in;
    __device__ __forceinline__ uint32_t operator()(uint64_t i) const { return in[i]; }
};
struct ChunkCountIn {
    const uint32_t* start;  // nb + 1 entries
    uint32_t nb, log_chunk;
    __device__ __forceinline__ uint32_t operator()(uint64_t b) const {
        if (b >= nb) return 0;
        const uint32_t s = start[b], e = start[b + 1];
        return s == e ? 0 : ((e - 1) >> log_chunk) - (s >> log_chunk) + 1;
    }
};

// per-block sums; with max_out, also the largest value (atomicMax, only where it exceeds 1)
template <class In>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_reduce(In in, uint64_t n, uint32_t* __restrict__ bsum,
                                                              uint32_t* max_out) {
    __shared__ uint32_t wsum[4];
    const uint64_t t0 = (uint64_t)blockIdx.x * SCAN_TILE;
    uint32_t s = 0, mx = 0;
    for (uint32_t j = 0; j < SCAN_ITEMS; j++) {
        const uint64_t i = t0 + j * SCAN_THREADS + threadIdx.x;
        const uint32_t v = i < n ? in(i) : 0u;
        s += v;
        mx = max(mx, v);
    }
    uint32_t tot;
    (void)block_excl_scan256(s, wsum, tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
    if (max_out) {
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o));
        if ((threadIdx.x & 63) == 0 && mx > 1 && mx > __atomic_load_n(max_out, __ATOMIC_RELAXED)) atomicMax(max_out, mx);
    }
}

// exclusive scan of the m block sums in place (one block)
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_top(uint32_t* bsum, uint32_t m) {
    __shared__ uint32_t wsum[4];
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < m; c0 += SCAN_THREADS) {
        const uint32_t i = c0 + threadIdx.x;
        const uint32_t v = i < m ? bsum[i] : 0u;
        uint32_t tot;
        const uint32_t e = block_excl_scan256(v, wsum, tot);
        if (i < m) bsum[i] = carry + e;
        carry += tot;
    }
}

template <class In>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_apply(In in, uint64_t n, const uint32_t* __restrict__ bsum,
                                                             uint32_t* __restrict__ out) {
    __shared__ uint32_t wsum[4];
    // blocked: thread t owns elements [t0 + t ITEMS, t0 + (t + 1) ITEMS)
    const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < SCAN_ITEMS; j++) {
        v[j] = i0 + j < n ? in(i0 + j) : 0u;
        s += v[j];
    }
    uint32_t tot;
    uint32_t run = bsum[blockIdx.x] + block_excl_scan256(s, wsum, tot);
#pragma unroll
    for (uint32_t j = 0; j < SCAN_ITEMS; j++) {
        if (i0 + j < n) out[i0 + j] = run;
        run += v[j];
    }
}

template <class In>
hipError_t scan_with(void* temp, In in, uint32_t* out, uint64_t n, uint32_t* max_out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)((n + SCAN_TILE - 1) / SCAN_TILE);
    uint32_t* bsum = static_cast<uint32_t*>(temp);
    hipLaunchKernelGGL(k_scan_reduce<In>, dim3(blocks), dim3(SCAN_THREADS), 0, st, in, n, bsum, max_out);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_THREADS), 0, st, bsum, blocks);
    hipLaunchKernelGGL(k_scan_apply<In>, dim3(blocks), dim3(SCAN_THREADS), 0, st, in, n, bsum, out);
    return hipGetLastError();
}

}  // namespace

RadixPasses radix_sort_passes(uint32_t bits) { return split_bits(bits); }

uint32_t* radix_sort_histograms(void* temp, uint64_t n) {
    return reinterpret_cast<uint32_t*>(static_cast<char*>(temp) + 2 * align256(n * 4));
}

// per pass: a 64-byte tile counter and the tiles' status words, every pass's zeroed by one memset
static size_t pass_state_bytes(uint64_t tiles) { return 64 + align256(tiles * 256 * 8); }

size_t radix_sort_temp_bytes(uint64_t n, uint32_t bits) {
    const uint64_t tiles = (n + SORT_TILE - 1) / SORT_TILE;
    const uint32_t passes = bits ? split_bits(bits).passes : 1;
    return 2 * align256(n * 4) + 2 * align256(MAX_PASSES * 256 * 4) + 256 + passes * pass_state_bytes(tiles);
}

hipError_t radix_sort_pairs(void* temp, const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, uint64_t n, uint32_t bits, hipStream_t st, bool hist_ready) {
    if (n == 0) return hipSuccess;
    if (n > RADIX_SORT_MAX_PAIRS || bits > 32) return hipErrorInvalidValue;
    if (bits == 0) {
        hipError_t e = hipMemcpyAsync(keys_out, keys_in, n * 4, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(vals_out, vals_in, n * 4, hipMemcpyDeviceToDevice, st);
        return e;
    }
    const PassBits pb = split_bits(bits);
    const uint32_t tiles = (uint32_t)((n + SORT_TILE - 1) / SORT_TILE);
    char* p = static_cast<char*>(temp);
    uint32_t* ktmp = reinterpret_cast<uint32_t*>(p);
    p += align256(n * 4);
    uint32_t* vtmp = reinterpret_cast<uint32_t*>(p);
    p += align256(n * 4);
    uint32_t* hist = reinterpret_cast<uint32_t*>(p);
    p += align256(MAX_PASSES * 256 * 4);
    uint32_t* base = reinterpret_cast<uint32_t*>(p);
    p += align256(MAX_PASSES * 256 * 4);
    p += 256;
    char* state = p;  // pass q: counter at state + q * pass_state_bytes, status words 64 bytes after
    const size_t psb = pass_state_bytes(tiles);

    hipError_t e = hipSuccess;
    if (!hist_ready) {
        if ((e = hipMemsetAsync(hist, 0, MAX_PASSES * 256 * 4, st)) != hipSuccess) return e;
        const uint32_t hblocks = (uint32_t)std::min<uint64_t>((n + 512ull * 16 - 1) / (512ull * 16), 2048);
        hipLaunchKernelGGL(k_sort_hist, dim3(hblocks), dim3(512), 0, st, keys_in, (uint32_t)n, pb, hist);
    }
    hipLaunchKernelGGL(k_sort_base, dim3(1), dim3(256), 0, st, hist, pb.passes, base);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    for (const void* k : {reinterpret_cast<const void*>(k_sort_pass<8>), reinterpret_cast<const void*>(k_sort_pass<0>)})
        if ((e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)SORT_LDS)) != hipSuccess)
            return e;
    if ((e = hipMemsetAsync(state, 0, pb.passes * psb, st)) != hipSuccess) return e;
    const uint32_t* sk = keys_in;
    const uint32_t* sv = vals_in;
    for (uint32_t q = 0; q < pb.passes; q++) {
        uint32_t* ctr = reinterpret_cast<uint32_t*>(state + q * psb);
        uint64_t* status = reinterpret_cast<uint64_t*>(state + q * psb + 64);
        // the last pass lands in the output; earlier ones alternate between the output and temp
        const bool to_out = ((pb.passes - 1 - q) & 1) == 0;
        uint32_t* dk = to_out ? keys_out : ktmp;
        uint32_t* dv = to_out ? vals_out : vtmp;
        hipLaunchKernelGGL(pb.bits[q] == 8 ? k_sort_pass<8> : k_sort_pass<0>, dim3(tiles), dim3(SORT_THREADS), SORT_LDS,
                           st, sk, sv, dk, dv, (uint32_t)n, pb.shift[q], pb.bits[q], base + q * 256, status, ctr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        sk = dk;
        sv = dv;
    }
    return hipSuccess;
}

size_t exclusive_scan_temp_bytes(uint64_t n) { return align256(((n + SCAN_TILE - 1) / SCAN_TILE + 1) * 4); }

hipError_t exclusive_scan_u32(void* temp, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st) {
    return scan_with(temp, PlainIn{in}, out, n, nullptr, st);
}

hipError_t exclusive_scan_chunk_counts(void* temp, const uint32_t* start, uint32_t nb, uint32_t log_chunk,
                                       uint32_t* out, uint32_t* max_out, hipStream_t st) {
    return scan_with(temp, ChunkCountIn{start, nb, log_chunk}, out, (uint64_t)nb + 1, max_out, st);
}

}  // namespace eon
