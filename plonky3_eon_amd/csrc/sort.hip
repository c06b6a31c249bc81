// Radix sort and exclusive scan for the MSM digit pipeline (sort.h), hand-written for gfx950.
//
// Radix sort (stable LSD, <= 8-bit digits; the MSM sorts its (bucket key, reference) pairs on the
// c = 16 low key bits in two passes):
//   k_sort_hist   one read of the keys: the digit histogram of every pass (LDS counters, one
//                 global atomic per bin and block)
//   k_sort_base   exclusive scan of each pass's 256 bins -> the digit's first output position
//   k_sort_pass   one launch per pass: sort_pass.h's tile (ranking in LDS, decoupled look-back,
//                 digit-run writes) over the stored pairs.  A producer may run the first pass
//                 itself over pairs it computes (radix_sort_prepare / radix_sort_pass_args /
//                 radix_sort_tail; the MSM's digits, msm.hip).
// Traffic per pass: 8 B read + 8 B written per pair (plus 4 B per pair once for the histograms).
//
// Exclusive scan (the MSM's piece offsets, <= a few million counts): per-block sums, one block
// scanning the block sums, per-block rescan + offset.
#include "sort.h"

#include <algorithm>
#include <type_traits>

#include "sort_pass.h"

namespace eon {
namespace {

using namespace sortpass;
constexpr uint32_t MAX_PASSES = RADIX_SORT_MAX_PASSES;

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

__global__ void __launch_bounds__(256) k_sort_base(const uint32_t* __restrict__ hist, uint32_t passes,
                                                   uint32_t* __restrict__ base) {
    __shared__ uint32_t wsum[4];
    for (uint32_t p = 0; p < passes; p++) {
        uint32_t tot;
        const uint32_t e = scan256(hist[p * 256 + threadIdx.x], wsum, tot);
        base[p * 256 + threadIdx.x] = e;
    }
}

template <uint32_t DBITS>
__global__ void __launch_bounds__(SORT_THREADS) k_sort_pass(const uint32_t* __restrict__ ks, const uint32_t* __restrict__ vs,
                                                            uint32_t* __restrict__ kd, uint32_t* __restrict__ vd, uint32_t n,
                                                            uint32_t shift, uint32_t dbits_rt,
                                                            const uint32_t* __restrict__ base, uint64_t* status,
                                                            uint32_t* tile_ctr) {
    sort_pass_tile<DBITS>(PairSource{ks, vs}, kd, vd, n, shift, dbits_rt, base, status, tile_ctr);
}

// the lean tile (sort_pass.h: LEAN_THREADS x LEAN_ITEMS pairs, at most 32 VGPRs)
template <uint32_t DBITS>
__global__ void __launch_bounds__(LEAN_THREADS) __attribute__((amdgpu_num_vgpr(32)))
k_sort_pass_lean(const uint32_t* __restrict__ ks, const uint32_t* __restrict__ vs, uint32_t* __restrict__ kd,
                 uint32_t* __restrict__ vd, uint32_t n, uint32_t shift, uint32_t dbits_rt,
                 const uint32_t* __restrict__ base, uint64_t* status, uint32_t* tile_ctr) {
    sort_pass_tile<DBITS, PairSource, LEAN_THREADS, LEAN_ITEMS>(PairSource{ks, vs}, kd, vd, n, shift, dbits_rt, base,
                                                                status, tile_ctr);
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

// tiles of a pass over n pairs (q: the pass index)
static uint64_t pass_tiles(uint64_t n, uint32_t q) {
    (void)q;
    const uint32_t tile = EON_SORT_LEAN ? LEAN_TILE : SORT_TILE;
    return (n + tile - 1) / tile;
}

// per pass: a 64-byte tile counter and the tiles' status words, every pass's zeroed by one memset
static size_t pass_state_bytes(uint64_t tiles) { return 64 + align256(tiles * 256 * 8); }

size_t radix_sort_temp_bytes(uint64_t n, uint32_t bits) {
    const uint64_t tiles = std::max(pass_tiles(n, 0), pass_tiles(n, 1));
    const uint32_t passes = bits ? split_bits(bits).passes : 1;
    return 2 * align256(n * 4) + 2 * align256(MAX_PASSES * 256 * 4) + 256 + passes * pass_state_bytes(tiles);
}

namespace {

// temp: [ktmp | vtmp | hist | base | 256 | pass state...]; pass q: a tile counter at
// state + q * psb, its status words 64 bytes after
struct SortLayout {
    uint32_t *ktmp, *vtmp, *hist, *base;
    char* state;
    size_t psb;
    uint32_t tiles;
    uint32_t* ctr(uint32_t q) const { return reinterpret_cast<uint32_t*>(state + q * psb); }
    uint64_t* status(uint32_t q) const { return reinterpret_cast<uint64_t*>(state + q * psb + 64); }
};

SortLayout sort_layout(void* temp, uint64_t n) {
    SortLayout L;
    L.tiles = (uint32_t)pass_tiles(n, 0);
    char* p = static_cast<char*>(temp);
    L.ktmp = reinterpret_cast<uint32_t*>(p);
    p += align256(n * 4);
    L.vtmp = reinterpret_cast<uint32_t*>(p);
    p += align256(n * 4);
    L.hist = reinterpret_cast<uint32_t*>(p);
    p += align256(MAX_PASSES * 256 * 4);
    L.base = reinterpret_cast<uint32_t*>(p);
    p += align256(MAX_PASSES * 256 * 4);
    p += 256;
    L.state = p;
    L.psb = pass_state_bytes(std::max(pass_tiles(n, 0), pass_tiles(n, 1)));
    return L;
}

// the digit offsets of every pass from the histograms, the pass state zeroed
hipError_t prepare(const SortLayout& L, const PassBits& pb, hipStream_t st) {
    hipLaunchKernelGGL(k_sort_base, dim3(1), dim3(256), 0, st, L.hist, pb.passes, L.base);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    for (const void* k : {reinterpret_cast<const void*>(k_sort_pass<8>), reinterpret_cast<const void*>(k_sort_pass<0>)})
        if ((e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)SORT_LDS)) != hipSuccess)
            return e;
    return hipMemsetAsync(L.state, 0, pb.passes * L.psb, st);
}

// passes q0 .. passes - 1 from (sk, sv): the last lands in the output, earlier ones alternate
// between the output and temp
hipError_t run_passes(const SortLayout& L, const PassBits& pb, uint32_t q0, const uint32_t* sk, const uint32_t* sv,
                      uint32_t* keys_out, uint32_t* vals_out, uint64_t n, hipStream_t st) {
    for (uint32_t q = q0; q < pb.passes; q++) {
        const bool to_out = ((pb.passes - 1 - q) & 1) == 0;
        uint32_t* dk = to_out ? keys_out : L.ktmp;
        uint32_t* dv = to_out ? vals_out : L.vtmp;
        if (EON_SORT_LEAN)
            hipLaunchKernelGGL(pb.bits[q] == 8 ? k_sort_pass_lean<8> : k_sort_pass_lean<0>, dim3((uint32_t)pass_tiles(n, q)),
                               dim3(LEAN_THREADS), LEAN_LDS, st, sk, sv, dk, dv, (uint32_t)n, pb.shift[q], pb.bits[q],
                               L.base + q * 256, L.status(q), L.ctr(q));
        else
            hipLaunchKernelGGL(pb.bits[q] == 8 ? k_sort_pass<8> : k_sort_pass<0>, dim3(L.tiles), dim3(SORT_THREADS),
                               SORT_LDS, st, sk, sv, dk, dv, (uint32_t)n, pb.shift[q], pb.bits[q], L.base + q * 256,
                               L.status(q), L.ctr(q));
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        sk = dk;
        sv = dv;
    }
    return hipSuccess;
}

}  // namespace

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
    const SortLayout L = sort_layout(temp, n);
    hipError_t e = hipSuccess;
    if (!hist_ready) {
        if ((e = hipMemsetAsync(L.hist, 0, MAX_PASSES * 256 * 4, st)) != hipSuccess) return e;
        const uint32_t hblocks = (uint32_t)std::min<uint64_t>((n + 512ull * 16 - 1) / (512ull * 16), 2048);
        hipLaunchKernelGGL(k_sort_hist, dim3(hblocks), dim3(512), 0, st, keys_in, (uint32_t)n, pb, L.hist);
    }
    if ((e = prepare(L, pb, st)) != hipSuccess) return e;
    return run_passes(L, pb, 0, keys_in, vals_in, keys_out, vals_out, n, st);
}

hipError_t radix_sort_prepare(void* temp, uint64_t n, uint32_t bits, hipStream_t st) {
    if (n == 0 || n > RADIX_SORT_MAX_PAIRS || bits == 0 || bits > 32) return hipErrorInvalidValue;
    return prepare(sort_layout(temp, n), split_bits(bits), st);
}

RadixPassArgs radix_sort_pass_args(void* temp, uint64_t n, uint32_t bits, uint32_t q) {
    const PassBits pb = split_bits(bits);
    const SortLayout L = sort_layout(temp, n);
    return RadixPassArgs{pb.shift[q], pb.bits[q], L.base + q * 256, L.status(q), L.ctr(q), L.tiles};
}

hipError_t radix_sort_tail(void* temp, const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_out,
                           uint32_t* vals_out, uint64_t n, uint32_t bits, hipStream_t st) {
    if (n == 0 || n > RADIX_SORT_MAX_PAIRS || bits == 0 || bits > 32) return hipErrorInvalidValue;
    const PassBits pb = split_bits(bits);
    if (pb.passes < 2) return hipErrorInvalidValue;
    return run_passes(sort_layout(temp, n), pb, 1, keys_in, vals_in, keys_out, vals_out, n, st);
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
