// Device-wide primitives of the MSM digit pipeline, written for gfx950 (no library sort / scan on
// the hot path): a stable LSD radix sort of (u32 key, u32 value) pairs and an exclusive sum of u32.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace eon {

// Largest n radix_sort_pairs takes: u32 positions, the last tile's indices must not wrap (tiles
// of up to 16384 pairs).
constexpr uint64_t RADIX_SORT_MAX_PAIRS = (1ull << 32) - 16384;

// The LSD passes of a sort on `bits` low key bits: pass p sorts key bits [shift[p], shift[p] +
// bits[p]) (<= 8 bits each).  A producer of the keys may count every pass's 256-bin histogram
// itself (radix_sort_histograms: hist[p * 256 + digit], zeroed first) and then call
// radix_sort_pairs with hist_ready, which skips the sort's own histogram read of the keys.
constexpr uint32_t RADIX_SORT_MAX_PASSES = 4;
struct RadixPasses {
    uint32_t shift[RADIX_SORT_MAX_PASSES], bits[RADIX_SORT_MAX_PASSES];
    uint32_t passes;
};
RadixPasses radix_sort_passes(uint32_t bits);
uint32_t* radix_sort_histograms(void* temp, uint64_t n);

// Scratch bytes of radix_sort_pairs for n pairs sorted on `bits` low key bits.
size_t radix_sort_temp_bytes(uint64_t n, uint32_t bits);

// Stable sort of the pairs (keys_in[i], vals_in[i]), i < n (n <= RADIX_SORT_MAX_PAIRS), by key
// bits [0, bits)
// into keys_out / vals_out; the inputs are left unchanged.  LSD passes of <= 8-bit digits (16
// bits: 2 passes); each pass is one kernel that ranks a tile of pairs in LDS and finds the tile's
// global digit offsets by a decoupled look-back over the preceding tiles, after one histogram
// kernel for every pass.  `temp` holds radix_sort_temp_bytes(n, bits) bytes.
hipError_t radix_sort_pairs(void* temp, const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, uint64_t n, uint32_t bits, hipStream_t st, bool hist_ready = false);

// A sort whose FIRST pass is run by the producer of the pairs over pairs it computes instead of
// stored ones (sort_pass.h's sort_pass_tile over its own source, one block of SORT_THREADS threads
// and SORT_LDS bytes of LDS per tile, radix_sort_pass_args(.., 0).tiles tiles; the MSM's digit
// pairs, msm.hip).  The histograms of every pass ready in radix_sort_histograms(temp, n):
//   radix_sort_prepare  the digit offsets of every pass and the zeroed look-back state;
//   (the producer's first pass, with radix_sort_pass_args(temp, n, bits, 0))
//   radix_sort_tail     passes 1 .. from the first pass's output (>= 2 passes), the last one into
//                       keys_out / vals_out.
struct RadixPassArgs {
    uint32_t shift, bits;
    const uint32_t* base;  // the pass's 256 digit offsets
    uint64_t* status;      // its tiles' look-back words (zeroed by radix_sort_prepare)
    uint32_t* tile_ctr;    // its virtual tile counter
    uint32_t tiles;
};
hipError_t radix_sort_prepare(void* temp, uint64_t n, uint32_t bits, hipStream_t st);
RadixPassArgs radix_sort_pass_args(void* temp, uint64_t n, uint32_t bits, uint32_t q);
hipError_t radix_sort_tail(void* temp, const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_out,
                           uint32_t* vals_out, uint64_t n, uint32_t bits, hipStream_t st);

// Scratch bytes of exclusive_scan_u32 for n elements.
size_t exclusive_scan_temp_bytes(uint64_t n);

// out[i] = in[0] + ... + in[i-1] (out[0] = 0), n < 2^32, sums modulo 2^32; in != out.
hipError_t exclusive_scan_u32(void* temp, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st);

// The MSM's piece offsets: the exclusive scan (nb + 1 outputs, exclusive_scan_temp_bytes(nb + 1)
// scratch) of count[b] = the 2^log_chunk-aligned runs bucket b's pairs [start[b], start[b + 1])
// touch (0 if empty; count[nb] = 0), computed from `start` on the fly -- no count array -- and
// *max_out raised to the largest count when that exceeds 1 (max_out zeroed before).
hipError_t exclusive_scan_chunk_counts(void* temp, const uint32_t* start, uint32_t nb, uint32_t log_chunk,
                                       uint32_t* out, uint32_t* max_out, hipStream_t st);

}  // namespace eon
