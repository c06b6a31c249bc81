// Device-wide primitives of the MSM digit pipeline, written for gfx950 (no library sort / scan on
// the hot path): a stable LSD radix sort of (u32 key, u32 value) pairs and an exclusive sum of u32.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace eon {

// Largest n radix_sort_pairs takes: u32 positions, the last tile's indices must not wrap.
constexpr uint64_t RADIX_SORT_MAX_PAIRS = (1ull << 32) - 8192;

// Scratch bytes of radix_sort_pairs for n pairs sorted on `bits` low key bits.
size_t radix_sort_temp_bytes(uint64_t n, uint32_t bits);

// Stable sort of the pairs (keys_in[i], vals_in[i]), i < n (n <= RADIX_SORT_MAX_PAIRS), by key
// bits [0, bits)
// into keys_out / vals_out; the inputs are left unchanged.  LSD passes of <= 8-bit digits (16
// bits: 2 passes); each pass is one kernel that ranks a tile of pairs in LDS and finds the tile's
// global digit offsets by a decoupled look-back over the preceding tiles, after one histogram
// kernel for every pass.  `temp` holds radix_sort_temp_bytes(n, bits) bytes.
hipError_t radix_sort_pairs(void* temp, const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, uint64_t n, uint32_t bits, hipStream_t st);

// Scratch bytes of exclusive_scan_u32 for n elements.
size_t exclusive_scan_temp_bytes(uint64_t n);

// out[i] = in[0] + ... + in[i-1] (out[0] = 0), n < 2^32, sums modulo 2^32; in != out.
hipError_t exclusive_scan_u32(void* temp, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st);

}  // namespace eon
