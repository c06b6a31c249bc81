// Internal NTT launch API (not part of the C ABI; see include/eon.h).
#pragma once
#include <vector>

#include "field.h"

namespace eon {

enum LoadMode : uint32_t {
    LOAD_DIRECT = 0,   // network position p reads source row p
    LOAD_BITREV = 1,   // reads source row reverse_bits(p, load_param)
    LOAD_SPREAD = 2,   // reads source row p >> load_param (LDE: bit-reversed coefficients spread)
    LOAD_ZEROPAD = 3,  // reads source row p if p < load_param, else zero
    // reads source row reverse_bits(p >> b, n) with b = load_param & 0xff, n = load_param >> 8:
    // the zero-padded natural vector's bit-reversed order after its first b DIT stages (which
    // only replicate values), for evaluating coefficients on a larger coset
    LOAD_BITREV_SPREAD = 4,
};

constexpr uint32_t NATURAL_IDX = 0xffffffffu;

// words per Shoup-quotient table entry (9 limbs of 29 bits, padded to three 16-B loads)
constexpr uint32_t TWQ_STRIDE = 12;

// One radix-2 network of size 2^log_m over `width` independent columns.
//   DIT (dif=false): stages first_stage .. log_m-1 ascending; bit-reversed input -> natural output.
//   DIF (dif=true):  stages log_m-1 .. first_stage descending; natural input -> bit-reversed output.
// The first pass reads `src` through the load transform (and may be out of place); later passes
// run in place on `dst`.
struct NetworkSpec {
    bool dif = false;
    uint32_t log_m = 0;
    uint32_t first_stage = 0;
    const Fr* src = nullptr;
    Fr* dst = nullptr;
    uint64_t width = 0;
    const Fr* tw = nullptr;         // stage-concatenated twiddles (forward or inverse), plain roots
    const uint32_t* twq = nullptr;  // their Shoup quotients, TWQ_STRIDE words per entry
    uint32_t load_mode = LOAD_DIRECT;
    uint32_t load_param = 0;
    const Fr* load_scale = nullptr;
    uint32_t has_load_const = 0;
    Fr load_const = Fr::one();
    const Fr* store_scale = nullptr;
    uint32_t max_stages_per_pass = 0;  // 0 = tile limit; tests force multi-pass plans with it
    uint32_t max_threads = 0;          // 0 = default (512, 1024 for 2048-element tiles); tuning knob
    uint32_t log_tile = 0;             // log2 elements per LDS tile (0 = 10); tuning knob
    int log_cb_override = -1;          // columns per tile = 2^log_cb; -1 = by width
    // DIT only: 36 * 2^log_m * width bytes for the unreduced 29-limb planes exchanged between the
    // passes (PassArgs::mid); null = values reduced and packed into `dst` between passes
    uint4* mid = nullptr;
};

// Optional per-launch timing (eon_ctx_profile_*): a launch is bracketed by two events.
struct LaunchRecord {
    const char* kernel;
    uint64_t alg_bytes;  // algorithmic bytes of this launch (each element read + written once)
    hipEvent_t start, stop;
    uint64_t alg_mulmods;  // algorithmic 256-bit Montgomery products of this launch (0: not counted)
    // bytes the kernel's own access pattern implies beyond alg_bytes' definition (e.g. the
    // fixed-base table gathers of k_piece_sum: 64 B per nonzero digit); 0 when equal
    uint64_t design_bytes;
};
struct Profiler {
    bool enabled = false;
    std::vector<LaunchRecord> recs;
    std::vector<hipEvent_t> pool;
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    void begin(const char* kernel, uint64_t bytes, hipStream_t st, uint64_t mulmods = 0,
               uint64_t design_bytes = 0) {
        if (!enabled) return;
        LaunchRecord r{kernel, bytes, get(), get(), mulmods, design_bytes};
        (void)hipEventRecord(r.start, st);
        recs.push_back(r);
    }
    void end(hipStream_t st) {
        if (!enabled || recs.empty()) return;
        (void)hipEventRecord(recs.back().stop, st);
    }
};

// The form in which k_ntt_pass29 takes every multiplier -- twiddle tables, load / store scale
// tables and the load constant: 32 c (in Montgomery form), so that the 29-limb product
// mul29(x, 32 c) = x c 2^256 mod p needs no conversion of the multiplier.
inline Fr ntt_scale_form(const Fr& c) { return mul(c, from_u64<FrP>(32)); }

hipError_t run_network(const NetworkSpec& s, hipStream_t st, Profiler* prof = nullptr);
// the number of passes (launches) run_network makes for `s`: a one-pass network exchanges nothing
// between passes and needs no NetworkSpec::mid
uint32_t network_passes(const NetworkSpec& s);
hipError_t launch_powers(Fr* out, uint64_t n, const Fr& base, const Fr& scale, uint32_t rev_log,
                         hipStream_t st);
hipError_t launch_twiddles(Fr* tw, uint32_t* twq, uint32_t L, const Fr& root_L, hipStream_t st);

}  // namespace eon
