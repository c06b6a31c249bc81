// eon_ctx: per-device state behind the C ABI (streams, twiddle and coset tables, scratch).
#pragma once
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/eon.h"
#include "field.h"
#include "ntt.h"

namespace eon {

// Device buffer that only grows; freed with the context.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            bytes = 0;
        }
        hipError_t e = hipMalloc(&p, need);
        if (e == hipSuccess) bytes = need;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
};

// Exact-size cache of large transient device buffers (the KZG opening bases' tables and their
// scratch): a proof builds the same-sized buffers again, so they go back here instead of
// hipFree (which synchronises the device and costs host time) and come back instead of hipMalloc.
// Trimmed past `cap` bytes (EON_POOL_CAP_GB at context creation, default 8); emptied by
// eon_ctx_trim and with the context.
struct DevPool {
    size_t cap = size_t(8) << 30;
    std::multimap<size_t, void*> free_;
    size_t bytes = 0;
    // `b` (empty or holding a smaller buffer, which returns to the pool) gets `need` bytes
    hipError_t take(DevBuf& b, size_t need) {
        if (b.p && b.bytes >= need) return hipSuccess;
        give(b);
        auto it = free_.find(need);
        if (it != free_.end()) {
            b.p = it->second;
            b.bytes = need;
            bytes -= need;
            free_.erase(it);
            return hipSuccess;
        }
        hipError_t e = hipMalloc(&b.p, need);
        if (e == hipErrorOutOfMemory) {
            (void)hipGetLastError();
            release_all();
            e = hipMalloc(&b.p, need);
        }
        if (e == hipSuccess)
            b.bytes = need;
        else
            b.p = nullptr;
        return e;
    }
    // work still queued on b must be finished (the caller synchronises first)
    void give(DevBuf& b) {
        if (!b.p) return;
        if (bytes + b.bytes <= cap) {
            free_.emplace(b.bytes, b.p);
            bytes += b.bytes;
        } else {
            (void)hipFree(b.p);
        }
        b.p = nullptr;
        b.bytes = 0;
    }
    void release_all() {
        for (auto& kv : free_) (void)hipFree(kv.second);
        free_.clear();
        bytes = 0;
    }
};

// The buffers local to one call, taken from a DevPool and given back when the scope ends -- on
// every path, early error returns included -- after the stream that used them has drained.  The
// scope keeps its own copy of each (pointer, size) it handed out, never a reference to the
// caller's DevBuf, so the order in which the scope and the caller's buffers are declared does
// not matter (a DevBuf declared after the scope ends its lifetime first).
struct PoolScope {
    DevPool& pool;
    hipStream_t st;
    std::vector<DevBuf> owned;
    PoolScope(DevPool& p, hipStream_t s) : pool(p), st(s) {}
    PoolScope(const PoolScope&) = delete;
    PoolScope& operator=(const PoolScope&) = delete;
    // `b` must be empty: one take per buffer and scope
    hipError_t take(DevBuf& b, size_t need) {
        if (b.p) return hipErrorInvalidValue;
        hipError_t e = pool.take(b, need);
        if (e == hipSuccess) owned.push_back(b);
        return e;
    }
    ~PoolScope() {
        (void)hipStreamSynchronize(st);
        for (DevBuf& b : owned) pool.give(b);
    }
};

struct Status {
    int code = EON_OK;
    std::string msg;
    static Status ok() { return {}; }
    static Status err(int c, std::string m) { return {c, std::move(m)}; }
    bool bad() const { return code != EON_OK; }
};

// device workspace of one MSM pipeline run (msm.hip); grows on demand, reused across calls
// A batch's sorted digit pairs: keys / values by bucket, bucket starts, piece offsets.  Owned by
// a workspace (streaming path) or by an eon_msm_scalars cache (prepared path, reused by every MSM
// of the same scalars against other bases).
struct SortedBufs {
    DevBuf keys2, vals2, start, piece_off;
    size_t bytes() const { return keys2.bytes + vals2.bytes + start.bytes + piece_off.bytes; }
    void release() {
        keys2.release();
        vals2.release();
        start.release();
        piece_off.release();
    }
};

struct MsmWork {
    DevBuf keys, vals, count, off2, off3, owner, piece_sums, piece_sums2, bucket_sums, red_a, red_b,
        temp, results, piece_raw, stat;
    DevBuf canon;  // canonical scalars, column-major (the fused digit sort, msm.hip)
    SortedBufs sorted;
    uint32_t* host_counts = nullptr;  // pinned read-back slots
    hipEvent_t counts_ev = nullptr;   // recorded after the count read-back's copies
    uint32_t* or_host = nullptr;      // pinned read-back of k_scalar_or's copies
    void release() {
        if (host_counts) (void)hipHostFree(host_counts);
        host_counts = nullptr;
        if (or_host) (void)hipHostFree(or_host);
        or_host = nullptr;
        if (counts_ev) (void)hipEventDestroy(counts_ev);
        counts_ev = nullptr;
        for (DevBuf* b : {&keys, &vals, &count, &off2, &off3, &owner, &piece_sums, &piece_sums2,
                          &bucket_sums, &red_a, &red_b, &temp, &results, &piece_raw, &stat, &canon})
            b->release();
        sorted.release();
    }
};

#define EON_HIP(call)                                                                     \
    do {                                                                                  \
        hipError_t _e = (call);                                                           \
        if (_e != hipSuccess)                                                             \
            return ::eon::Status::err(_e == hipErrorOutOfMemory ? EON_E_OOM : EON_E_DEVICE, \
                                      std::string(#call ": ") + hipGetErrorString(_e));   \
    } while (0)

#define EON_TRY(expr)                  \
    do {                               \
        ::eon::Status _s = (expr);     \
        if (_s.bad()) return _s;       \
    } while (0)

}  // namespace eon

struct eon_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::string last_error;

    // stage-concatenated twiddles for sizes up to 2^tw_log (forward and inverse): the plain roots w
    // (32 B each) and their Shoup quotients floor(w 2^261 / p) (9 limbs of 29 bits in 48 B)
    eon::DevBuf tw_fwd, tw_inv, twq_fwd, twq_inv;
    uint32_t tw_log = 0;

    // coset / scaling tables keyed by (kind, log_n, base, scale)
    std::map<std::string, eon::DevBuf> tables;

    // EON_NTT_MAX_STAGES: cap on radix-2 stages per NTT pass (0 = tile limit); read at creation
    uint32_t ntt_max_stages = 0;
    // EON_NTT_TPB / EON_NTT_LOG_CB: tuning knobs (threads per block cap, columns per tile)
    uint32_t ntt_tpb = 0;
    uint32_t ntt_log_tile = 0;  // EON_NTT_TILE: log2 elements per LDS tile (0 = 10)
    int ntt_log_cb = -1;

    // per-launch HIP-event timing (eon_ctx_profile_*)
    eon::Profiler prof;

    // serial mode (EON_SERIAL=1 at creation, eon_ctx_set_serial): every launch of this context on
    // `stream`, no side streams -- kernel durations are then isolated (profiling), not overlapped
    bool serial = false;
    hipStream_t side(hipStream_t s) const { return serial ? stream : s; }

    // process group for work replicated on every rank (eon_ctx_set_collective; world 0 = none)
    eon_collective coll{0, 0, nullptr, nullptr};

    // MSM pipeline: workspaces msm / msm_b / msm_c for batches k % 3; piece sums + reductions on
    // `stream` / msm_side, digit sorts on the high-priority msm_sort (msm.hip: msm_run_columns)
    eon::MsmWork msm, msm_b, msm_c;
    hipStream_t msm_side = nullptr, msm_sort = nullptr;
    // third compute stream of the prepared path (jobs round-robin over stream / msm_side / msm_side2)
    hipStream_t msm_side2 = nullptr;
    hipEvent_t msm_ev[3] = {nullptr, nullptr, nullptr};
    hipEvent_t msm_sorted[3] = {nullptr, nullptr, nullptr}, msm_reduced[3] = {nullptr, nullptr, nullptr};

    // sorted-digit buffers of destroyed eon_msm_scalars, reused by the next prepared MSM (the
    // prover commits matrices of the same shape every proof: keeping ~22 GB resident beats a
    // hipMalloc/hipFree of it per proof); trimmed past MSM_SORTED_CACHE_CAP bytes
    std::vector<eon::SortedBufs> sorted_cache;

    // call-wide first-level segment sums of the MSM bucket reduction (msm.hip DeferredFinish)
    eon::DevBuf fin_T, fin_U;

    // four-step DFT working blocks; the sharded MSM's partials (sharded.hip)
    eon::DevBuf fs_a, fs_b, shard_send, shard_recv;

    // quotient: vanishing-polynomial table (kept while its domains repeat); KZG opening scan workspace
    eon::DevBuf sel_tab, kzg_tmp;
    bool van_valid = false;
    uint32_t van_log_n = 0, van_log_q = 0;
    eon::Fr van_shift{};
    // opening bases' tables and scratch, reused across proofs (opening.hip, msm.hip)
    eon::DevPool pool;

    // scratch: NTT intermediates, host-API staging; the DIT networks' unreduced 29-limb planes
    // between passes (NetworkSpec::mid)
    eon::DevBuf scratch, stage_in, stage_out, mid29;
};

namespace eon {

Status ensure_twiddles(eon_ctx* ctx, uint32_t log_n);
// DevBuf::ensure for the large per-call workspaces: on an out-of-memory error it first drains the
// context's streams and gives back what the context keeps only for speed -- the idle pool buffers,
// the cached sorted-digit buffers, the NTT plane buffer (what eon_ctx_trim frees) -- and tries
// once more (capi_dft.hip)
hipError_t ctx_ensure(eon_ctx* ctx, DevBuf& b, size_t need);
// table[j] = scale * base^j (natural) or table[j] = scale * base^reverse_bits(j, log_n) (bitrev)
Status get_power_table(eon_ctx* ctx, uint32_t log_n, const Fr& base, const Fr& scale, bool bitrev,
                       const Fr** out);

// forward dft_batch (natural order in and out) of a height x width device matrix on ctx->stream
Status dft_natural_dev(eon_ctx* ctx, const Fr* in, Fr* out, uint64_t height, uint32_t width);
// four-step middle step (fourstep.hip): twiddle and pack the rank's size-N1 column DFTs
Status fourstep_twiddle_pack(eon_ctx* ctx, const Fr* y, uint32_t log_n, uint32_t log_n1, uint64_t col0,
                             uint32_t cols, uint32_t parts, Fr* send);

inline Fr fr_two_adic_generator(uint32_t bits) {
    // bn254/src/field.rs:556-573: square TWO_ADIC_GENERATOR (order 2^28) 28 - bits times
    Fr w;
    const uint64_t g[4] = {0x636e735580d13d9cull, 0xa22bf3742445ffd6ull, 0x56452ac01eb203d8ull,
                           0x1860ef942963f9e7ull};
    for (int i = 0; i < 4; i++) {
        w.v[2 * i] = (uint32_t)g[i];
        w.v[2 * i + 1] = (uint32_t)(g[i] >> 32);
    }
    for (uint32_t i = bits; i < 28; i++) w = sqr(w);
    return w;
}

inline Fr fr_from_abi(const eon_fr* x) {
    Fr r;
    for (int i = 0; i < 4; i++) {
        r.v[2 * i] = (uint32_t)x->l[i];
        r.v[2 * i + 1] = (uint32_t)(x->l[i] >> 32);
    }
    return r;
}

inline bool fr_is_canonical(const Fr& x) {
    for (int i = 7; i >= 0; i--) {
        if (x.v[i] < FrP::P[i]) return true;
        if (x.v[i] > FrP::P[i]) return false;
    }
    return false;
}

}  // namespace eon
