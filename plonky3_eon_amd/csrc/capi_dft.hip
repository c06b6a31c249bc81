// C ABI: context management and the TwoAdicSubgroupDft<Fr> entry points (include/eon.h).
//
// Each entry point is planned as one or two radix-2 networks (ntt.hip) whose first pass folds
// in the input permutation and coset scaling, mirroring the reference trait defaults:
//   dft           (dft/src/traits.rs:61)       natural: DIT over bit-reversed gather; bitrev: DIF
//   idft          (dft/src/traits.rs:111-122)  DIT with inverse twiddles, 1/N folded into the load
//   coset_dft     (dft/src/traits.rs:83-91)    as dft, coefficient j scaled by shift^j on load
//   coset_idft    (dft/src/traits.rs:144-153)  as idft, output j scaled by shift^-j on store
//   coset_lde     (dft/src/traits.rs:226-249, Radix2DitParallel :169-228)
//        natural: inverse DIF (evals -> bit-reversed coefficients) then a forward DIT of size
//                 N*2^b that starts at stage b on the spread coefficients (the first b stages
//                 of a zero-padded DIT only copy), coefficient scaling shift^j / N on load.
//        bitrev:  inverse DIT (natural coefficients) then forward DIF on the zero-padded
//                 vector, which lands directly in Radix2DitParallel's bit-reversed storage.
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <vector>

#include "context.h"

#include <algorithm>
#include "ntt.h"

using namespace eon;

namespace eon {

Status ensure_twiddles(eon_ctx* ctx, uint32_t log_n) {
    if (log_n == 0 || log_n <= ctx->tw_log) return Status::ok();
    const uint32_t L = log_n < 12 ? 12 : log_n;  // build small tables once
    const size_t bytes = ((size_t)1 << L) * sizeof(Fr);
    EON_HIP(ctx->tw_fwd.ensure(bytes));
    EON_HIP(ctx->tw_inv.ensure(bytes));
    EON_HIP(ctx->twq_fwd.ensure(((size_t)1 << L) * TWQ_STRIDE * sizeof(uint32_t)));
    EON_HIP(ctx->twq_inv.ensure(((size_t)1 << L) * TWQ_STRIDE * sizeof(uint32_t)));
    const Fr root = fr_two_adic_generator(L);
    EON_HIP(launch_twiddles(ctx->tw_fwd.as<Fr>(), ctx->twq_fwd.as<uint32_t>(), L, root, ctx->stream));
    EON_HIP(launch_twiddles(ctx->tw_inv.as<Fr>(), ctx->twq_inv.as<uint32_t>(), L, inverse(root), ctx->stream));
    ctx->tw_log = L;
    return Status::ok();
}

Status get_power_table(eon_ctx* ctx, uint32_t log_n, const Fr& base, const Fr& scale, bool bitrev,
                       const Fr** out) {
    std::string key(1, bitrev ? 'r' : 'n');
    key.push_back((char)log_n);
    key.append(reinterpret_cast<const char*>(base.v), 32);
    key.append(reinterpret_cast<const char*>(scale.v), 32);
    auto it = ctx->tables.find(key);
    if (it == ctx->tables.end()) {
        if (ctx->tables.size() >= 64) {
            // bounded cache: drop everything (tables are cheap to rebuild)
            EON_HIP(hipStreamSynchronize(ctx->stream));
            for (auto& kv : ctx->tables) kv.second.release();
            ctx->tables.clear();
        }
        DevBuf buf;
        const uint64_t n = 1ull << log_n;
        EON_HIP(buf.ensure(n * sizeof(Fr)));
        hipError_t e = launch_powers(buf.as<Fr>(), n, base, scale, bitrev ? log_n : NATURAL_IDX,
                                     ctx->stream);
        if (e != hipSuccess) {
            buf.release();
            EON_HIP(e);
        }
        it = ctx->tables.emplace(key, buf).first;
    }
    *out = it->second.as<Fr>();
    return Status::ok();
}

}  // namespace eon

namespace {

enum class Op { Dft, Idft, CosetDft, CosetIdft, CosetLde, CosetDftPadded };

int finish(eon_ctx* ctx, const Status& s) {
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

Status check_shape(uint64_t height, uint32_t added_bits, uint32_t* log_h) {
    if (height == 0 || (height & (height - 1)) != 0)
        return Status::err(EON_E_SHAPE, "height must be a power of two (log2_strict_usize)");
    const uint32_t lg = 63 - __builtin_clzll(height);
    if (lg + (uint64_t)added_bits > 28)
        return Status::err(EON_E_SHAPE, "log2(height) + added_bits exceeds Fr::TWO_ADICITY = 28");
    *log_h = lg;
    return Status::ok();
}

Status dft_dev(eon_ctx* ctx, Op op, const Fr* in, Fr* out, uint64_t height, uint32_t width,
               uint32_t added_bits, const eon_fr* shift_abi, int out_order) {
    uint32_t n = 0;
    const bool grows = op == Op::CosetLde || op == Op::CosetDftPadded;
    EON_TRY(check_shape(height, grows ? added_bits : 0, &n));
    if (out_order != EON_ORDER_NATURAL && out_order != EON_ORDER_BITREV)
        return Status::err(EON_E_ARG, "out_order must be EON_ORDER_NATURAL or EON_ORDER_BITREV");
    if (width == 0) return Status::ok();
    if (!in || !out) return Status::err(EON_E_ARG, "null matrix pointer");
    Fr shift = Fr::one();
    if (shift_abi) {
        shift = fr_from_abi(shift_abi);
        if (!fr_is_canonical(shift)) return Status::err(EON_E_ARG, "shift is not a canonical Fr");
    }
    const bool natural = out_order == EON_ORDER_NATURAL;
    const uint32_t b = grows ? added_bits : 0;
    EON_TRY(ensure_twiddles(ctx, n + b));
    const size_t mat_bytes = (size_t)height * width * sizeof(Fr);
    hipStream_t st = ctx->stream;

    const Fr n_inv = inverse(from_u64<FrP>(height));

#ifndef EON_LDE_DIT
#define EON_LDE_DIT 1
#endif
// the DIT networks exchange unreduced 29-limb planes between passes (EON_NTT_MID, ntt.hip PassArgs::mid)
#ifndef EON_NTT_MID
#define EON_NTT_MID 1
#endif
    // the plane buffer of a DIT network, allocated only when the network runs more than one pass
    // (a one-pass network exchanges nothing); it grows with the largest multi-pass transform and
    // is given back by eon_ctx_trim, and by ctx_ensure when another allocation runs out of memory
    auto mid_for = [&](std::initializer_list<NetworkSpec*> specs) {
        uint64_t need = 0;
        for (NetworkSpec* sp : specs)
            if (!sp->dif && network_passes(*sp) > 1) need = std::max<uint64_t>(need, (1ull << sp->log_m) * sp->width * 36);
        if (!EON_NTT_MID || need == 0) return;
        if (ctx_ensure(ctx, ctx->mid29, need) != hipSuccess) {
            (void)hipGetLastError();
            return;  // the packed exchange through `dst` instead
        }
        for (NetworkSpec* sp : specs)
            if (!sp->dif && network_passes(*sp) > 1) sp->mid = ctx->mid29.as<uint4>();
    };
    if (op == Op::CosetLde) {
        EON_HIP(ctx->scratch.ensure(mat_bytes));
        Fr* coeffs = ctx->scratch.as<Fr>();
        NetworkSpec a;  // evals -> coefficients (times N), into scratch
        a.log_m = n;
        a.src = in;
        a.dst = coeffs;
        a.width = width;
        a.tw = ctx->tw_inv.as<Fr>();
        a.twq = ctx->twq_inv.as<uint32_t>();
        NetworkSpec f;  // coefficients -> evaluations on shift * K
        f.log_m = n + b;
        f.src = coeffs;
        f.dst = out;
        f.width = width;
        f.tw = ctx->tw_fwd.as<Fr>();
        f.twq = ctx->twq_fwd.as<uint32_t>();
        const Fr* table = nullptr;
        bool want_mid = false;
        if (natural && EON_LDE_DIT) {
            // two DIT networks: bit-reversed gather -> natural coefficients, then the forward
            // network gathers them bit-reversed and spread.  The DIT butterfly (lazy sums, carries
            // every third stage) costs ~18 % less than the DIF one (profiles/r05/s14: 0.35 ms per
            // inverse DIF stage of 2^19 x 64 butterflies against 0.56 per forward DIT stage of twice
            // as many)
            a.dif = false;
            a.load_mode = LOAD_BITREV;
            a.load_param = n;
            EON_TRY(get_power_table(ctx, n, shift, ntt_scale_form(n_inv), false, &table));
            f.dif = false;
            f.first_stage = b;
            f.load_mode = LOAD_BITREV_SPREAD;
            f.load_param = b | (n << 8);
            // one plane buffer serves both networks (they run one after the other on `st`)
            want_mid = true;
        } else if (natural) {
            a.dif = true;  // natural evals -> bit-reversed coefficients
            EON_TRY(get_power_table(ctx, n, shift, ntt_scale_form(n_inv), true, &table));
            f.dif = false;
            f.first_stage = b;
            f.load_mode = LOAD_SPREAD;
            f.load_param = b;
        } else {
            a.dif = false;  // bit-reversed gather -> natural coefficients
            a.load_mode = LOAD_BITREV;
            a.load_param = n;
            EON_TRY(get_power_table(ctx, n, shift, ntt_scale_form(n_inv), false, &table));
            f.dif = true;
            f.load_mode = LOAD_ZEROPAD;
            f.load_param = (uint32_t)height;
        }
        // coefficient j times shift^j / N, applied as the inverse network stores coefficient j
        // (its output row; the table is in that row order): once per coefficient, where the
        // forward network's loads would read each coefficient 2^b times
        a.store_scale = table;
        a.max_stages_per_pass = f.max_stages_per_pass = ctx->ntt_max_stages;
        a.max_threads = f.max_threads = ctx->ntt_tpb;
        a.log_tile = f.log_tile = ctx->ntt_log_tile;
        a.log_cb_override = f.log_cb_override = ctx->ntt_log_cb;
        if (want_mid) mid_for({&a, &f});
        EON_HIP(run_network(a, st, &ctx->prof));
        EON_HIP(run_network(f, st, &ctx->prof));
        return Status::ok();
    }

    if (op == Op::CosetDftPadded) {
        // coset_dft of the coefficients zero-padded to height * 2^b: coset_lde_batch without its
        // idft (dft/src/traits.rs:226-249), i.e. KzgPcs::get_evaluations_on_domain from the
        // committed coefficients (kzg/src/pcs.rs:267-287; commit/src/testing.rs:93-105)
        if (in == out) return Status::err(EON_E_ARG, "padded coset DFT cannot run in place");
        const Fr* table = nullptr;
        EON_TRY(get_power_table(ctx, n, shift, ntt_scale_form(Fr::one()), false, &table));
        NetworkSpec f;
        f.log_m = n + b;
        f.src = in;
        f.dst = out;
        f.width = width;
        f.tw = ctx->tw_fwd.as<Fr>();
        f.twq = ctx->twq_fwd.as<uint32_t>();
        f.load_scale = table;  // coefficient j times shift^j, indexed by source row
        if (natural) {
            f.dif = false;
            f.first_stage = b;
            f.load_mode = LOAD_BITREV_SPREAD;
            f.load_param = b | (n << 8);
        } else {
            f.dif = true;
            f.load_mode = LOAD_ZEROPAD;
            f.load_param = (uint32_t)height;
        }
        f.max_stages_per_pass = ctx->ntt_max_stages;
        f.max_threads = ctx->ntt_tpb;
        f.log_tile = ctx->ntt_log_tile;
        f.log_cb_override = ctx->ntt_log_cb;
        if (natural) mid_for({&f});
        EON_HIP(run_network(f, st, &ctx->prof));
        return Status::ok();
    }

    NetworkSpec s;
    s.log_m = n;
    s.src = in;
    s.dst = out;
    s.width = width;
    const bool inv = op == Op::Idft || op == Op::CosetIdft;
    s.tw = inv ? ctx->tw_inv.as<Fr>() : ctx->tw_fwd.as<Fr>();
    s.twq = inv ? ctx->twq_inv.as<uint32_t>() : ctx->twq_fwd.as<uint32_t>();
    // idft / coset_idft always return natural-order coefficients (RowMajorMatrix)
    s.dif = !(inv || natural);
    if (!s.dif) {
        s.load_mode = LOAD_BITREV;
        s.load_param = n;
        if (in == out && n > 0) {  // the gather cannot run in place
            EON_HIP(ctx->scratch.ensure(mat_bytes));
            EON_HIP(hipMemcpyAsync(ctx->scratch.p, in, mat_bytes, hipMemcpyDeviceToDevice, st));
            s.src = ctx->scratch.as<Fr>();
        }
    }
    if (op == Op::CosetDft) {
        const Fr* table = nullptr;
        EON_TRY(get_power_table(ctx, n, shift, ntt_scale_form(Fr::one()), false, &table));
        s.load_scale = table;
    }
    if (inv) {
        s.has_load_const = 1;
        s.load_const = ntt_scale_form(n_inv);
    }
    // coset_idft with shift 1 (KzgPcs::commit of the trace, kzg/src/pcs.rs:242) is the idft: no
    // output scaling by the all-ones powers of 1^-1
    if (op == Op::CosetIdft && !(shift == Fr::one())) {
        const Fr* table = nullptr;
        EON_TRY(get_power_table(ctx, n, inverse(shift), ntt_scale_form(Fr::one()), false, &table));
        s.store_scale = table;
    }
    s.max_stages_per_pass = ctx->ntt_max_stages;
    s.max_threads = ctx->ntt_tpb;
    s.log_tile = ctx->ntt_log_tile;
    s.log_cb_override = ctx->ntt_log_cb;
    if (!s.dif) mid_for({&s});
    EON_HIP(run_network(s, st, &ctx->prof));
    return Status::ok();
}

// Host-pointer wrapper: stage in, run, stage out, synchronize.
Status dft_host(eon_ctx* ctx, Op op, const eon_fr* in, eon_fr* out, uint64_t height,
                uint32_t width, uint32_t added_bits, const eon_fr* shift, int out_order) {
    uint32_t n = 0;
    const bool grows = op == Op::CosetLde || op == Op::CosetDftPadded;
    EON_TRY(check_shape(height, grows ? added_bits : 0, &n));
    if (width == 0) return Status::ok();
    if (!in || !out) return Status::err(EON_E_ARG, "null matrix pointer");
    const size_t in_bytes = (size_t)height * width * sizeof(Fr);
    const size_t out_bytes = in_bytes << (grows ? added_bits : 0);
    EON_HIP(ctx->stage_in.ensure(in_bytes));
    EON_HIP(ctx->stage_out.ensure(out_bytes));
    EON_HIP(hipMemcpyAsync(ctx->stage_in.p, in, in_bytes, hipMemcpyHostToDevice, ctx->stream));
    EON_TRY(dft_dev(ctx, op, ctx->stage_in.as<Fr>(), ctx->stage_out.as<Fr>(), height, width,
                    added_bits, shift, out_order));
    EON_HIP(hipMemcpyAsync(out, ctx->stage_out.p, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    EON_HIP(hipStreamSynchronize(ctx->stream));
    return Status::ok();
}

int entry(eon_ctx* ctx, bool dev, Op op, const eon_fr* in, eon_fr* out, uint64_t height,
          uint32_t width, uint32_t added_bits, const eon_fr* shift, int out_order) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess)
        return finish(ctx, Status::err(EON_E_DEVICE, "hipSetDevice failed"));
    Status s = dev ? dft_dev(ctx, op, reinterpret_cast<const Fr*>(in), reinterpret_cast<Fr*>(out),
                             height, width, added_bits, shift, out_order)
                   : dft_host(ctx, op, in, out, height, width, added_bits, shift, out_order);
    return finish(ctx, s);
}

}  // namespace

namespace eon {

Status dft_natural_dev(eon_ctx* ctx, const Fr* in, Fr* out, uint64_t height, uint32_t width) {
    return dft_dev(ctx, Op::Dft, in, out, height, width, 0, nullptr, EON_ORDER_NATURAL);
}

}  // namespace eon

namespace eon {
hipError_t ctx_ensure(eon_ctx* ctx, DevBuf& b, size_t need) {
    hipError_t e = b.ensure(need);
    if (e != hipErrorOutOfMemory) return e;
    (void)hipGetLastError();
    // the buffers below may still be read by queued work: drain the context's streams first
    for (hipStream_t st : {ctx->stream, ctx->msm_side, ctx->msm_side2, ctx->msm_sort})
        if (st && (e = hipStreamSynchronize(st)) != hipSuccess) return e;
    ctx->pool.release_all();
    for (auto& sb : ctx->sorted_cache) sb.release();
    ctx->sorted_cache.clear();
    if (&b != &ctx->mid29) ctx->mid29.release();
    return b.ensure(need);
}
}  // namespace eon

extern "C" {

uint32_t eon_abi_version(void) { return 4; }

int eon_ctx_create(int device_ordinal, eon_ctx** out) {
    if (!out) return EON_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device_ordinal < 0 || device_ordinal >= n)
        return EON_E_DEVICE;
    if (hipSetDevice(device_ordinal) != hipSuccess) return EON_E_DEVICE;
    eon_ctx* c = new eon_ctx();
    c->device = device_ordinal;
    // blocking stream: host-API work stays ordered with null-stream work of other libraries
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamDefault) != hipSuccess) {
        delete c;
        return EON_E_DEVICE;
    }
    c->stream = c->own_stream;
    // MSM streams: non-blocking so that they overlap null-stream work (ordered by events); the
    // sort stream at the highest priority
    int prio_least = 0, prio_greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    bool ok = hipStreamCreateWithFlags(&c->msm_side, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&c->msm_side2, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipStreamCreateWithPriority(&c->msm_sort, hipStreamNonBlocking, prio_greatest) == hipSuccess;
    for (hipEvent_t* e : {&c->msm_ev[0], &c->msm_ev[1], &c->msm_ev[2], &c->msm_sorted[0], &c->msm_sorted[1],
                          &c->msm_sorted[2], &c->msm_reduced[0], &c->msm_reduced[1], &c->msm_reduced[2]})
        ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return EON_E_DEVICE;
    }
    if (const char* e = getenv("EON_SERIAL")) c->serial = e[0] == '1';
    if (const char* e = getenv("EON_POOL_CAP_GB")) c->pool.cap = (size_t)std::max(0, atoi(e)) << 30;
    if (const char* e = getenv("EON_NTT_MAX_STAGES")) c->ntt_max_stages = (uint32_t)atoi(e);
#ifdef EON_TUNING_KNOBS
    // NTT plan overrides for tuning builds only (_build.build_variant(..., ["EON_TUNING_KNOBS"]))
    if (const char* e = getenv("EON_NTT_TPB")) c->ntt_tpb = (uint32_t)atoi(e);
    if (const char* e = getenv("EON_NTT_TILE")) c->ntt_log_tile = (uint32_t)atoi(e);
    if (const char* e = getenv("EON_NTT_LOG_CB")) c->ntt_log_cb = atoi(e) > 3 ? 3 : atoi(e);
#endif
    *out = c;
    return EON_OK;
}

void eon_ctx_destroy(eon_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamSynchronize(ctx->msm_side);
    (void)hipStreamSynchronize(ctx->msm_side2);
    (void)hipStreamSynchronize(ctx->msm_sort);
    ctx->tw_fwd.release();
    ctx->tw_inv.release();
    ctx->twq_fwd.release();
    ctx->twq_inv.release();
    for (auto& kv : ctx->tables) kv.second.release();
    for (auto& r : ctx->prof.recs) {
        (void)hipEventDestroy(r.start);
        (void)hipEventDestroy(r.stop);
    }
    for (auto e : ctx->prof.pool) (void)hipEventDestroy(e);
    ctx->msm.release();
    ctx->msm_b.release();
    ctx->msm_c.release();
    for (auto& sb : ctx->sorted_cache) sb.release();
    ctx->sorted_cache.clear();
    ctx->sel_tab.release();
    ctx->kzg_tmp.release();
    ctx->fin_T.release();
    ctx->fin_U.release();
    ctx->fs_a.release();
    ctx->fs_b.release();
    ctx->shard_send.release();
    ctx->shard_recv.release();
    ctx->pool.release_all();
    ctx->scratch.release();
    ctx->stage_in.release();
    ctx->stage_out.release();
    ctx->mid29.release();
    (void)hipStreamDestroy(ctx->own_stream);
    (void)hipStreamDestroy(ctx->msm_side);
    (void)hipStreamDestroy(ctx->msm_side2);
    (void)hipStreamDestroy(ctx->msm_sort);
    for (hipEvent_t e : {ctx->msm_ev[0], ctx->msm_ev[1], ctx->msm_ev[2], ctx->msm_sorted[0], ctx->msm_sorted[1],
                         ctx->msm_sorted[2], ctx->msm_reduced[0], ctx->msm_reduced[1], ctx->msm_reduced[2]})
        (void)hipEventDestroy(e);
    delete ctx;
}

const char* eon_last_error(const eon_ctx* ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

int eon_ctx_set_stream(eon_ctx* ctx, void* hip_stream) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    // used verbatim: NULL is the HIP null (legacy default) stream, which is torch's default
    ctx->stream = reinterpret_cast<hipStream_t>(hip_stream);
    return EON_OK;
}

int eon_ctx_device(const eon_ctx* ctx) { return ctx ? ctx->device : -1; }

int eon_ctx_set_serial(eon_ctx* ctx, int serial) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    (void)hipSetDevice(ctx->device);
    // drain the side streams before their work moves to `stream` (or back)
    for (hipStream_t st : {ctx->stream, ctx->msm_side, ctx->msm_side2, ctx->msm_sort})
        (void)hipStreamSynchronize(st);
    ctx->serial = serial != 0;
    return EON_OK;
}

int eon_ctx_serial(const eon_ctx* ctx) { return ctx && ctx->serial ? 1 : 0; }

int eon_ctx_set_collective(eon_ctx* ctx, const eon_collective* coll) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!coll || coll->world <= 1) {
        ctx->coll = eon_collective{0, 0, nullptr, nullptr};
        return EON_OK;
    }
    if (!coll->all_gather || coll->rank >= coll->world) return EON_E_ARG;
    ctx->coll = *coll;
    return EON_OK;
}

void* eon_ctx_stream(eon_ctx* ctx) {
    if (!ctx) return nullptr;
    std::lock_guard<std::mutex> lk(ctx->mu);
    return reinterpret_cast<void*>(ctx->stream);
}

int eon_ctx_synchronize(eon_ctx* ctx) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    (void)hipSetDevice(ctx->device);
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        ctx->last_error = hipGetErrorString(e);
        return EON_E_DEVICE;
    }
    return EON_OK;
}

int eon_ctx_trim(eon_ctx* ctx) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    (void)hipSetDevice(ctx->device);
    for (hipStream_t st : {ctx->stream, ctx->msm_side, ctx->msm_side2, ctx->msm_sort}) {
        hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            ctx->last_error = hipGetErrorString(e);
            return EON_E_DEVICE;
        }
    }
    ctx->pool.release_all();
    for (auto& sb : ctx->sorted_cache) sb.release();
    ctx->sorted_cache.clear();
    ctx->mid29.release();
    return EON_OK;
}

int eon_ctx_profile(eon_ctx* ctx, int enable) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& r : ctx->prof.recs) {
        ctx->prof.pool.push_back(r.start);
        ctx->prof.pool.push_back(r.stop);
    }
    ctx->prof.recs.clear();
    ctx->prof.enabled = enable != 0;
    return EON_OK;
}

int eon_ctx_profile_report(eon_ctx* ctx, char* buf, uint64_t len) {
    // JSON: {"kernel name": {"launches": n, "total_ms": t, "busy_ms": u, "alg_bytes": b,
    //        "alg_mulmods": m, "design_bytes": d}, ...}
    if (!ctx || !buf || len == 0) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    (void)hipSetDevice(ctx->device);
    // busy_ms: the union of a kernel's launch intervals (launches on several streams overlap, so
    // total_ms / launches overstates what one launch would take alone)
    struct Agg {
        uint64_t n = 0, bytes = 0, mulmods = 0, design = 0;
        double ms = 0;
        std::vector<std::pair<double, double>> iv;
    };
    std::map<std::string, Agg> agg;
    hipEvent_t t0 = ctx->prof.recs.empty() ? nullptr : ctx->prof.recs.front().start;
    for (auto& r : ctx->prof.recs) {
        if (hipEventSynchronize(r.stop) != hipSuccess) continue;
        float ms = 0, a0 = 0, a1 = 0;
        if (hipEventElapsedTime(&ms, r.start, r.stop) != hipSuccess) continue;
        Agg& a = agg[r.kernel];
        a.n++;
        a.ms += ms;
        a.bytes += r.alg_bytes;
        a.mulmods += r.alg_mulmods;
        a.design += r.design_bytes;
        if (hipEventElapsedTime(&a0, t0, r.start) == hipSuccess && hipEventElapsedTime(&a1, t0, r.stop) == hipSuccess)
            a.iv.emplace_back(a0, a1);
    }
    auto busy = [](std::vector<std::pair<double, double>> iv) {
        std::sort(iv.begin(), iv.end());
        double tot = 0, s = 0, e = -1e300;
        for (auto& x : iv) {
            if (x.first > e) {
                if (e > s) tot += e - s;
                s = x.first;
                e = x.second;
            } else if (x.second > e) {
                e = x.second;
            }
        }
        if (e > s) tot += e - s;
        return tot;
    };
    std::string out = "{";
    char tmp[384];
    for (auto& kv : agg) {
        snprintf(tmp, sizeof tmp,
                 "%s\"%s\": {\"launches\": %llu, \"total_ms\": %.6f, \"busy_ms\": %.6f, "
                 "\"alg_bytes\": %llu, \"alg_mulmods\": %llu, \"design_bytes\": %llu}",
                 out.size() > 1 ? ", " : "", kv.first.c_str(), (unsigned long long)kv.second.n,
                 kv.second.ms, busy(kv.second.iv), (unsigned long long)kv.second.bytes,
                 (unsigned long long)kv.second.mulmods, (unsigned long long)kv.second.design);
        out += tmp;
    }
    out += "}";
    if (out.size() + 1 > len) return EON_E_ARG;
    memcpy(buf, out.c_str(), out.size() + 1);
    return EON_OK;
}

int eon_dft_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height, uint32_t width,
                  int out_order) {
    return entry(ctx, false, Op::Dft, in, out, height, width, 0, nullptr, out_order);
}
int eon_idft_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height, uint32_t width) {
    return entry(ctx, false, Op::Idft, in, out, height, width, 0, nullptr, EON_ORDER_NATURAL);
}
int eon_coset_dft_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                        uint32_t width, const eon_fr* shift, int out_order) {
    if (!shift) return EON_E_ARG;
    return entry(ctx, false, Op::CosetDft, in, out, height, width, 0, shift, out_order);
}
int eon_coset_idft_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                         uint32_t width, const eon_fr* shift) {
    if (!shift) return EON_E_ARG;
    return entry(ctx, false, Op::CosetIdft, in, out, height, width, 0, shift, EON_ORDER_NATURAL);
}
int eon_coset_lde_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                        uint32_t width, uint32_t added_bits, const eon_fr* shift, int out_order) {
    return entry(ctx, false, Op::CosetLde, in, out, height, width, added_bits, shift, out_order);
}

int eon_coset_dft_padded_batch(eon_ctx* ctx, const eon_fr* coeffs, eon_fr* out, uint64_t height,
                               uint32_t width, uint32_t added_bits, const eon_fr* shift,
                               int out_order) {
    if (!shift) return EON_E_ARG;
    return entry(ctx, false, Op::CosetDftPadded, coeffs, out, height, width, added_bits, shift, out_order);
}
int eon_coset_dft_padded_batch_dev(eon_ctx* ctx, const eon_fr* coeffs, eon_fr* out, uint64_t height,
                                   uint32_t width, uint32_t added_bits, const eon_fr* shift,
                                   int out_order) {
    if (!shift) return EON_E_ARG;
    return entry(ctx, true, Op::CosetDftPadded, coeffs, out, height, width, added_bits, shift, out_order);
}

int eon_dft_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                      uint32_t width, int out_order) {
    return entry(ctx, true, Op::Dft, in, out, height, width, 0, nullptr, out_order);
}
int eon_idft_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                       uint32_t width) {
    return entry(ctx, true, Op::Idft, in, out, height, width, 0, nullptr, EON_ORDER_NATURAL);
}
int eon_coset_dft_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                            uint32_t width, const eon_fr* shift, int out_order) {
    if (!shift) return EON_E_ARG;
    return entry(ctx, true, Op::CosetDft, in, out, height, width, 0, shift, out_order);
}
int eon_coset_idft_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                             uint32_t width, const eon_fr* shift) {
    if (!shift) return EON_E_ARG;
    return entry(ctx, true, Op::CosetIdft, in, out, height, width, 0, shift, EON_ORDER_NATURAL);
}
int eon_coset_lde_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                            uint32_t width, uint32_t added_bits, const eon_fr* shift,
                            int out_order) {
    return entry(ctx, true, Op::CosetLde, in, out, height, width, added_bits, shift, out_order);
}

}  // extern "C"
