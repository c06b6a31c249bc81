// See prover.h.  Stage order and span names follow prove_with_preprocessed
// (eon-uni-stark/src/prover.rs): commit (186-187) -> quotient domain (307-308) -> LDE (315) ->
// quotient_values (328-342) -> commit_quotient (371-372) -> open at [zeta, zeta h] and [zeta] per
// chunk (416-442).
//
// Lane sharding: the vectorized AIR evaluates its lanes one after another
// (poseidon2-air/src/vectorized.rs:259-274), so lane v owns columns [164 v, 164 v + 164) and
// constraints [K v, K v + K), K = 160.  A rank proving lanes [l0, l1) commits, extends and opens
// its own columns, and its folder accumulator times alpha^(K (VL - l1)) is its exact share of the
// full one (folder.rs:81-85).  The partials are all-gathered (Q x 32 B, the one data-path
// exchange) and combined on device; the per-column results are all-gathered at the end.
#include "prover.h"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>

namespace eon_host {

uint32_t log_quotient_degree(uint32_t max_constraint_degree) {
    const uint32_t d = (max_constraint_degree > 2 ? max_constraint_degree : 2) - 1;
    uint32_t b = 0;
    while ((1u << b) < d) b++;
    return b;
}

namespace {

// per-column record of the final all-gather: commitment (8) | value at zeta (4) | value at zeta h
// (4) | witness at zeta (8) | witness at zeta h (8), in u64
constexpr uint32_t RECORD = 32;

void all_gather(eon_ctx* ctx, const eon_collective* coll, const void* send, void* recv, uint64_t bytes) {
    const int rc = coll->all_gather(coll->user, send, recv, bytes, eon_ctx_stream(ctx));
    if (rc != 0) throw Error(EON_E_DEVICE, "collective all_gather failed (" + std::to_string(rc) + ")");
}

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Error(EON_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

uint32_t AirRef::width() const {
    if (p2) return eon_p2air_width(p2);
    eon_air_program_stats st{};
    if (prog && eon_air_program_info(prog, &st) == EON_OK) return st.width;
    return 0;
}

Proof prove(KzgPcs& pcs, const AirRef& air, const eon_fr* trace, uint64_t height, const Fr& alpha_in,
            const Fr& zeta_in, uint32_t max_constraint_degree, const eon_collective* shard,
            DuplexChallenger* challenger) {
    eon_ctx* ctx = pcs.ctx();
    using clock = std::chrono::steady_clock;
    auto tick = [&] {
        check(ctx, eon_ctx_synchronize(ctx), "eon_ctx_synchronize");
        return clock::now();
    };
    auto ms = [](clock::time_point a, clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    if (height == 0 || (height & (height - 1))) throw Error(EON_E_SHAPE, "trace height must be a power of two");
    if ((air.p2 == nullptr) == (air.prog == nullptr)) throw Error(EON_E_ARG, "exactly one of p2air / program");
    if (air.n_public && !air.publics) throw Error(EON_E_ARG, "null public values");
    if (air.p2 && air.n_public) throw Error(EON_E_SHAPE, "the Poseidon2-AIR has no public values");
    const uint32_t width = air.width();
    const uint32_t local_vl = air.p2 ? eon_p2air_vector_len(air.p2) : 1;
    const uint32_t k_lane = air.p2 ? eon_p2air_constraints_per_perm(air.p2) : 0;
    if (shard && shard->world <= 1) shard = nullptr;
    if (shard && (!shard->all_gather || shard->rank >= shard->world))
        throw Error(EON_E_ARG, "invalid collective");
    if (shard && !air.p2) throw Error(EON_E_ARG, "lane sharding needs the (vectorized) Poseidon2-AIR");
    const uint32_t world = shard ? shard->world : 1, rank = shard ? shard->rank : 0;
    const uint32_t vector_len = local_vl * world;
    const uint32_t log_n = 63 - __builtin_clzll(height);
    // get_log_quotient_degree (prover.rs:150-157): the program's own constraint degrees
    const uint32_t log_qd =
        air.prog ? eon_air_program_log_quotient_degree(air.prog, 0) : log_quotient_degree(max_constraint_degree);
    const uint32_t num_chunks = 1u << log_qd;
    hipStream_t st = static_cast<hipStream_t>(eon_ctx_stream(ctx));

    Proof proof;
    proof.degree_bits = log_n;
    const Domain trace_domain = pcs.natural_domain_for_degree(height);

    auto t0 = tick();
    std::vector<std::vector<eon_g1_affine>> trace_commit;
    std::vector<MatrixProverData> trace_data;
    const Domain quotient_domain = trace_domain.create_disjoint_domain(1ull << (log_n + log_qd));
    const uint64_t q_rows = quotient_domain.size();
    DeviceMatrix lde;
    clock::time_point t1, t2;
    {
        std::vector<std::pair<Domain, DeviceMatrix>> ev;
        ev.emplace_back(trace_domain, DeviceMatrix::borrow(trace, height, width));
        pcs.commit_coeffs(std::move(ev), trace_data);
    }
    pcs.commit_columns(trace_data, 0, trace_commit);
    t1 = tick();
    // Fiat-Shamir up to alpha (prover.rs:196-208, 300) on a host thread while the device extends
    // the trace: sharded, every rank observes the full commitment (all-gathered in rank = lane
    // order first)
    Fr alpha = alpha_in;
    std::thread fs_thread;
    std::vector<eon_g1_affine> full_commit;
    if (challenger) {
        if (shard) {
            const uint64_t bytes = (uint64_t)width * sizeof(eon_g1_affine);
            DeviceBuffer send(bytes), recv(bytes * world);
            hip_ok(hipMemcpyAsync(send.get(), trace_commit[0].data(), bytes, hipMemcpyHostToDevice, st), "commit");
            all_gather(ctx, shard, send.get(), recv.get(), bytes);
            full_commit.resize((uint64_t)width * world);
            hip_ok(hipMemcpyAsync(full_commit.data(), recv.get(), bytes * world, hipMemcpyDeviceToHost, st), "commit");
            hip_ok(hipStreamSynchronize(st), "commit");
        } else {
            full_commit = trace_commit[0];
        }
        fs_thread = std::thread([&] {
            challenger->observe(fr_from_u64(log_n));  // log_ext_degree (ZK off)
            challenger->observe(fr_from_u64(log_n));  // log_degree
            challenger->observe(fr_from_u64(0));      // preprocessed width
            challenger->observe_g1(full_commit.data(), full_commit.size());
            for (uint32_t i = 0; i < air.n_public; i++)  // observe_slice(public_values), prover.rs:208
                challenger->observe(Fr::from_abi(air.publics[i]));
            alpha = challenger->sample();  // no lookups
        });
    }
    // the trace LDE (prover.rs:315) while the host thread runs the transcript up to alpha
    try {
        lde = pcs.get_evaluations_on_domain(trace_data, 0, quotient_domain);
    } catch (...) {
        if (fs_thread.joinable()) fs_thread.join();
        throw;
    }
    if (fs_thread.joinable()) fs_thread.join();
    DeviceMatrix qv = DeviceMatrix::alloc(q_rows, 1);
    {
        t2 = tick();
        const eon_fr a = alpha.abi();
        if (air.p2)
            check(ctx, eon_p2air_quotient_values_dev(ctx, air.p2, lde.data(), log_n, log_qd, &a, qv.mutable_data()),
                  "quotient_values");
        else
            check(ctx,
                  eon_quotient_values_dev(ctx, air.prog, lde.data(), log_n, log_qd, &a, air.publics, air.n_public,
                                          qv.mutable_data()),
                  "quotient_values");
    }
    check(ctx, eon_ctx_synchronize(ctx), "quotient_values");
    lde = DeviceMatrix();  // back to the buffer cache before the opening
    auto t3 = tick();
    if (shard) {
        DeviceBuffer parts(sizeof(eon_fr) * q_rows * world);
        all_gather(ctx, shard, qv.data(), parts.get(), sizeof(eon_fr) * q_rows);
        std::vector<eon_fr> w(world);
        for (uint32_t g = 0; g < world; g++)
            w[g] = fr_pow(alpha, (uint64_t)k_lane * (vector_len - (g + 1) * local_vl)).abi();
        check(ctx, eon_fr_lincomb_dev(ctx, parts.as<eon_fr>(), world, q_rows, w.data(), qv.mutable_data()),
              "combine partial quotients");
        (void)tick();
    }
    auto t3x = tick();
    // commit_quotient (prover.rs:371-372).  Sharded, chunk c is committed and opened by rank
    // c % world alone (commit/src/pcs.rs:82-101 commits the chunks independently) and the chunk
    // commitments are all-gathered before zeta; unsharded, every chunk here.
    std::vector<uint32_t> my_chunks;
    for (uint32_t c = rank; c < num_chunks; c += world) my_chunks.push_back(c);
    const uint32_t chunk_slots = (num_chunks + world - 1) / world;  // per rank, padded
    std::vector<std::vector<eon_g1_affine>> quotient_commit;
    std::vector<MatrixProverData> quotient_data;
    pcs.commit_quotient(quotient_domain, qv, num_chunks, quotient_commit, quotient_data, &my_chunks);
    std::vector<eon_g1_affine> chunk_commit(num_chunks);
    if (shard) {
        std::vector<eon_g1_affine> mine(chunk_slots, eon_g1_affine{});
        for (size_t i = 0; i < my_chunks.size(); i++) mine[i] = quotient_commit[i][0];
        const uint64_t bytes = chunk_slots * sizeof(eon_g1_affine);
        DeviceBuffer send(bytes), recv(bytes * world);
        hip_ok(hipMemcpyAsync(send.get(), mine.data(), bytes, hipMemcpyHostToDevice, st), "quotient commit");
        all_gather(ctx, shard, send.get(), recv.get(), bytes);
        std::vector<eon_g1_affine> all((uint64_t)chunk_slots * world);
        hip_ok(hipMemcpyAsync(all.data(), recv.get(), bytes * world, hipMemcpyDeviceToHost, st), "quotient commit");
        hip_ok(hipStreamSynchronize(st), "quotient commit");
        for (uint32_t c = 0; c < num_chunks; c++) chunk_commit[c] = all[(uint64_t)(c % world) * chunk_slots + c / world];
    } else {
        for (uint32_t c = 0; c < num_chunks; c++) chunk_commit[c] = quotient_commit[c][0];
    }
    Fr zeta = zeta_in;
    if (challenger) {
        for (const auto& q : chunk_commit) challenger->observe_g1(&q, 1);  // :373
        zeta = challenger->sample();                                        // :416
    }
    proof.alpha = alpha;
    proof.zeta = zeta;
    auto t4 = tick();
    const Fr zeta_next = trace_domain.next_point(zeta);  // prover.rs:416-419
    std::vector<OpenRound> rounds(2);
    rounds[0].data = &trace_data;
    rounds[0].points = {{zeta, zeta_next}};
    rounds[1].data = &quotient_data;
    rounds[1].points.assign(quotient_data.size(), std::vector<Fr>{zeta});
    // the opening bases are the same on every rank: sharded over the process group
    // (eon_ctx_set_collective)
    struct CollectiveScope {
        eon_ctx* c;
        CollectiveScope(eon_ctx* c_, const eon_collective* s) : c(c_) {
            if (s) check(c, eon_ctx_set_collective(c, s), "eon_ctx_set_collective");
        }
        ~CollectiveScope() { (void)eon_ctx_set_collective(c, nullptr); }
    };
    std::vector<Opened> opened;
    {
        CollectiveScope scope(ctx, shard);
        opened = pcs.open(rounds);  // prover.rs:424-442
    }
    auto t5 = tick();

    proof.quotient_commit = chunk_commit;
    proof.quotient_opened.resize(num_chunks);
    proof.quotient_witnesses.resize(num_chunks);
    if (!shard) {
        for (uint32_t c = 0; c < num_chunks; c++) {
            proof.quotient_opened[c] = opened[1].values[c][0][0];
            proof.quotient_witnesses[c] = opened[1].witnesses[c][0][0];
        }
    } else {
        // every rank's chunk openings to every rank: value (4 u64) | witness (8 u64) per slot
        constexpr uint32_t QREC = 12;
        std::vector<uint64_t> rec((uint64_t)chunk_slots * QREC, 0);
        for (size_t i = 0; i < my_chunks.size(); i++) {
            std::memcpy(&rec[i * QREC], &opened[1].values[i][0][0], 32);
            std::memcpy(&rec[i * QREC + 4], &opened[1].witnesses[i][0][0], 64);
        }
        const uint64_t bytes = rec.size() * sizeof(uint64_t);
        DeviceBuffer send(bytes), recv(bytes * world);
        hip_ok(hipMemcpyAsync(send.get(), rec.data(), bytes, hipMemcpyHostToDevice, st), "quotient openings");
        all_gather(ctx, shard, send.get(), recv.get(), bytes);
        std::vector<uint64_t> all(rec.size() * world);
        hip_ok(hipMemcpyAsync(all.data(), recv.get(), bytes * world, hipMemcpyDeviceToHost, st), "quotient openings");
        hip_ok(hipStreamSynchronize(st), "quotient openings");
        for (uint32_t c = 0; c < num_chunks; c++) {
            const uint64_t* r = &all[((uint64_t)(c % world) * chunk_slots + c / world) * QREC];
            std::memcpy(&proof.quotient_opened[c], r, 32);
            std::memcpy(&proof.quotient_witnesses[c], r + 4, 64);
        }
    }
    const Opened& tr = opened[0];
    if (!shard) {
        proof.trace_commit = trace_commit[0];
        for (int p = 0; p < 2; p++) {
            proof.trace_opened[p] = tr.values[0][p];
            proof.trace_witnesses[p] = tr.witnesses[0][p];
        }
    } else {
        // every rank's columns land at their global positions (rank order = lane order)
        std::vector<uint64_t> rec((uint64_t)width * RECORD);
        for (uint32_t c = 0; c < width; c++) {
            uint64_t* r = rec.data() + (uint64_t)c * RECORD;
            std::memcpy(r, &trace_commit[0][c], 64);
            std::memcpy(r + 8, &tr.values[0][0][c], 32);
            std::memcpy(r + 12, &tr.values[0][1][c], 32);
            std::memcpy(r + 16, &tr.witnesses[0][0][c], 64);
            std::memcpy(r + 24, &tr.witnesses[0][1][c], 64);
        }
        const uint64_t bytes = rec.size() * sizeof(uint64_t);
        DeviceBuffer send(bytes), recv(bytes * world);
        hip_ok(hipMemcpyAsync(send.get(), rec.data(), bytes, hipMemcpyHostToDevice, st), "records");
        all_gather(ctx, shard, send.get(), recv.get(), bytes);
        std::vector<uint64_t> all(rec.size() * world);
        hip_ok(hipMemcpyAsync(all.data(), recv.get(), bytes * world, hipMemcpyDeviceToHost, st), "records");
        hip_ok(hipStreamSynchronize(st), "records");
        const uint64_t full = (uint64_t)width * world;
        proof.trace_commit.resize(full);
        for (int p = 0; p < 2; p++) {
            proof.trace_opened[p].resize(full);
            proof.trace_witnesses[p].resize(full);
        }
        for (uint64_t c = 0; c < full; c++) {
            const uint64_t* r = all.data() + c * RECORD;
            std::memcpy(&proof.trace_commit[c], r, 64);
            std::memcpy(&proof.trace_opened[0][c], r + 8, 32);
            std::memcpy(&proof.trace_opened[1][c], r + 12, 32);
            std::memcpy(&proof.trace_witnesses[0][c], r + 16, 64);
            std::memcpy(&proof.trace_witnesses[1][c], r + 24, 64);
        }
    }
    auto t6 = tick();
    proof.stage_ms[EON_STAGE_COMMIT_TRACE] = ms(t0, t1);
    proof.stage_ms[EON_STAGE_TRACE_LDE] = ms(t1, t2);
    proof.stage_ms[EON_STAGE_QUOTIENT] = ms(t2, t3);
    proof.stage_ms[EON_STAGE_EXCHANGE] = ms(t3, t3x);
    proof.stage_ms[EON_STAGE_COMMIT_QUOTIENT] = ms(t3x, t4);
    proof.stage_ms[EON_STAGE_OPEN] = ms(t4, t5);
    proof.stage_ms[EON_STAGE_ASSEMBLE] = ms(t5, t6);
    (void)rank;
    return proof;
}

}  // namespace eon_host
