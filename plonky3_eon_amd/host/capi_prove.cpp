// extern "C" surface of the prove driver (include/eon_prove.h).
#include <cstring>
#include <string>

#include "eon_prove.h"
#include "prover.h"
#include "transcript.h"

struct eon_kzg_pcs {
    eon_host::KzgPcs* pcs = nullptr;
    std::string last_error;
};

struct eon_challenger {
    eon_host::DuplexChallenger ch;
};

namespace {

template <class F>
int guarded(eon_kzg_pcs* h, F&& f) {
    try {
        f();
        if (h) h->last_error.clear();
        return EON_OK;
    } catch (const eon_host::Error& e) {
        if (h) h->last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        if (h) h->last_error = "host allocation failed";
        return EON_E_OOM;
    } catch (const std::exception& e) {
        if (h) h->last_error = e.what();
        return EON_E_DEVICE;
    }
}

void copy_out(const eon_host::Proof& p, eon_proof* out);

}  // namespace

extern "C" {

uint32_t eon_prove_abi_version(void) { return 3; }

int eon_kzg_pcs_create(eon_ctx* ctx, uint64_t max_degree, const eon_fr* srs_alpha, eon_kzg_pcs** out) {
    if (!ctx || !srs_alpha || !out) return EON_E_ARG;
    eon_kzg_pcs* h = new eon_kzg_pcs();
    const int rc = guarded(h, [&] {
        h->pcs = new eon_host::KzgPcs(ctx, max_degree, eon_host::Fr::from_abi(*srs_alpha));
    });
    if (rc != EON_OK) {
        delete h;
        return rc;
    }
    *out = h;
    return EON_OK;
}

void eon_kzg_pcs_destroy(eon_kzg_pcs* pcs) {
    if (!pcs) return;
    delete pcs->pcs;
    delete pcs;
}

const char* eon_kzg_pcs_last_error(const eon_kzg_pcs* pcs) { return pcs ? pcs->last_error.c_str() : "null pcs"; }

int eon_poseidon2_bn254_permute(const eon_poseidon2_constants* perm, eon_fr state[3]) {
    if (!perm || !state) return EON_E_ARG;
    return guarded(nullptr, [&] {
        using namespace eon_host;
        const Poseidon2Bn254 p(*perm);
        Fr s[3] = {Fr::from_abi(state[0]), Fr::from_abi(state[1]), Fr::from_abi(state[2])};
        p.permute(s);
        for (int i = 0; i < 3; i++) state[i] = s[i].abi();
    });
}

int eon_g1_to_bytes(const eon_g1_affine* point, uint8_t out[32]) {
    if (!point || !out) return EON_E_ARG;
    eon_host::g1_to_bytes(*point, out);
    return EON_OK;
}

int eon_challenger_create(const eon_poseidon2_constants* perm, eon_challenger** out) {
    if (!perm || !out) return EON_E_ARG;
    return guarded(nullptr, [&] { *out = new eon_challenger{eon_host::DuplexChallenger(eon_host::Poseidon2Bn254(*perm))}; });
}

void eon_challenger_destroy(eon_challenger* ch) { delete ch; }

int eon_challenger_observe(eon_challenger* ch, const eon_fr* values, uint64_t n) {
    if (!ch || (n && !values)) return EON_E_ARG;
    for (uint64_t i = 0; i < n; i++) {
        const eon_host::Fr v = eon_host::Fr::from_abi(values[i]);
        for (int k = 3; k >= 0; k--) {  // canonical (Fr deserialisation rejects >= r)
            if (v.l[k] != eon_host::Fr::P[k]) {
                if (v.l[k] > eon_host::Fr::P[k]) return EON_E_ARG;
                break;
            }
            if (k == 0) return EON_E_ARG;
        }
    }
    for (uint64_t i = 0; i < n; i++) ch->ch.observe(eon_host::Fr::from_abi(values[i]));
    return EON_OK;
}

int eon_challenger_observe_g1(eon_challenger* ch, const eon_g1_affine* points, uint64_t n) {
    if (!ch || (n && !points)) return EON_E_ARG;
    ch->ch.observe_g1(points, n);
    return EON_OK;
}

int eon_challenger_sample(eon_challenger* ch, eon_fr* out) {
    if (!ch || !out) return EON_E_ARG;
    *out = ch->ch.sample().abi();
    return EON_OK;
}

int eon_challenger_state(const eon_challenger* ch, eon_fr out[3]) {
    if (!ch || !out) return EON_E_ARG;
    for (int i = 0; i < 3; i++) out[i] = ch->ch.state()[i].abi();
    return EON_OK;
}

int eon_prove_p2air(eon_kzg_pcs* pcs, const eon_p2air* air, const eon_fr* trace, uint64_t height,
                    const eon_fr* alpha, const eon_fr* zeta, uint32_t max_constraint_degree,
                    const eon_collective* shard, eon_proof* out) {
    if (!pcs || !pcs->pcs || !air || !trace || !alpha || !zeta || !out) return EON_E_ARG;
    if (!out->trace_commit || !out->quotient_commit || !out->trace_opened || !out->trace_witnesses ||
        !out->quotient_opened || !out->quotient_witnesses)
        return EON_E_ARG;
    return guarded(pcs, [&] {
        using namespace eon_host;
        AirRef a;
        a.p2 = air;
        Proof p = prove(*pcs->pcs, a, trace, height, Fr::from_abi(*alpha), Fr::from_abi(*zeta),
                        max_constraint_degree, shard);
        copy_out(p, out);
    });
}

int eon_prove_air(eon_kzg_pcs* pcs, const eon_air_program* prog, const eon_fr* trace, uint64_t height,
                  const eon_fr* publics, uint32_t n_public, const eon_fr* alpha, const eon_fr* zeta,
                  eon_proof* out) {
    if (!pcs || !pcs->pcs || !prog || !trace || !alpha || !zeta || !out || (n_public && !publics))
        return EON_E_ARG;
    if (!out->trace_commit || !out->quotient_commit || !out->trace_opened || !out->trace_witnesses ||
        !out->quotient_opened || !out->quotient_witnesses)
        return EON_E_ARG;
    return guarded(pcs, [&] {
        using namespace eon_host;
        AirRef a;
        a.prog = prog;
        a.publics = publics;
        a.n_public = n_public;
        Proof p = prove(*pcs->pcs, a, trace, height, Fr::from_abi(*alpha), Fr::from_abi(*zeta), 0, nullptr);
        copy_out(p, out);
    });
}

int eon_prove_air_fs(eon_kzg_pcs* pcs, const eon_air_program* prog, const eon_fr* trace, uint64_t height,
                     const eon_fr* publics, uint32_t n_public, eon_challenger* challenger, eon_proof* out,
                     eon_fr* alpha_out, eon_fr* zeta_out) {
    if (!pcs || !pcs->pcs || !prog || !trace || !challenger || !out || (n_public && !publics)) return EON_E_ARG;
    if (!out->trace_commit || !out->quotient_commit || !out->trace_opened || !out->trace_witnesses ||
        !out->quotient_opened || !out->quotient_witnesses)
        return EON_E_ARG;
    return guarded(pcs, [&] {
        using namespace eon_host;
        AirRef a;
        a.prog = prog;
        a.publics = publics;
        a.n_public = n_public;
        Proof p = prove(*pcs->pcs, a, trace, height, Fr::zero(), Fr::zero(), 0, nullptr, &challenger->ch);
        copy_out(p, out);
        if (alpha_out) *alpha_out = p.alpha.abi();
        if (zeta_out) *zeta_out = p.zeta.abi();
    });
}

int eon_prove_p2air_fs(eon_kzg_pcs* pcs, const eon_p2air* air, const eon_fr* trace, uint64_t height,
                       eon_challenger* challenger, uint32_t max_constraint_degree,
                       const eon_collective* shard, eon_proof* out, eon_fr* alpha_out, eon_fr* zeta_out) {
    if (!pcs || !pcs->pcs || !air || !trace || !challenger || !out) return EON_E_ARG;
    if (!out->trace_commit || !out->quotient_commit || !out->trace_opened || !out->trace_witnesses ||
        !out->quotient_opened || !out->quotient_witnesses)
        return EON_E_ARG;
    return guarded(pcs, [&] {
        using namespace eon_host;
        AirRef a;
        a.p2 = air;
        Proof p = prove(*pcs->pcs, a, trace, height, Fr::zero(), Fr::zero(), max_constraint_degree, shard,
                        &challenger->ch);
        copy_out(p, out);
        if (alpha_out) *alpha_out = p.alpha.abi();
        if (zeta_out) *zeta_out = p.zeta.abi();
    });
}

}  // extern "C"

namespace {

void copy_out(const eon_host::Proof& p, eon_proof* out) {
    const size_t w = p.trace_commit.size(), c = p.quotient_commit.size();
    std::memcpy(out->trace_commit, p.trace_commit.data(), w * sizeof(eon_g1_affine));
    for (int k = 0; k < 2; k++) {
        std::memcpy(out->trace_opened + k * w, p.trace_opened[k].data(), w * sizeof(eon_fr));
        std::memcpy(out->trace_witnesses + k * w, p.trace_witnesses[k].data(), w * sizeof(eon_g1_affine));
    }
    std::memcpy(out->quotient_commit, p.quotient_commit.data(), c * sizeof(eon_g1_affine));
    std::memcpy(out->quotient_opened, p.quotient_opened.data(), c * sizeof(eon_fr));
    std::memcpy(out->quotient_witnesses, p.quotient_witnesses.data(), c * sizeof(eon_g1_affine));
    out->degree_bits = p.degree_bits;
    for (int s = 0; s < EON_STAGES; s++) out->stage_ms[s] = p.stage_ms[s];
}

}  // namespace
