// extern "C" surface of the prove driver (include/eon_prove.h).
#include <cstring>
#include <string>

#include "eon_prove.h"
#include "prover.h"

struct eon_kzg_pcs {
    eon_host::KzgPcs* pcs = nullptr;
    std::string last_error;
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

}  // namespace

extern "C" {

uint32_t eon_prove_abi_version(void) { return 1; }

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

int eon_prove_p2air(eon_kzg_pcs* pcs, const eon_p2air* air, const eon_fr* trace, uint64_t height,
                    const eon_fr* alpha, const eon_fr* zeta, uint32_t max_constraint_degree,
                    const eon_collective* shard, eon_proof* out) {
    if (!pcs || !pcs->pcs || !air || !trace || !alpha || !zeta || !out) return EON_E_ARG;
    if (!out->trace_commit || !out->quotient_commit || !out->trace_opened || !out->trace_witnesses ||
        !out->quotient_opened || !out->quotient_witnesses)
        return EON_E_ARG;
    return guarded(pcs, [&] {
        using namespace eon_host;
        Proof p = prove(*pcs->pcs, air, trace, height, Fr::from_abi(*alpha), Fr::from_abi(*zeta),
                        max_constraint_degree, shard);
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
    });
}

}  // extern "C"
