// prove_with_preprocessed (eon-uni-stark/src/prover.rs:28-512) over KzgPcs, as a C++ driver above
// eon.h, for the Poseidon2-AIR (fused quotient kernel) or any AIR given as a constraint program
// with public values: no preprocessed columns, no lookups, ZK off (KzgPcs::ZK = false,
// kzg/src/pcs.rs:216), Challenge = Fr; alpha and zeta are inputs or sampled from a
// DuplexChallenger.
#pragma once
#include "eon_prove.h"
#include "pcs.h"
#include "transcript.h"

namespace eon_host {

// get_log_quotient_degree (eon-uni-stark/src/symbolic_builder.rs:15-43), ZK off
uint32_t log_quotient_degree(uint32_t max_constraint_degree);

struct Proof {
    std::vector<eon_g1_affine> trace_commit;        // [W]
    std::vector<eon_g1_affine> quotient_commit;     // [C]
    std::vector<eon_fr> trace_opened[2];            // at zeta, zeta * h: [W] each
    std::vector<eon_g1_affine> trace_witnesses[2];  // [W] each
    std::vector<eon_fr> quotient_opened;            // [C]
    std::vector<eon_g1_affine> quotient_witnesses;  // [C]
    uint32_t degree_bits = 0;
    double stage_ms[EON_STAGES] = {};
    Fr alpha, zeta;  // the challenges used
};

// The AIR being proved: the fused Poseidon2-AIR kernel (lane-shardable), or a generic constraint
// program compiled from get_symbolic_constraints (eon_air_program) with its public values.
struct AirRef {
    const eon_p2air* p2 = nullptr;
    const eon_air_program* prog = nullptr;
    const eon_fr* publics = nullptr;
    uint32_t n_public = 0;
    uint32_t width() const;
};

// `trace`: this rank's height x width(air) device trace.  With `shard` (world > 1, Poseidon2 only)
// the AIR is the rank's lane range; every rank returns the full proof.  With `challenger`, alpha
// and zeta are sampled from it (prover.rs:196-208, 300, 373, 416) and the inputs are ignored.
// max_constraint_degree is the Poseidon2-AIR's (3); a program carries its own.
Proof prove(KzgPcs& pcs, const AirRef& air, const eon_fr* trace, uint64_t height, const Fr& alpha,
            const Fr& zeta, uint32_t max_constraint_degree, const eon_collective* shard,
            DuplexChallenger* challenger = nullptr);

}  // namespace eon_host
