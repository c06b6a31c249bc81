/*
 * eon_prove.h -- C ABI of the native prove driver (libeonprove.so), the host side ABOVE eon.h.
 *
 * The reference's prover is compiled Rust; its toolchain is absent here, so the orchestration is
 * C++ (plonky3_eon_amd/host/) calling only the eon.h entry points, with the reference's shapes:
 *   eon_kzg_pcs      KzgPcs (kzg/src/pcs.rs:143-402) with the test SRS init_srs_unsafe
 *                    (kzg/src/params.rs:123-139): commit / get_evaluations_on_domain /
 *                    commit_quotient / open of the Pcs trait (commit/src/pcs.rs:21-187)
 *   eon_prove_p2air  prove_with_preprocessed (eon-uni-stark/src/prover.rs:28-512) for the
 *                    Poseidon2-AIR: no preprocessed columns, no lookups,
 *                    ZK off, Challenge = Fr.  alpha and zeta are either inputs
 *                    (eon_prove_p2air) or sampled from the Fiat-Shamir transcript
 *                    (eon_prove_p2air_fs with an eon_challenger).
 *   eon_prove_air    the same for any AIR compiled into an eon_air_program (eon.h), with public
 *                    values (e.g. eon-uni-stark/tests/fib_air.rs's FibonacciAir)
 *   eon_challenger   DuplexChallenger<Fr, Poseidon2Bn254<3>, 3, 2>
 *                    (challenger/src/duplex_challenger.rs, bn254/src/poseidon2.rs) on the host.
 * Conventions are eon.h's: 0 / negative EON_E_* codes (the reference panics), host outputs,
 * device inputs, work on the context's stream.
 */
#ifndef EON_PROVE_H
#define EON_PROVE_H

#include <stdint.h>

#include "eon.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct eon_kzg_pcs eon_kzg_pcs;

/* KzgPcs::new(max_degree, alpha): SRS g1_powers[0..=max_degree] generated and kept on device as
 * fixed-base MSM bases (alpha is a host pointer). */
int eon_kzg_pcs_create(eon_ctx* ctx, uint64_t max_degree, const eon_fr* srs_alpha, eon_kzg_pcs** out);
void eon_kzg_pcs_destroy(eon_kzg_pcs* pcs);
/* message of the last failing call on this pcs (driver-side errors and eon.h errors) */
const char* eon_kzg_pcs_last_error(const eon_kzg_pcs* pcs);

/* Lane-sharded prove: this rank's share of VECTOR_LEN and an all-gather over
 * DEVICE buffers (eon_collective, declared in eon.h). */

/* An RCCL (NCCL API over xGMI) all-gather for eon_collective: rank 0 creates the unique id
 * (128 bytes), every rank receives it out of band (e.g. torch.distributed) and initialises its
 * communicator on the current HIP device (the context's). */
int eon_rccl_unique_id(uint8_t id[128]);
int eon_rccl_collective_init(uint32_t rank, uint32_t world, const uint8_t id[128], eon_collective* out);
/* What the communicator itself reports (evidence that RCCL saw `world` ranks on distinct GPUs):
 * ncclCommCount, ncclCommUserRank, ncclCommCuDevice and that device's PCI bus id (NUL-terminated,
 * at most pci_len bytes); any output pointer may be NULL.  EON_E_ARG if `coll` is not an RCCL
 * collective of eon_rccl_collective_init. */
int eon_rccl_collective_info(const eon_collective* coll, int32_t* count, int32_t* user_rank, int32_t* device,
                             char* pci_bus_id, uint32_t pci_len);
void eon_rccl_collective_finalize(eon_collective* coll);
/* The one-GPU proxy of rank `rank` in a `world`-rank lane-sharded prove (bench.py
 * --emulate-world): its all-gather writes this rank's block into every slot, its all-to-all
 * keeps every block, both as device copies on the given stream.  Results are NOT a valid
 * proof; the point is the rank's own work, including the full replicated transcript. */
int eon_emulated_collective_init(uint32_t rank, uint32_t world, eon_collective* out);

enum {
    EON_STAGE_COMMIT_TRACE = 0,    /* "commit to trace data" (prover.rs:186-187) */
    EON_STAGE_TRACE_LDE = 1,       /* get_evaluations_on_domain (prover.rs:315) */
    EON_STAGE_QUOTIENT = 2,        /* quotient_values (prover.rs:328-342) */
    EON_STAGE_EXCHANGE = 3,        /* sharded: all-gather + combine of partial quotients */
    EON_STAGE_COMMIT_QUOTIENT = 4, /* "commit to quotient poly chunks" (prover.rs:371-372) */
    EON_STAGE_OPEN = 5,            /* "open" (prover.rs:424-442) */
    EON_STAGE_ASSEMBLE = 6,        /* sharded: all-gather of per-column results */
    EON_STAGES = 8
};

/* Proof fields (eon-uni-stark/src/proof.rs:19-44), caller-allocated host arrays; W is the FULL
 * trace width (164 * VECTOR_LEN over all ranks), C = 2^log_qd quotient chunks (2 for degree 3). */
typedef struct {
    eon_g1_affine* trace_commit;       /* [W] */
    eon_g1_affine* quotient_commit;    /* [C] */
    eon_fr* trace_opened;              /* [2][W]: values at zeta, zeta * h */
    eon_g1_affine* trace_witnesses;    /* [2][W] */
    eon_fr* quotient_opened;           /* [C]: chunk c at zeta */
    eon_g1_affine* quotient_witnesses; /* [C] */
    uint32_t degree_bits;              /* out: log2 of the trace height */
    double stage_ms[EON_STAGES];       /* out: host clock around each stage (device synchronized) */
} eon_proof;

/* prove: `trace` is this rank's (height x width(air)) trace on device; `alpha`, `zeta` host.
 * `shard` NULL = the whole AIR on this device.  max_constraint_degree = 3 for the Poseidon2-AIR
 * (log_qd = 1, get_log_quotient_degree, symbolic_builder.rs:15-43). */
int eon_prove_p2air(eon_kzg_pcs* pcs, const eon_p2air* air, const eon_fr* trace, uint64_t height,
                    const eon_fr* alpha, const eon_fr* zeta, uint32_t max_constraint_degree,
                    const eon_collective* shard, eon_proof* out);

/* ---- Fiat-Shamir transcript, host only ---------------------------------
 * Poseidon2Bn254<3>::permute_mut (poseidon2/src/lib.rs:107-111) of state[3] in place, with the
 * round constants of `perm` (the AIR's constant layout; the reference draws them with
 * Poseidon2::new_from_rng(2 * half_full_rounds, partial_rounds), lib.rs:66-74). */
int eon_poseidon2_bn254_permute(const eon_poseidon2_constants* perm, eon_fr state[3]);
/* G1Affine::to_bytes, the 32-byte compressed form KzgCommitment observation reads
 * (kzg/src/pcs.rs:417-436): canonical x little-endian, bit 7 of byte 31 = y odd, bit 6 =
 * identity.  halo2curves' encoding, absent here: parity unpinned. */
int eon_g1_to_bytes(const eon_g1_affine* point, uint8_t out[32]);

typedef struct eon_challenger eon_challenger;
/* DuplexChallenger::new(Poseidon2Bn254<3>) (duplex_challenger.rs:68-78): zero sponge state */
int eon_challenger_create(const eon_poseidon2_constants* perm, eon_challenger** out);
void eon_challenger_destroy(eon_challenger* ch);
/* observe(Fr) for each of values[0..n) (duplex_challenger.rs:111-121) */
int eon_challenger_observe(eon_challenger* ch, const eon_fr* values, uint64_t n);
/* observe(KzgCommitment) for one matrix's n column commitments (kzg/src/pcs.rs:417-436) */
int eon_challenger_observe_g1(eon_challenger* ch, const eon_g1_affine* points, uint64_t n);
/* sample() -> Fr = sample_algebra_element for Challenge = Fr (duplex_challenger.rs:185-200) */
int eon_challenger_sample(eon_challenger* ch, eon_fr* out);
/* the sponge state (3 Fr), for tests */
int eon_challenger_state(const eon_challenger* ch, eon_fr out[3]);

/* prove with the transcript of prove_with_preprocessed: observe log_ext_degree, log_degree, the
 * preprocessed width (0) and the trace commitment (prover.rs:196-202), sample alpha (:300),
 * observe the quotient commitment (:373), sample zeta (:416).  `challenger` is the config's
 * initialised challenger and is advanced as the reference's; alpha_out / zeta_out (host,
 * nullable) receive the sampled challenges.  Sharded: the trace commitments are all-gathered
 * before alpha so every rank observes the full transcript. */
int eon_prove_p2air_fs(eon_kzg_pcs* pcs, const eon_p2air* air, const eon_fr* trace, uint64_t height,
                       eon_challenger* challenger, uint32_t max_constraint_degree,
                       const eon_collective* shard, eon_proof* out, eon_fr* alpha_out, eon_fr* zeta_out);

/* prove_with_preprocessed (prover.rs:28-512) for ANY AIR given as an eon_air_program (eon.h: the
 * compiled get_symbolic_constraints DAG) with its public values (host, n_public Fr): the quotient
 * degree is the program's get_log_quotient_degree (prover.rs:150-157), C = 2^that chunks, the
 * public values are observed after the trace commitment (prover.rs:208) and read by the
 * constraints (Entry::Public).  No sharding.  The trace is height x width(prog) on device. */
int eon_prove_air(eon_kzg_pcs* pcs, const eon_air_program* prog, const eon_fr* trace, uint64_t height,
                  const eon_fr* publics, uint32_t n_public, const eon_fr* alpha, const eon_fr* zeta,
                  eon_proof* out);
int eon_prove_air_fs(eon_kzg_pcs* pcs, const eon_air_program* prog, const eon_fr* trace, uint64_t height,
                     const eon_fr* publics, uint32_t n_public, eon_challenger* challenger, eon_proof* out,
                     eon_fr* alpha_out, eon_fr* zeta_out);

uint32_t eon_prove_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* EON_PROVE_H */
