// The prover's Fiat-Shamir transcript: DuplexChallenger<Fr, Poseidon2Bn254<3>,
// 3, 2> on the host, and the KzgCommitment observation through compressed G1 bytes.
//
//   Poseidon2Bn254<3>   Poseidon2::permute_mut (poseidon2/src/lib.rs:107-111): initial mds_light
//                       (external.rs:128-133, 321-336), the initial full rounds (add_rc_and_sbox,
//                       generic.rs:24-30, then mds_light), the partial rounds on state[0] with the
//                       internal matrix [2,1,1;1,2,1;1,1,3] (bn254/src/poseidon2.rs:55-63,
//                       internal.rs:70-84), the terminal full rounds.  x^5 S-box.  Round constants
//                       are inputs (the reference draws them with new_from_rng, lib.rs:66-74).
//   DuplexChallenger    challenger/src/duplex_challenger.rs:62-200: observe overwrites the rate
//                       part when RATE inputs are buffered; sample pops the LAST output element.
//   observe(commitment) kzg/src/pcs.rs:403-437: every column's G1 compressed to 32 bytes, read as
//                       four little-endian u64 chunks, each observed as Fr::from_u64.
//
// The compressed encoding is halo2curves' (an absent dependency, semver 0.9): x canonical little-
// endian with the two spare top bits as flags -- bit 7 of byte 31 = y is odd, bit 6 = identity
// (then x = 0).  No fixture in the reference pins these bytes: parity unpinned.
// One transcript costs ~2.6k permutations at the benchmark width (1312 commitments x 4 chunks / 2),
// a few ms on one host core; the driver runs it while the device extends the trace.
#pragma once
#include <stdint.h>

#include <vector>

#include "eon_prove.h"
#include "fr_host.h"

namespace eon_host {

Fr fr_add(const Fr& a, const Fr& b);

class Poseidon2Bn254 {
   public:
    explicit Poseidon2Bn254(const eon_poseidon2_constants& c);
    void permute(Fr s[3]) const;

   private:
    template <bool ADX>
    void permute_impl(Fr s[3]) const;
    std::vector<FrLazy> begin_, partial_, end_;  // begin_/end_: half_full_rounds x 3
    uint32_t hf_ = 0;
};

class DuplexChallenger {
   public:
    static constexpr int WIDTH = 3, RATE = 2;
    explicit DuplexChallenger(const Poseidon2Bn254& perm) : perm_(perm) {}
    void observe(const Fr& v);
    // CanObserve<KzgCommitment> (kzg/src/pcs.rs:417-436) for one matrix's columns
    void observe_g1(const eon_g1_affine* points, uint64_t n);
    Fr sample();
    const Fr* state() const { return state_; }

   private:
    void duplexing();
    Poseidon2Bn254 perm_;
    Fr state_[WIDTH] = {Fr::zero(), Fr::zero(), Fr::zero()};
    std::vector<Fr> in_, out_;
};

// G1Affine::to_bytes (halo2curves compressed, see above) of an eon_g1_affine
void g1_to_bytes(const eon_g1_affine& p, uint8_t out[32]);

}  // namespace eon_host
