"""Host-side mirror of eon_uni_stark::prove for the Poseidon2-AIR with KzgPcs, on device.

Reference: prove / prove_with_preprocessed (eon-uni-stark/src/prover.rs:28-534), specialised to
what the benchmark AIR exercises: no preprocessed columns, no lookups, ZK off
(KzgPcs::ZK = false, kzg/src/pcs.rs:216), Challenge = Fr.

Fiat-Shamir: the reference samples alpha and zeta from a DuplexChallenger over
Poseidon2Bn254 (prover.rs:196-208,300,416).  The transcript is out of scope this round
(its G1 byte encoding is halo2curves-internal and unpinned), so alpha and
zeta are explicit inputs; every value the prover computes from them is the reference's.

Stage timings (HIP events via the host clock after a device synchronize) are returned under
the reference's span names ("commit to trace data", "commit to quotient poly chunks", "open").
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field

from .field import FR_MODULUS
from .kzg import Domain, GpuKzgPcs


@dataclass
class Proof:
    """eon-uni-stark/src/proof.rs:19-44 (commitments, opened values, opening proof, degree bits)."""

    trace_commit: object
    quotient_commit: object
    opened: object
    degree_bits: int
    timings_ms: dict = field(default_factory=dict)


def log_quotient_degree(max_constraint_degree: int) -> int:
    """get_log_quotient_degree (eon-uni-stark/src/symbolic_builder.rs:15-43), ZK off."""
    d = max(max_constraint_degree, 2) - 1
    return (d - 1).bit_length()


def prove(air, pcs: GpuKzgPcs, trace, alpha: int, zeta: int, max_constraint_degree: int = 3,
          sync=None) -> Proof:
    """trace: (N, width, 4) device tensor.  The Poseidon2-AIR's constraints have degree 3."""
    import torch

    def tick():
        torch.cuda.synchronize(trace.device)
        return time.perf_counter()

    t = {}
    n = int(trace.shape[0])
    log_n = n.bit_length() - 1
    log_qd = log_quotient_degree(max_constraint_degree)
    num_chunks = 1 << log_qd
    trace_domain = pcs.natural_domain_for_degree(n)

    t0 = tick()
    trace_commit, trace_data = pcs.commit([(trace_domain, trace)])  # prover.rs:186-187
    t1 = tick()
    quotient_domain = trace_domain.create_disjoint_domain(1 << (log_n + log_qd))  # prover.rs:307-308
    lde = pcs.get_evaluations_on_domain(trace_data, 0, quotient_domain)  # prover.rs:315
    t2 = tick()
    qv = air.quotient_values(lde, log_n, log_qd, alpha)  # prover.rs:328-342
    del lde
    t3 = tick()
    quotient_commit, quotient_data = pcs.commit_quotient(quotient_domain, qv, num_chunks)  # :371-372
    t4 = tick()
    zeta_next = trace_domain.next_point(zeta)  # prover.rs:416-419
    opened = pcs.open([(trace_data, [[zeta, zeta_next]]),
                       (quotient_data, [[zeta]] * num_chunks)])  # prover.rs:424-442
    t5 = tick()
    t.update({
        "commit to trace data": (t1 - t0) * 1e3,
        "trace LDE (get_evaluations_on_domain)": (t2 - t1) * 1e3,
        "quotient_values": (t3 - t2) * 1e3,
        "commit to quotient poly chunks": (t4 - t3) * 1e3,
        "open": (t5 - t4) * 1e3,
    })
    return Proof(trace_commit, quotient_commit, opened, log_n, t)


def zeta_next_of(zeta: int, log_n: int) -> int:
    return Domain(1, log_n).next_point(zeta) % FR_MODULUS
