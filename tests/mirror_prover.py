"""TEST-ONLY Python mirror of eon_uni_stark::prove for the Poseidon2-AIR with KzgPcs, on device.

The product host is the C++ driver (plonky3_eon_amd/host, libeonprove.so); this second host over
the same C ABI stays in tests/ to cross-check it field by field (tests/test_gpu_prove.py) and to
exercise the lane-sharded Python orchestration (tests/_dist_worker.py).

Reference: prove / prove_with_preprocessed (eon-uni-stark/src/prover.rs:28-534), specialised to
what the benchmark AIR exercises: no preprocessed columns, no lookups, ZK off
(KzgPcs::ZK = false, kzg/src/pcs.rs:216), Challenge = Fr.

Fiat-Shamir: the reference samples alpha and zeta from a DuplexChallenger over
Poseidon2Bn254 (prover.rs:196-208,300,373,416).  With `challenger` (native.Challenger, the host
transcript of libeonprove) they are sampled the same way; without it they
are explicit inputs.  The compressed G1 bytes the transcript reads are halo2curves-internal and
unpinned.

Stage timings (HIP events via the host clock after a device synchronize) are returned under
the reference's span names ("commit to trace data", "commit to quotient poly chunks", "open").
"""

from __future__ import annotations

import time

import numpy as np

from mirror_kzg import Domain, GpuKzgPcs
from plonky3_eon_amd.field import FR_MODULUS, fr_mont, fr_unmont
from plonky3_eon_amd.proof import Proof, log_quotient_degree  # noqa: F401 (re-exported)


def prove(air, pcs: GpuKzgPcs, trace, alpha: int | None, zeta: int | None, max_constraint_degree: int = 3,
          shard=None, challenger=None) -> Proof:
    """trace: (N, width, 4) device tensor.  The Poseidon2-AIR's constraints have degree 3.

    challenger: a native.Challenger (DuplexChallenger<Fr, Poseidon2Bn254<3>, 3, 2>); alpha and
    zeta are then sampled from the transcript (prover.rs:196-208, 300, 373, 416) and returned in
    proof.alpha / proof.zeta, the arguments ignored.

    shard: a distributed.Shard when the prove is split by vector lane over several ranks; `air`
    and `trace` are then this rank's lanes (a VectorizedPoseidon2Air of shard.lanes' length and
    its trace columns), and every rank returns the full proof (plonky3_eon_amd/distributed.py).
    """
    import torch

    from plonky3_eon_amd import distributed as D

    def tick():
        torch.cuda.synchronize(trace.device)
        return time.perf_counter()

    t = {}
    n = int(trace.shape[0])
    log_n = n.bit_length() - 1
    log_qd = log_quotient_degree(max_constraint_degree)
    num_chunks = 1 << log_qd
    trace_domain = pcs.natural_domain_for_degree(n)
    if shard is not None and shard.world > 1:
        l0, l1 = shard.lanes
        if air.vector_len != l1 - l0:
            raise ValueError(f"rank {shard.rank} owns lanes [{l0}, {l1}) but the AIR has {air.vector_len}")
    else:
        shard = None

    t0 = tick()
    trace_commit, trace_data = pcs.commit([(trace_domain, trace)])  # prover.rs:186-187
    t1 = tick()
    if challenger is not None:
        commit_all = trace_commit[0]
        if shard is not None:  # every rank observes the full commitment, in lane order
            local = torch.from_numpy(np.ascontiguousarray(trace_commit[0]).view(np.int64)).to(trace.device)
            commit_all = D.all_gather_rows(local, shard.group).cpu().numpy().view(np.uint64).reshape(-1, 8)
        challenger.observe(np.stack([_lim(log_n), _lim(log_n), _lim(0)]))  # prover.rs:196-198
        challenger.observe_g1(commit_all)  # :202
        alpha = fr_unmont(_limbs_int(challenger.sample()))  # :300
    quotient_domain = trace_domain.create_disjoint_domain(1 << (log_n + log_qd))  # prover.rs:307-308
    lde = pcs.get_evaluations_on_domain(trace_data, 0, quotient_domain)  # prover.rs:315
    t2 = tick()
    qv = air.quotient_values(lde, log_n, log_qd, alpha)  # prover.rs:328-342
    del lde
    t3 = tick()
    if shard is not None:
        parts = D.all_gather_rows(qv, shard.group)
        weights = D.lane_weights(alpha, shard.vector_len, shard.world, air.constraints_per_perm)
        qv = D.combine_partials(pcs.ctx, parts, weights)
        del parts
    t3x = tick()
    quotient_commit, quotient_data = pcs.commit_quotient(quotient_domain, qv, num_chunks)  # :371-372
    if challenger is not None:
        for m in quotient_commit:
            challenger.observe_g1(m)  # :373
        zeta = fr_unmont(_limbs_int(challenger.sample()))  # :416
    t4 = tick()
    zeta_next = trace_domain.next_point(zeta)  # prover.rs:416-419
    opened = pcs.open([(trace_data, [[zeta, zeta_next]]),
                       (quotient_data, [[zeta]] * num_chunks)])  # prover.rs:424-442
    t5 = tick()
    if shard is not None:
        tr = opened[0]
        rec = D.pack_columns(trace_commit[0], tr.values[0], tr.witnesses[0])
        commit_all, values_all, wits_all = D.unpack_columns(D.gather_columns(rec, trace.device, shard.group))
        trace_commit = [commit_all]
        tr.values[0], tr.witnesses[0] = values_all, wits_all
    t6 = tick()
    t.update({
        "commit to trace data": (t1 - t0) * 1e3,
        "trace LDE (get_evaluations_on_domain)": (t2 - t1) * 1e3,
        "quotient_values": (t3 - t2) * 1e3,
        "commit to quotient poly chunks": (t4 - t3x) * 1e3,
        "open": (t5 - t4) * 1e3,
    })
    if shard is not None:
        t["exchange partial quotients"] = (t3x - t3) * 1e3
        t["assemble columns"] = (t6 - t5) * 1e3
    return Proof(trace_commit, quotient_commit, opened, log_n, t, alpha, zeta)


def _lim(x: int) -> np.ndarray:
    m = fr_mont(x % FR_MODULUS)
    return np.array([(m >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)


def _limbs_int(a) -> int:
    return sum(int(v) << (64 * i) for i, v in enumerate(np.asarray(a).reshape(4)))


def zeta_next_of(zeta: int, log_n: int) -> int:
    return Domain(1, log_n).next_point(zeta) % FR_MODULUS
