"""The headline proof is VALID at full size: bench.py's exact configs[3] workload (Poseidon2-AIR,
VECTOR_LEN 8, log-trace-length 17 = 2^20 permutations, width 1312, KzgPcs with the alpha = 12345
test SRS, Fiat-Shamir transcript) proved by the native driver on the GPU, then checked on the CPU
by the verifier restatement (oracle/verify_oracle.py):

* the GPU trace equals the C restatement's trace generation (generation.rs) bit for bit;
* alpha and zeta re-derived by replaying the transcript (the oracle's DuplexChallenger);
* the out-of-domain identity of verify_constraints (eon-uni-stark/src/verifier.rs:77-160);
* every opened trace value (1312 columns x {zeta, zeta h}) equals the column polynomial there
  (barycentric evaluation of the oracle trace);
* every KZG opening (2624 trace + 2 quotient) satisfies C - [v]G == [s - z]W with the SRS
  trapdoor s (verify_batch's equation, kzg/src/util.rs:245-292) and every trace commitment is
  [f_c(s)]G -- one random linear combination, one CPU MSM.

Parity note: the challenger's Poseidon2 round constants and the compressed-G1 bytes it observes
are restated, not pinned by a reference vector; the checks above do not depend on
them beyond both sides using the same ones."""

import numpy as np
import pytest

from oracle import coracle as C
from oracle import pyoracle as O
from oracle import verify_oracle as V

pytestmark = pytest.mark.gpu


def _py_consts(limbs):
    b, p, e = limbs
    return ([[V.fr_int(x) for x in r] for r in b], [V.fr_int(x) for x in p], [[V.fr_int(x) for x in r] for r in e])


@pytest.mark.parametrize("log_n,vl", [(17, 8), (12, 2)])
def test_headline_proof_valid(gpu_ctx, log_n, vl):
    import torch

    import bench
    from plonky3_eon_amd.air import Poseidon2Air
    from plonky3_eon_amd.native import Challenger, NativeKzgPcs, Poseidon2Constants, prove_native

    n = 1 << log_n
    consts = bench.p2_constants_limbs(99)
    ch_consts = bench.p2_constants_limbs(77)
    air = Poseidon2Air(*consts, vl, gpu_ctx)
    pcs = NativeKzgPcs(n, 12345, gpu_ctx)
    inputs = bench.synthetic_fr(n * vl, 3, 5).reshape(-1, 3, 4)
    trace = air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to("cuda:0"))
    proof = prove_native(air, pcs, trace, None, None, challenger=Challenger(Poseidon2Constants(*ch_consts)))
    assert proof.degree_bits == log_n
    host_trace = trace.cpu().numpy().view(np.uint64)
    del trace
    pcs.close()

    want = C.p2_generate_trace(inputs, vl, C.P2Constants(*consts))
    assert np.array_equal(host_trace, want), "GPU trace differs from the restated generation.rs"
    del want
    res = V.verify_kzg_proof(proof, V.p2air_constraint_fn(_py_consts(consts), vl), log_n, 1, 12345,
                             challenger=O.DuplexChallenger(_py_consts(ch_consts)), trace=host_trace)
    assert res == {"transcript": True, "ood": True, "opened_vs_trace": True, "kzg": True}, res
    # the reference's own verifier equation with a real pairing (KzgPcs::verify -> verify_batch,
    # kzg/src/pcs.rs:337-400, kzg/src/util.rs:245-292) on a sample of the openings: 3 trace columns
    # at zeta and zeta h, and the quotient chunks at zeta (oracle/pairing.py, ~0.15 s per loop)
    from oracle import pairing as E

    def pt(row):
        return O.g1_from_bytes(np.ascontiguousarray(row, dtype=np.uint64).reshape(8).tobytes())

    tc = np.asarray(proof.trace_commit[0]).reshape(-1, 8)
    zn = proof.zeta * O.two_adic_generator(log_n) % O.P
    tr, qo = proof.opened
    openings = []
    for c in (0, tc.shape[0] // 2, tc.shape[0] - 1):
        for p, z in enumerate((proof.zeta, zn)):
            openings.append((pt(tc[c]), pt(np.asarray(tr.witnesses[0][p]).reshape(-1, 8)[c]),
                             V.fr_int(np.asarray(tr.values[0][p]).reshape(-1, 4)[c]), z))
    for c, qc in enumerate(proof.quotient_commit):
        openings.append((pt(qc), pt(qo.witnesses[c][0]), V.fr_int(np.asarray(qo.values[c][0]).reshape(-1, 4)[0]),
                         proof.zeta))
    g2a = E.g2_alpha(12345)
    assert E.verify_batch(openings, g2a)
    bad = list(openings)
    bad[0] = (bad[0][0], bad[0][1], (bad[0][2] + 1) % O.P, bad[0][3])
    assert not E.verify_batch(bad, g2a)
    # ALL 2626 openings (2 x 1312 trace + 2 quotient chunks) through the GPU verify_batch
    # (eon_kzg_verify_batch: the same multi-pairing, merged per opening point), and a tampered one
    from plonky3_eon_amd import verify as GV

    def fr_l(x):
        return np.array(O.int_to_limbs(O.to_mont(x % O.P)), dtype=np.uint64)

    com, wit, val, pts = [], [], [], []
    for p, z in enumerate((proof.zeta, zn)):
        com.append(tc)
        wit.append(np.asarray(tr.witnesses[0][p]).reshape(-1, 8))
        val.append(np.asarray(tr.values[0][p]).reshape(-1, 4))
        pts.append(np.tile(fr_l(z), (tc.shape[0], 1)))
    for c, qc in enumerate(proof.quotient_commit):
        com.append(np.asarray(qc).reshape(1, 8))
        wit.append(np.asarray(qo.witnesses[c][0]).reshape(1, 8))
        val.append(np.asarray(qo.values[c][0]).reshape(1, 4))
        pts.append(fr_l(proof.zeta)[None])
    com, wit, val, pts = (np.ascontiguousarray(np.concatenate(a), dtype=np.uint64) for a in (com, wit, val, pts))
    assert com.shape[0] == 2 * tc.shape[0] + len(proof.quotient_commit)
    g2a_gpu = GV.g2_mul(12345, ctx=gpu_ctx)
    assert GV.verify_batch(com, wit, val, pts, g2a_gpu, ctx=gpu_ctx) is True
    val[tc.shape[0] + 5] = fr_l(V.fr_int(val[tc.shape[0] + 5]) + 1)
    assert GV.verify_batch(com, wit, val, pts, g2a_gpu, ctx=gpu_ctx) is False
