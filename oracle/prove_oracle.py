"""CPU restatement of eon_uni_stark::prove for the Poseidon2-AIR with KzgPcs, assembled from the
C restatement oracle.  TEST INFRASTRUCTURE ONLY.

Follows prove_with_preprocessed (eon-uni-stark/src/prover.rs:28-534) with the reference's own
algorithms where they differ from the GPU path: get_evaluations_on_domain is the Horner loop of
kzg/src/pcs.rs:267-287, openings run quotient_and_eval per column (kzg/src/util.rs:100-111),
every commitment is commit_column = G1::multi_exp (kzg/src/util.rs:37-40).  alpha and zeta are
inputs, or, with a pyoracle.DuplexChallenger, sampled from the transcript as prover.rs:196-208,
300, 373, 416 (observe log_ext_degree, log_degree, preprocessed width 0, the trace commitment;
alpha; observe the quotient commitment; zeta).
"""

import numpy as np

from . import coracle as C
from . import pyoracle as O


def _lim(x):
    return np.array(O.int_to_limbs(O.to_mont(x % O.P)), dtype=np.uint64)


def _points(abi_rows):
    return [O.g1_from_bytes(np.ascontiguousarray(r, dtype=np.uint64).tobytes()) for r in abi_rows]


def prove(trace, srs, consts, vl, alpha_int, zeta_int, log_qd=1, challenger=None, constraint_fn=None, publics=(),
          lde_fn=None, timings=None):
    """consts / vl: the Poseidon2-AIR (C restatement of its quotient); or constraint_fn (the
    signature of pyoracle.quotient_values_fn) for any other AIR, with its public values.

    lde_fn: None = the reference's Horner get_evaluations_on_domain; or a substitute (coeffs,
    log_q, shift) -> LDE (the coset-DFT restatement), for CPU baselines at sizes the Horner loop
    cannot reach.  timings: an optional dict that receives per-stage seconds."""
    import time

    t0 = time.perf_counter()
    n, w = trace.shape[0], trace.shape[1]
    log_n = n.bit_length() - 1
    coeffs = C.idft_batch(trace)  # coset_idft_batch(evals, shift 1) (kzg/src/pcs.rs:242)
    trace_commit = C.g1_msm_columns(srs[:n], coeffs)  # commit_column per column (pcs.rs:244-251)
    t1 = time.perf_counter()
    if challenger is not None:
        for v in (log_n, log_n, 0):
            challenger.observe(v)
        challenger.observe_g1(_points(trace_commit))
        for v in publics:  # observe_slice(public_values) (prover.rs:208)
            challenger.observe(v)
        alpha_int = challenger.sample()
    alpha = _lim(alpha_int)
    lde = (lde_fn or C.kzg_evaluations_on_domain)(coeffs, log_n + log_qd, _lim(O.GENERATOR))
    t2 = time.perf_counter()
    if constraint_fn is None:
        qv = C.p2_quotient_values(lde, log_n, log_qd, vl, consts, alpha)
    else:
        rows = [[O.from_mont(O.limbs_to_int([int(v) for v in e])) for e in r] for r in lde]
        qv = np.stack([_lim(v) for v in O.quotient_values_fn(rows, log_n, log_qd, constraint_fn, alpha_int,
                                                               list(publics))])
    t3 = time.perf_counter()
    chunks = 1 << log_qd
    g_q = O.two_adic_generator(log_n + log_qd)
    q_coeffs, quotient_commit = [], []
    for c in range(chunks):
        ev = np.ascontiguousarray(qv.reshape(n, chunks, 4)[:, c:c + 1, :])
        shift = O.GENERATOR * pow(g_q, c, O.P) % O.P
        cc = C.coset_idft_batch(ev, _lim(shift))
        q_coeffs.append(cc)
        quotient_commit.append(C.g1_msm(srs[:n], cc[:, 0]))
    if challenger is not None:
        challenger.observe_g1(_points(quotient_commit))
        zeta_int = challenger.sample()
    zeta_next = zeta_int * O.two_adic_generator(log_n) % O.P
    t4 = time.perf_counter()

    def open_matrix(cf, points):
        # per (point, column): quotient_and_eval + commit_column(quotient) (pcs.rs:289-335)
        vals, wits = [], []
        for z in points:
            v, wt = C.open_columns(srs[:max(n - 1, 1)], cf, _lim(z))
            vals.append(v)
            wits.append(wt)
        return vals, wits

    trace_open = open_matrix(coeffs, [zeta_int, zeta_next])
    quot_open = [open_matrix(cc, [zeta_int]) for cc in q_coeffs]
    t5 = time.perf_counter()
    if timings is not None:
        timings.update({"commit to trace data": t1 - t0, "trace LDE (get_evaluations_on_domain)": t2 - t1,
                        "quotient_values": t3 - t2, "commit to quotient poly chunks": t4 - t3, "open": t5 - t4})
    return {
        "trace_commit": trace_commit,
        "quotient_commit": np.stack(quotient_commit),
        "trace_open": trace_open,
        "quotient_open": quot_open,
        "quotient_values": qv,
        "alpha": alpha_int,
        "zeta": zeta_int,
    }
