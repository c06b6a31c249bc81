"""CPU restatement of the eon-uni-stark verifier for KzgPcs proofs.  TEST INFRASTRUCTURE ONLY.

Checks a proof (the shapes prover.Proof / native.prove_native return: ABI limb arrays) the way the
reference's verifier does, so a full-size GPU proof can be shown VALID, not only equal to itself:

* transcript replay (eon-uni-stark/src/verifier.rs, the same observe order as prover.rs:196-208,
  300, 373, 416): alpha and zeta must be the ones the proof was built with;
* the out-of-domain identity of verify_constraints (verifier.rs:77-160): the AIR's constraints at
  (local = trace(zeta), next = trace(zeta h)) folded by the VerifierConstraintFolder
  (folder.rs:188-190: acc = acc * alpha + C), times 1 / Z_H(zeta) from selectors_at_point
  (commit/src/domain.rs:237-246), equals quotient(zeta) recomposed from the chunk openings by
  recompose_quotient_from_chunks (verifier.rs:29-71, vanishing_poly_at_point domain.rs:226-228);
* every KZG opening with the test SRS's known trapdoor s (init_srs_unsafe, kzg/src/params.rs:
  123-139): C - [v]G == [s - z]W, which is verify_batch's pairing equation
  e(C - vG + zW, H) == e(W, sH) (kzg/src/util.rs:245-292) with the pairing replaced by the
  trapdoor.  All claims are combined with independent random 128-bit weights into ONE multi-scalar
  multiplication on the CPU (oracle/eon_oracle.c Pippenger), which must be the identity;
* optionally, against the trace itself: every opened trace value equals the column polynomial at
  zeta / zeta h (barycentric, or_bary_eval_cols) and sum_c r_c C_c == [sum_c r_c f_c(s)] G.
"""

from __future__ import annotations

import random

import numpy as np

from . import coracle as C
from . import pyoracle as O


def fr_int(limbs) -> int:
    """Montgomery limbs -> canonical int."""
    return O.from_mont(O.limbs_to_int([int(x) for x in np.asarray(limbs, dtype=np.uint64).reshape(4)]))


def fr_limbs(x: int) -> np.ndarray:
    return np.array(O.int_to_limbs(O.to_mont(x % O.P)), dtype=np.uint64)


def replay_transcript(challenger: O.DuplexChallenger, log_n: int, trace_commit, quotient_commit, publics=()):
    """prover.rs:196-202 (log_ext_degree, log_degree, preprocessed width 0, trace commitment),
    :208 (public values), :300 (alpha), :373 (quotient commitment), :416 (zeta).  Commitments are
    ABI rows (.., 8)."""
    pts = lambda rows: [O.g1_from_bytes(np.ascontiguousarray(r, dtype=np.uint64).tobytes())  # noqa: E731
                        for r in np.asarray(rows, dtype=np.uint64).reshape(-1, 8)]
    for v in (log_n, log_n, 0):
        challenger.observe(v)
    challenger.observe_g1(pts(trace_commit))
    for v in publics:
        challenger.observe(v)
    alpha = challenger.sample()
    challenger.observe_g1(pts(quotient_commit))
    zeta = challenger.sample()
    return alpha, zeta


def vanishing_at(shift: int, log_size: int, x: int) -> int:
    """TwoAdicMultiplicativeCoset::vanishing_poly_at_point (commit/src/domain.rs:226-228)."""
    return (pow(x * pow(shift, -1, O.P) % O.P, 1 << log_size, O.P) - 1) % O.P


def selectors_at_point(log_n: int, x: int, shift: int = 1):
    """commit/src/domain.rs:237-246: (is_first_row, is_last_row, is_transition, inv_vanishing)."""
    u = x * pow(shift, -1, O.P) % O.P
    z_h = (pow(u, 1 << log_n, O.P) - 1) % O.P
    h_inv = pow(O.two_adic_generator(log_n), -1, O.P)
    return (z_h * pow(u - 1, -1, O.P) % O.P, z_h * pow(u - h_inv, -1, O.P) % O.P, (u - h_inv) % O.P,
            pow(z_h, -1, O.P))


def recompose_quotient(log_n: int, log_qd: int, chunk_values, zeta: int) -> int:
    """recompose_quotient_from_chunks (verifier.rs:29-71) for the chunks of the quotient domain
    (shift GENERATOR, size 2^(log_n + log_qd)) split round-robin (commit/src/domain.rs:174-221):
    chunk c has shift GENERATOR * w_Q^c and size 2^log_n."""
    g_q = O.two_adic_generator(log_n + log_qd)
    shifts = [O.GENERATOR * pow(g_q, c, O.P) % O.P for c in range(1 << log_qd)]
    total = 0
    for i, si in enumerate(shifts):
        zp = 1
        for j, sj in enumerate(shifts):
            if j != i:
                zp = zp * vanishing_at(sj, log_n, zeta) % O.P * pow(vanishing_at(sj, log_n, si), -1, O.P) % O.P
        total += zp * chunk_values[i]
    return total % O.P


def fold_constraints(constraints, alpha: int) -> int:
    """VerifierConstraintFolder::assert_zero (folder.rs:188-190): acc = acc * alpha + x."""
    acc = 0
    for c in constraints:
        acc = (acc * alpha + c) % O.P
    return acc


def ood_check(constraint_fn, local, nxt, quotient_chunks, alpha: int, zeta: int, log_n: int, log_qd: int) -> bool:
    """verify_constraints (verifier.rs:77-160).  constraint_fn(local, next, sels) -> the AIR's
    assert_zero values in eval order (sels = selectors_at_point of the trace domain)."""
    sels = selectors_at_point(log_n, zeta)
    folded = fold_constraints(constraint_fn(local, nxt, sels), alpha)
    quotient = recompose_quotient(log_n, log_qd, quotient_chunks, zeta)
    return folded * sels[3] % O.P == quotient


def fib_constraint_fn(publics):
    """FibonacciAir (eon-uni-stark/tests/fib_air.rs:21-51) at the opened point: the selectors of
    selectors_at_point (is_first_row, is_last_row, is_transition)."""

    def fn(local, nxt, sels):
        return O.fib_constraints(local, nxt, sels[:3], publics)

    return fn


def p2air_constraint_fn(consts_int, vl: int):
    """The (vectorized) Poseidon2-AIR's constraints (poseidon2-air/src/air.rs:108-288, lanes in
    order as vectorized.rs:259-274); no selectors, no next row."""
    nc = O.p2_num_cols(len(consts_int[0]), len(consts_int[1]))

    def fn(local, nxt, sels):
        out = []
        for v in range(vl):
            out += O.p2_constraints(local[v * nc:(v + 1) * nc], consts_int)
        return out

    return fn


def kzg_claims_identity(claims, srs_alpha: int, seed: int = 2024, extra=()) -> bool:
    """Every claim (commitment_row, z, v, witness_row) satisfies C - [v]G == [s - z]W; `extra`
    holds (point_row, g_scalar) pairs for equations sum r P == [sum r g] G (commitments against
    their polynomials' values at s).  One random linear combination, one CPU MSM."""
    rng = random.Random(seed)
    idx, pts, sc = {}, [], []

    def add(row, k):
        row = np.ascontiguousarray(row, dtype=np.uint64).reshape(8)
        key = row.tobytes()
        if key not in idx:
            idx[key] = len(pts)
            pts.append(row)
            sc.append(0)
        sc[idx[key]] = (sc[idx[key]] + k) % O.P

    g_coef = 0
    for crow, z, v, wrow in claims:
        r = rng.getrandbits(128)
        add(crow, r)
        add(wrow, -r * (srs_alpha - z))
        g_coef -= r * v
    for prow, gv in extra:
        r = rng.getrandbits(128)
        add(prow, r)
        g_coef -= r * gv
    add(C.g1_generator(), g_coef)
    out = C.g1_msm(np.stack(pts), np.stack([fr_limbs(s) for s in sc]))
    return not np.any(out)


def verify_kzg_proof(proof, constraint_fn, log_n: int, log_qd: int, srs_alpha: int, alpha: int | None = None,
                     zeta: int | None = None, challenger: O.DuplexChallenger | None = None, trace=None,
                     seed: int = 2024, publics=(), pairing: bool = False) -> dict:
    """Verify a prove() output.  With `challenger` (a fresh pyoracle.DuplexChallenger with the
    config's permutation) alpha / zeta are re-derived from the transcript; otherwise the given
    ones are used.  `trace`: the (n, w, 4) host trace, for the check against the trace.
    `pairing`: also run KzgPcs::verify exactly as the reference does -- every opening into ONE
    verify_batch multi-pairing (kzg/src/pcs.rs:337-400, kzg/src/util.rs:245-292) with the pairing
    restatement (oracle/pairing.py; ~0.15 s per Miller loop: small proofs only).  Returns the
    named checks (all must be True)."""
    tc = np.asarray(proof.trace_commit[0], dtype=np.uint64).reshape(-1, 8)
    qc = np.stack([np.asarray(c, dtype=np.uint64).reshape(8) for c in proof.quotient_commit])
    w = tc.shape[0]
    res = {}
    if challenger is not None:
        alpha, zeta = replay_transcript(challenger, log_n, tc, qc, publics)
        res["transcript"] = (proof.alpha, proof.zeta) == (alpha, zeta) if proof.alpha is not None else True
    zeta_next = zeta * O.two_adic_generator(log_n) % O.P
    tr = proof.opened[0]
    local = [fr_int(x) for x in np.asarray(tr.values[0][0]).reshape(-1, 4)]
    nxt = [fr_int(x) for x in np.asarray(tr.values[0][1]).reshape(-1, 4)]
    qo = proof.opened[1]
    qvals = [fr_int(np.asarray(qo.values[c][0]).reshape(-1, 4)[0]) for c in range(len(qo.values))]
    res["ood"] = ood_check(constraint_fn, local, nxt, qvals, alpha, zeta, log_n, log_qd)

    claims = []
    for p, z in enumerate((zeta, zeta_next)):
        vals = np.asarray(tr.values[0][p]).reshape(-1, 4)
        wits = np.asarray(tr.witnesses[0][p]).reshape(-1, 8)
        for c in range(w):
            claims.append((tc[c], z, fr_int(vals[c]), wits[c]))
    for c in range(len(qo.values)):
        claims.append((qc[c], zeta, qvals[c], np.asarray(qo.witnesses[c][0]).reshape(-1, 8)[0]))
    extra = []
    if trace is not None:
        t = np.ascontiguousarray(trace, dtype=np.uint64)
        ev = C.bary_eval_cols(t, np.stack([fr_limbs(zeta), fr_limbs(zeta_next), fr_limbs(srs_alpha)]))
        res["opened_vs_trace"] = bool(np.array_equal(ev[0], np.asarray(tr.values[0][0]).reshape(-1, 4))
                                      and np.array_equal(ev[1], np.asarray(tr.values[0][1]).reshape(-1, 4)))
        extra = [(tc[c], fr_int(ev[2][c])) for c in range(w)]
    res["kzg"] = kzg_claims_identity(claims, srs_alpha, seed, extra)
    if pairing:
        from . import pairing as E

        def pt(row):
            return O.g1_from_bytes(np.ascontiguousarray(row, dtype=np.uint64).reshape(8).tobytes())

        openings = [(pt(c), pt(wr), v, z) for c, z, v, wr in claims]
        res["kzg_pairing"] = E.verify_batch(openings, E.g2_alpha(srs_alpha))
    return res


def proof_from_oracle(d: dict):
    """prove_oracle.prove's dict in the prove() output shape verify_kzg_proof reads."""
    from types import SimpleNamespace

    tv, tw = d["trace_open"]
    opened = [SimpleNamespace(values=[[tv[0], tv[1]]], witnesses=[[tw[0], tw[1]]]),
              SimpleNamespace(values=[[qo[0][0]] for qo in d["quotient_open"]],
                              witnesses=[[qo[1][0]] for qo in d["quotient_open"]])]
    return SimpleNamespace(trace_commit=[d["trace_commit"]], quotient_commit=list(d["quotient_commit"]),
                           opened=opened, alpha=d.get("alpha"), zeta=d.get("zeta"))
