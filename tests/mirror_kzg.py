"""TEST-ONLY Python mirror of p3-kzg's KzgPcs over the C ABI, with every matrix device-resident
(the product is the C++ KzgPcs in plonky3_eon_amd/host/pcs.cpp; this one cross-checks it).

Reference: ``KzgPcs`` (kzg/src/pcs.rs:143-402) implementing ``Pcs<Fr, Challenger>``
(commit/src/pcs.rs:21-187) over ``TwoAdicMultiplicativeCoset`` domains (commit/src/domain.rs).

* ``commit``                     -- coset_idft_batch of each matrix (pcs.rs:242) and one KZG
                                    commitment (MSM over the SRS g1_powers) per column
                                    (pcs.rs:244-251), as one batched device MSM.
* ``get_evaluations_on_domain``  -- pcs.rs:267-287 evaluates every column's coefficients at
                                    every point by Horner; the same values come from one coset
                                    DFT of the zero-padded coefficients.
* ``commit_quotient``            -- commit/src/pcs.rs:82-101: split_evals / split_domains
                                    (domain.rs:174-221), then commit.
* ``open``                       -- pcs.rs:289-335: per (matrix, point) every column's value and
                                    the commitment of its synthetic-division quotient, computed as
                                    the MSM of the column's own coefficients against the opening
                                    bases H(z) (eon_kzg_opening_bases_create) over the digits
                                    sorted at commit time.  EON_KZG_OPEN=quotient keeps the
                                    reference's route (quotients, then their commitments).

Commitments / witnesses are (width, 8) u64 arrays of affine G1 points (x, y Fq Montgomery).
"""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from plonky3_eon_amd import _lib
from plonky3_eon_amd.dft import Context, Radix2Dit, default_context
from plonky3_eon_amd.field import FR_MODULUS, fr_mont, fr_to_abi, fr_unmont  # noqa: F401
from plonky3_eon_amd.msm import MsmBases, srs_powers
from plonky3_eon_amd.proof import Opened

GENERATOR = 5
_TWO_ADIC_GENERATOR_MONT = (0x636E735580D13D9C, 0xA22BF3742445FFD6, 0x56452AC01EB203D8, 0x1860EF942963F9E7)


def two_adic_generator(bits: int) -> int:
    """bn254/src/field.rs:567-573 (host-side domain bookkeeping)."""
    g = fr_unmont(sum(x << (64 * i) for i, x in enumerate(_TWO_ADIC_GENERATOR_MONT)))
    for _ in range(bits, 28):
        g = g * g % FR_MODULUS
    return g


@dataclass(frozen=True)
class Domain:
    """TwoAdicMultiplicativeCoset (field/src/coset.rs): shift * <w_(2^log_size)>."""

    shift: int
    log_size: int

    @property
    def size(self):
        return 1 << self.log_size

    def generator(self):
        return two_adic_generator(self.log_size)

    def next_point(self, x: int) -> int:
        """commit/src/domain.rs:115-117."""
        return x * self.generator() % FR_MODULUS

    def create_disjoint_domain(self, min_size: int) -> "Domain":
        """commit/src/domain.rs:155-168."""
        return Domain(self.shift * GENERATOR % FR_MODULUS, max(0, (min_size - 1).bit_length()))

    def split_domains(self, num_chunks: int):
        """commit/src/domain.rs:174-186."""
        lc = num_chunks.bit_length() - 1
        g = self.generator()
        return [Domain(self.shift * pow(g, i, FR_MODULUS) % FR_MODULUS, self.log_size - lc) for i in range(num_chunks)]


@dataclass
class MatrixProverData:
    """kzg/src/pcs.rs:46-63: the committed evaluations and their coefficients (device)."""

    domain: Domain
    evals: object
    coeffs: object
    prepared: object = None  # msm.PreparedScalars of coeffs (the commitment's sorted digits)


class GpuKzgPcs:
    def __init__(self, max_degree: int, alpha: int, ctx: Context | None = None):
        """KzgPcs::new(max_degree, alpha) with the test SRS init_srs_unsafe
        (kzg/src/params.rs:123-139); the g1_powers stay on device as fixed-base MSM bases."""
        self.ctx = ctx or default_context(0)
        self.max_degree = max_degree
        self.bases = MsmBases(srs_powers(max_degree + 1, alpha, self.ctx), self.ctx, precompute=True)
        self.dft = Radix2Dit(self.ctx)
        self.keep_digits = os.environ.get("EON_KZG_OPEN") != "quotient"

    # -- Pcs surface -----------------------------------------------------------------------------
    def natural_domain_for_degree(self, degree: int) -> Domain:
        return Domain(1, (degree - 1).bit_length() if degree > 1 else 0)

    def ensure_supported(self, degree: int):
        """kzg/src/params.rs:164-173 (KzgError::DegreeTooLarge)."""
        if degree > self.max_degree:
            raise _lib.EonError(_lib.EON_E_DEGREE_TOO_LARGE, f"degree {degree} > max {self.max_degree}")

    def commit(self, evaluations):
        commitments, data = [], []
        for domain, evals in evaluations:
            h = int(evals.shape[0])
            if h != domain.size:
                raise _lib.EonError(_lib.EON_E_SHAPE, "evaluation height must match domain size")
            self.ensure_supported(max(h - 1, 0))
            coeffs = self.dft.coset_idft_batch(evals, domain.shift)
            prepared = None
            if self.keep_digits:
                cm, prepared = self.bases.prepare_columns(coeffs)
            else:
                cm = self.bases.msm_columns(coeffs)
            commitments.append(cm)
            data.append(MatrixProverData(domain, evals, coeffs, prepared))
        return commitments, data

    def get_evaluations_on_domain(self, prover_data, idx: int, domain: Domain):
        m = prover_data[idx]
        if m.domain == domain:
            return m.evals
        if domain.log_size < m.domain.log_size:
            raise _lib.EonError(_lib.EON_E_SHAPE, "evaluation domain smaller than the committed domain")
        # the reference evaluates the committed coefficients at every point by Horner; the same
        # values are the coset DFT of the zero-padded coefficients (one forward network)
        return self.dft.coset_dft_padded_batch(m.coeffs, domain.log_size - m.domain.log_size, domain.shift)

    def commit_quotient(self, quotient_domain: Domain, quotient_evals, num_chunks: int):
        """commit/src/pcs.rs:82-101; chunk c holds rows {i * num_chunks + c} (domain.rs:188-221)."""
        q = quotient_evals.reshape(quotient_domain.size // num_chunks, num_chunks, 4)
        chunks = [q[:, c:c + 1, :].contiguous() for c in range(num_chunks)]
        return self.commit(list(zip(quotient_domain.split_domains(num_chunks), chunks)))

    def open(self, rounds):
        """rounds: [(prover_data, points_per_matrix)] -> (opened values, witnesses) per round.

        pcs.rs:289-335 commits, per (matrix, point z, column c), the quotient of c by (X - z).
        That commitment equals sum_j c_j H_j(z) with H_j(z) = sum_{i<j} z^(j-1-i) G_i, so every
        point's witnesses are one run over the digits sorted when the matrix was committed."""
        import torch

        for prover_data, _ in rounds:
            if any(m.prepared is None for m in prover_data):
                return self.open_quotients(rounds)
        bases_at = {}  # (height, point) -> opening bases, shared across matrices
        todo = {}
        for prover_data, points_per_matrix in rounds:
            for m, points in zip(prover_data, points_per_matrix):
                n = int(m.coeffs.shape[0])
                for z in points:
                    if (n, z) not in bases_at and z not in todo.setdefault(n, []):
                        todo[n].append(z)
        for n, zs in todo.items():  # each height's points in one call
            for z, b in zip(zs, self.bases.opening_bases_many(n, zs)):
                bases_at[(n, z)] = b
        out = []
        for prover_data, points_per_matrix in rounds:
            if len(prover_data) != len(points_per_matrix):
                raise _lib.EonError(_lib.EON_E_SHAPE, "one point list per matrix")
            o = Opened(values=[[None] * len(p) for p in points_per_matrix],
                       witnesses=[[None] * len(p) for p in points_per_matrix])
            for mi, (m, points) in enumerate(zip(prover_data, points_per_matrix)):
                n, w = int(m.coeffs.shape[0]), int(m.coeffs.shape[1])
                # every point's values in one pass over the coefficients (eon_eval_columns_dev)
                v = torch.empty((max(len(points), 1), w, 4), dtype=torch.int64, device=m.coeffs.device)
                zs = (_lib.eon_fr * max(len(points), 1))(*[fr_to_abi(z) for z in points])
                self.ctx.set_stream(torch.cuda.current_stream(m.coeffs.device).cuda_stream)
                self.ctx.check(self.ctx.lib.eon_eval_columns_dev(
                    self.ctx.handle, ctypes.c_void_p(m.coeffs.data_ptr()), n, w, zs, len(points),
                    ctypes.c_void_p(v.data_ptr())))
                vh = v.cpu().numpy().view(np.uint64)
                hb = []
                for pi, z in enumerate(points):
                    o.values[mi][pi] = vh[pi]
                    hb.append(bases_at[(n, z)])
                wits = m.prepared.msm(hb)
                for pi in range(len(points)):
                    o.witnesses[mi][pi] = wits[pi]
            out.append(o)
        for b in bases_at.values():
            b.close()
        return out

    def open_quotients(self, rounds):
        """open by the reference's route: pcs.rs:289-335 computes, per (matrix, point), every
        column's synthetic-division quotient and commits each one.  All quotients of one height share the SRS prefix, so they are
        gathered into one matrix and committed by ONE batched column MSM (one pipeline fill and
        drain instead of one per (matrix, point))."""
        import torch

        jobs = []  # (round, matrix, point index, height n, width w)
        for ri, (prover_data, points_per_matrix) in enumerate(rounds):
            if len(prover_data) != len(points_per_matrix):
                raise _lib.EonError(_lib.EON_E_SHAPE, "one point list per matrix")
            for mi, (m, points) in enumerate(zip(prover_data, points_per_matrix)):
                for pi in range(len(points)):
                    jobs.append((ri, mi, pi, int(m.coeffs.shape[0]), int(m.coeffs.shape[1])))
        # one witness matrix per quotient height n - 1, columns in job order
        groups = {}
        for j in jobs:
            groups.setdefault(j[3], []).append(j)
        mats, col0 = {}, {}
        for n, js in groups.items():
            dev = rounds[js[0][0]][0][js[0][1]].coeffs.device
            mats[n] = torch.empty((max(n - 1, 1), sum(j[4] for j in js), 4), dtype=torch.int64, device=dev)
            c = 0
            for j in js:
                col0[j[:3]] = c
                c += j[4]
        out = [Opened(values=[[None] * len(pts) for pts in p], witnesses=[[None] * len(pts) for pts in p])
               for _, p in rounds]
        for ri, mi, pi, n, w in jobs:
            m = rounds[ri][0][mi]
            z = rounds[ri][1][mi][pi]
            quo = torch.empty((max(n - 1, 1), w, 4), dtype=torch.int64, device=m.coeffs.device)
            v = torch.empty((w, 4), dtype=torch.int64, device=m.coeffs.device)
            pz = fr_to_abi(z)
            self.ctx.set_stream(torch.cuda.current_stream(m.coeffs.device).cuda_stream)
            self.ctx.check(self.ctx.lib.eon_quotient_and_eval_columns_dev(
                self.ctx.handle, ctypes.c_void_p(m.coeffs.data_ptr()), n, w, ctypes.byref(pz),
                ctypes.c_void_p(quo.data_ptr()), ctypes.c_void_p(v.data_ptr())))
            c = col0[(ri, mi, pi)]
            mats[n][:, c:c + w] = quo
            out[ri].values[mi][pi] = v.cpu().numpy().view(np.uint64)
        for n, js in groups.items():
            wits = self.bases.msm_columns(mats[n][:n - 1])
            for ri, mi, pi, _, w in js:
                c = col0[(ri, mi, pi)]
                out[ri].witnesses[mi][pi] = wits[c:c + w]
        return out
