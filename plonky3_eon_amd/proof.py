"""The proof the native driver returns (libeonprove.so, native.prove_native), in the reference's
shape: eon-uni-stark/src/proof.rs:19-44 (commitments, opened values, opening proof, degree bits)
with KzgPcs's per-column witnesses (kzg/src/pcs.rs:289-335)."""

from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class Opened:
    values: list = field(default_factory=list)     # [matrix][point] -> (width, 4) u64 Fr
    witnesses: list = field(default_factory=list)  # [matrix][point] -> (width, 8) u64 G1


@dataclass
class Proof:
    """eon-uni-stark/src/proof.rs:19-44 (commitments, opened values, opening proof, degree bits)."""

    trace_commit: object
    quotient_commit: object
    opened: object
    degree_bits: int
    timings_ms: dict = field(default_factory=dict)
    alpha: int | None = None  # the challenges used (canonical ints)
    zeta: int | None = None


def log_quotient_degree(max_constraint_degree: int) -> int:
    """get_log_quotient_degree (eon-uni-stark/src/symbolic_builder.rs:15-43), ZK off."""
    d = max(max_constraint_degree, 2) - 1
    return (d - 1).bit_length()
