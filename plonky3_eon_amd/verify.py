"""Host-side mirror of the reference's KZG verifier pairings over the C ABI (include/eon.h, N4).

* ``g2_mul(k)``          -- G2::generator().mul_scalar(k); KzgParams.g2_alpha = [alpha] G2
                            (kzg/src/params.rs:123-139).
* ``multi_pairing``      -- multi_pairing (bn254/src/curve.rs:439-452): prod e(P_i, Q_i) in Gt.
* ``verify_batch``       -- verify_batch / verify_single (kzg/src/util.rs:150-168, 245-292):
                            True for Ok(()), False for Err(KzgError::ProofShapeMismatch).

Layouts (numpy uint64): G1 affine (8,) = x[4], y[4]; G2 affine (16,) = x.c0, x.c1, y.c0, y.c1
(Fq Montgomery limbs; identity = zeros); Gt (12, 4) = the Fq12 tower coefficients c0.c0.c0,
c0.c0.c1, c0.c1.c0, ..., c1.c2.c1; Fr values (4,) Montgomery limbs.
"""

from __future__ import annotations

import ctypes

import numpy as np

from .dft import Context, default_context
from .field import fr_to_abi


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def g2_mul(k, base=None, ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or default_context(0)
    out = np.zeros(16, dtype=np.uint64)
    kk = fr_to_abi(k)
    b = None if base is None else np.ascontiguousarray(base, dtype=np.uint64).reshape(16)
    ctx.check(ctx.lib.eon_g2_mul(ctx.handle, None if b is None else _p(b), ctypes.byref(kk), _p(out)))
    return out


def multi_pairing(g1_points, g2_points, ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or default_context(0)
    p = np.ascontiguousarray(g1_points, dtype=np.uint64).reshape(-1, 8)
    q = np.ascontiguousarray(g2_points, dtype=np.uint64).reshape(-1, 16)
    if p.shape[0] != q.shape[0]:
        from ._lib import EON_E_SHAPE, EonError

        raise EonError(EON_E_SHAPE, "one G2 point per G1 point")
    out = np.zeros((12, 4), dtype=np.uint64)
    ctx.check(ctx.lib.eon_multi_pairing(ctx.handle, _p(p), _p(q), p.shape[0], _p(out)))
    return out


def pairing(g1_point, g2_point, ctx: Context | None = None) -> np.ndarray:
    return multi_pairing(np.reshape(g1_point, (1, 8)), np.reshape(g2_point, (1, 16)), ctx)


def verify_batch(commitments, witnesses, values, points, g2_alpha, ctx: Context | None = None) -> bool:
    """openings i: (commitment (8,), witness (8,), value (4,) Fr limbs, point (4,) Fr limbs)."""
    ctx = ctx or default_context(0)
    c = np.ascontiguousarray(commitments, dtype=np.uint64).reshape(-1, 8)
    w = np.ascontiguousarray(witnesses, dtype=np.uint64).reshape(-1, 8)
    v = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1, 4)
    z = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, 4)
    n = c.shape[0]
    if not (w.shape[0] == v.shape[0] == z.shape[0] == n):
        from ._lib import EON_E_SHAPE, EonError

        raise EonError(EON_E_SHAPE, "one witness, value and point per commitment")
    g = np.ascontiguousarray(g2_alpha, dtype=np.uint64).reshape(16)
    ok = ctypes.c_int(0)
    ctx.check(ctx.lib.eon_kzg_verify_batch(ctx.handle, _p(c), _p(w), _p(v), _p(z), n, _p(g), ctypes.byref(ok)))
    return bool(ok.value)
