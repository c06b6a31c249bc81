"""Host-side mirror of the reference's G1 MSM surface over the C ABI (include/eon.h).

* ``multi_exp(points, scalars)``  -- G1::multi_exp (bn254/src/curve.rs:158-179): one-shot.
* ``MsmBases``                    -- device-resident bases reused across MSMs, as KzgPcs reuses
                                     the SRS g1_powers for every commit_column
                                     (kzg/src/util.rs:37-40); ``precompute=True`` builds the
                                     fixed-base window table (EON_MSM_PRECOMPUTE).

Points are numpy uint64 arrays (..., 8): x[4], y[4] as Fq Montgomery limbs, identity = zeros.
Scalars are Fr Montgomery limbs (n, 4): numpy (host) or a torch CUDA tensor (device-resident).
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .dft import Context, default_context, _is_torch


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class MsmBases:
    def __init__(self, bases: np.ndarray, ctx: Context | None = None, precompute: bool = True):
        self.ctx = ctx or default_context(0)
        b = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, 8)
        h = ctypes.c_void_p()
        flags = _lib.EON_MSM_PRECOMPUTE if precompute else 0
        self.ctx.check(self.ctx.lib.eon_msm_bases_create(self.ctx.handle, _p(b), b.shape[0], flags,
                                                          ctypes.byref(h)))
        self._h = h
        self.n = b.shape[0]

    def msm(self, scalars) -> np.ndarray:
        out = np.zeros(8, dtype=np.uint64)
        lib, ctx = self.ctx.lib, self.ctx
        if _is_torch(scalars):
            import torch

            s = scalars.contiguous()
            ctx.set_stream(torch.cuda.current_stream(s.device).cuda_stream)
            ctx.check(lib.eon_msm_g1_dev(ctx.handle, self._h, ctypes.c_void_p(s.data_ptr()), s.shape[0],
                                         _p(out)))
        else:
            s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
            ctx.check(lib.eon_msm_g1(ctx.handle, self._h, _p(s), s.shape[0], _p(out)))
        return out

    def msm_columns(self, mat) -> np.ndarray:
        """One MSM per column of a (rows, width, 4) Fr matrix -> (width, 8) affine points."""
        lib, ctx = self.ctx.lib, self.ctx
        rows, width = int(mat.shape[0]), int(mat.shape[1])
        out = np.zeros((width, 8), dtype=np.uint64)
        if _is_torch(mat):
            import torch

            m = mat.contiguous()
            ctx.set_stream(torch.cuda.current_stream(m.device).cuda_stream)
            ctx.check(lib.eon_msm_g1_columns_dev(ctx.handle, self._h, ctypes.c_void_p(m.data_ptr()), rows, width,
                                                 _p(out)))
        else:
            m = np.ascontiguousarray(mat, dtype=np.uint64)
            ctx.check(lib.eon_msm_g1_columns(ctx.handle, self._h, _p(m), rows, width, _p(out)))
        return out

    def close(self):
        if getattr(self, "_h", None):
            self.ctx.lib.eon_msm_bases_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def srs_powers(n: int, alpha, ctx: Context | None = None) -> np.ndarray:
    """init_srs_unsafe g1_powers (kzg/src/params.rs:123-139) computed on device: (n, 8)."""
    from .field import fr_to_abi

    ctx = ctx or default_context(0)
    out = np.zeros((n, 8), dtype=np.uint64)
    a = fr_to_abi(alpha)
    ctx.check(ctx.lib.eon_g1_srs_powers(ctx.handle, ctypes.byref(a), n, _p(out)))
    return out


def multi_exp(points, scalars, ctx: Context | None = None) -> np.ndarray:
    """G1::multi_exp: panics (EonError) on a length mismatch, identity for empty input."""
    ctx = ctx or default_context(0)
    p = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, 8)
    s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
    if p.shape[0] != s.shape[0]:
        raise _lib.EonError(_lib.EON_E_SHAPE, "points and scalars must have the same length")
    out = np.zeros(8, dtype=np.uint64)
    ctx.check(ctx.lib.eon_g1_multi_exp(ctx.handle, _p(p), _p(s), p.shape[0], _p(out)))
    return out
