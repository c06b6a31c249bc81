"""Host-side mirror of the reference's G1 MSM surface over the C ABI (include/eon.h).

* ``multi_exp(points, scalars)``  -- G1::multi_exp (bn254/src/curve.rs:158-179): one-shot.
* ``MsmBases``                    -- device-resident bases reused across MSMs, as KzgPcs reuses
                                     the SRS g1_powers for every commit_column
                                     (kzg/src/util.rs:37-40); ``precompute=True`` builds the
                                     fixed-base window table (EON_MSM_PRECOMPUTE).
* ``MsmBases.prepare_columns``    -- the column MSMs of a matrix that also keep its sorted
                                     bucket digits (``PreparedScalars``) for later MSMs of the
                                     same columns against other bases of that layout.
* ``MsmBases.opening_bases(n, z)``-- H_j(z) = sum_{i<j} z^(j-1-i) G_i: sum_j c_j H_j(z) is the
                                     KZG witness of quotient_and_eval(c, z) (kzg/src/pcs.rs:305-316).

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

    @classmethod
    def _from_handle(cls, h, n: int, ctx: Context) -> "MsmBases":
        b = cls.__new__(cls)
        b.ctx, b._h, b.n = ctx, h, n
        return b

    def prepare_columns(self, mat, want_commitments: bool = True):
        """Column MSMs of a device (rows, width, 4) Fr matrix (as msm_columns) plus the
        ``PreparedScalars`` that keep its sorted digits -> (commitments (width, 8) | None, prep)."""
        import torch

        lib, ctx = self.ctx.lib, self.ctx
        m = mat.contiguous()
        rows, width = int(m.shape[0]), int(m.shape[1])
        out = np.zeros((width, 8), dtype=np.uint64)
        ctx.set_stream(torch.cuda.current_stream(m.device).cuda_stream)
        h = ctypes.c_void_p()
        ctx.check(lib.eon_msm_g1_columns_prepare_dev(ctx.handle, self._h, ctypes.c_void_p(m.data_ptr()), rows,
                                                     width, _p(out) if want_commitments else None,
                                                     ctypes.byref(h)))
        return (out if want_commitments else None), PreparedScalars(h, rows, width, ctx)

    def opening_bases(self, n: int, point) -> "MsmBases":
        """KZG opening bases for `point` (Fr limbs or int, Montgomery via fr_to_abi) over the
        first n - 1 bases (eon_kzg_opening_bases_create)."""
        from .field import fr_to_abi

        h = ctypes.c_void_p()
        z = fr_to_abi(point)
        self.ctx.check(self.ctx.lib.eon_kzg_opening_bases_create(self.ctx.handle, self._h, n, ctypes.byref(z),
                                                                 ctypes.byref(h)))
        return MsmBases._from_handle(h, n, self.ctx)

    def opening_bases_many(self, n: int, points) -> list:
        """opening_bases for several points at once (eon_kzg_opening_bases_create_many)."""
        from .field import fr_to_abi

        k = len(points)
        zs = (_lib.eon_fr * max(k, 1))(*[fr_to_abi(p) for p in points])
        hs = (ctypes.c_void_p * max(k, 1))()
        self.ctx.check(self.ctx.lib.eon_kzg_opening_bases_create_many(self.ctx.handle, self._h, n, zs, k, hs))
        return [MsmBases._from_handle(ctypes.c_void_p(hs[t]), n, self.ctx) for t in range(k)]

    def close(self):
        if getattr(self, "_h", None):
            self.ctx.lib.eon_msm_bases_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PreparedScalars:
    """Sorted bucket digits of a scalar matrix kept on device (eon_msm_scalars)."""

    def __init__(self, h, rows: int, width: int, ctx: Context):
        self._h, self.rows, self.width, self.ctx = h, rows, width, ctx

    def msm(self, bases_list) -> np.ndarray:
        """(len(bases_list), width, 8): column j of the prepared matrix against each bases."""
        arr = (ctypes.c_void_p * max(len(bases_list), 1))(*[b._h for b in bases_list])
        out = np.zeros((len(bases_list), self.width, 8), dtype=np.uint64)
        self.ctx.check(self.ctx.lib.eon_msm_g1_columns_prepared(self.ctx.handle, arr, len(bases_list), self._h,
                                                                _p(out)))
        return out

    def close(self):
        if getattr(self, "_h", None):
            self.ctx.lib.eon_msm_scalars_destroy(self._h)
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
