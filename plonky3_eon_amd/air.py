"""Host-side mirror of the Poseidon2-AIR and eon-uni-stark's quotient over the C ABI.

* ``Poseidon2Air``      -- Poseidon2Air / VectorizedPoseidon2Air (poseidon2-air/src/air.rs,
                           vectorized.rs) for BN254 (width 3, x^5, one register):
                           ``generate_trace`` (generation.rs) and ``quotient_values``
                           (eon-uni-stark/src/prover.rs:539-709) on device-resident matrices.
* ``selectors_on_coset`` -- commit/src/domain.rs:252-292.

Device matrices are torch CUDA int64 tensors of shape (rows, cols, 4) (Fr Montgomery limbs).
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .dft import Context, default_context
from .field import fr_to_abi


def _dp(t):
    return ctypes.c_void_p(t.data_ptr())


class Poseidon2Air:
    def __init__(self, begin, partial, end, vector_len: int = 1, ctx: Context | None = None):
        """begin/end: (half_full_rounds, 3, 4) u64 limbs; partial: (partial_rounds, 4)."""
        self.ctx = ctx or default_context(0)
        self._b = np.ascontiguousarray(begin, dtype=np.uint64).reshape(-1, 3, 4)
        self._p = np.ascontiguousarray(partial, dtype=np.uint64).reshape(-1, 4)
        self._e = np.ascontiguousarray(end, dtype=np.uint64).reshape(-1, 3, 4)
        k = _lib.eon_poseidon2_constants(self._b.shape[0], self._p.shape[0],
                                         self._b.ctypes.data_as(ctypes.c_void_p),
                                         self._p.ctypes.data_as(ctypes.c_void_p),
                                         self._e.ctypes.data_as(ctypes.c_void_p))
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx.lib.eon_p2air_create(self.ctx.handle, ctypes.byref(k), vector_len, ctypes.byref(h)))
        self._h = h
        self.vector_len = vector_len
        self.width = int(self.ctx.lib.eon_p2air_width(h))
        self.constraints_per_perm = 12 * self._b.shape[0] + 2 * self._p.shape[0]

    @property
    def handle(self):
        return self._h

    def _stream(self, t):
        import torch

        self.ctx.set_stream(torch.cuda.current_stream(t.device).cuda_stream)

    def generate_trace(self, inputs):
        """inputs: (n_perms, 3, 4) device tensor -> (n_perms / VECTOR_LEN, width, 4) trace."""
        import torch

        n = inputs.shape[0]
        out = torch.empty((n // self.vector_len, self.width, 4), dtype=torch.int64, device=inputs.device)
        self._stream(inputs)
        self.ctx.check(self.ctx.lib.eon_p2air_generate_trace_dev(self.ctx.handle, self._h, _dp(inputs.contiguous()),
                                                                 n, _dp(out)))
        return out

    def quotient_values(self, lde, log_n: int, log_qd: int, alpha):
        """quotient_values on the trace's LDE over GENERATOR * K (natural order)."""
        import torch

        q = 1 << (log_n + log_qd)
        out = torch.empty((q, 4), dtype=torch.int64, device=lde.device)
        a = fr_to_abi(alpha)
        self._stream(lde)
        self.ctx.check(self.ctx.lib.eon_p2air_quotient_values_dev(self.ctx.handle, self._h, _dp(lde.contiguous()),
                                                                  log_n, log_qd, ctypes.byref(a), _dp(out)))
        return out

    def close(self):
        if getattr(self, "_h", None):
            self.ctx.lib.eon_p2air_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def selectors_on_coset(log_n: int, log_q: int, shift, device=0, ctx: Context | None = None):
    """-> (4, 2^log_q, 4) device tensor: is_first_row, is_last_row, is_transition, inv_vanishing."""
    import torch

    ctx = ctx or default_context(device)
    out = torch.empty((4, 1 << log_q, 4), dtype=torch.int64, device=f"cuda:{device}")
    s = fr_to_abi(shift)
    ctx.set_stream(torch.cuda.current_stream(out.device).cuda_stream)
    ctx.check(ctx.lib.eon_selectors_on_coset_dev(ctx.handle, log_n, log_q, ctypes.byref(s), _dp(out)))
    return out
