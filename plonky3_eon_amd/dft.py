"""Host-side mirror of p3-dft's TwoAdicSubgroupDft<Fr> over the C ABI (include/eon.h).

Reference interface: dft/src/traits.rs:27-249.  Two implementations mirror the reference's:

* ``Radix2Dit``          -- natural-order RowMajorMatrix results (dft/src/radix_2_dit.rs:61-77),
                            the DFT KzgPcs uses (kzg/src/pcs.rs:148).
* ``Radix2DitParallel``  -- ``dft_batch`` / ``coset_dft_batch`` / ``lde_batch`` /
                            ``coset_lde_batch`` return a BitReversedMatrixView whose storage is
                            bit-reversed (dft/src/radix_2_dit_parallel.rs:146,165,227); here that
                            is a ``BitReversedMatrix`` holding the storage.

Matrices are Fr arrays of shape (height, width, 4) of little-endian u64 Montgomery limbs -- the
in-memory layout of RowMajorMatrix<Fr> -- either numpy (host; the call is synchronous) or a
torch CUDA tensor (device-resident; the call is enqueued on torch's current stream).  Errors are
raised as EonError where the reference panics (non-power-of-two heights, TWO_ADICITY overflow).
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .field import fr_to_abi



class Context:
    """An eon_ctx on one device (eon_ctx_create / eon_ctx_destroy)."""

    def __init__(self, device: int = 0):
        lib = _lib.load()
        h = ctypes.c_void_p()
        rc = lib.eon_ctx_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise _lib.EonError(rc, f"eon_ctx_create({device}) failed")
        self._h = h
        self.device = device
        self.lib = lib

    @property
    def handle(self):
        return self._h

    def check(self, rc: int):
        if rc != 0:
            raise _lib.EonError(rc, self.lib.eon_last_error(self._h).decode())

    def set_stream(self, stream_ptr: int | None):
        self.check(self.lib.eon_ctx_set_stream(self._h, ctypes.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        self.check(self.lib.eon_ctx_synchronize(self._h))

    def profile(self, enable: bool = True):
        """Start (clearing) or stop per-launch HIP-event timing (eon_ctx_profile)."""
        self.check(self.lib.eon_ctx_profile(self._h, 1 if enable else 0))

    def set_serial(self, serial: bool = True):
        """Serial mode (eon_ctx_set_serial): every kernel on the context stream, none on the MSM /
        opening side streams -- isolated launch durations for profiles; same results."""
        self.check(self.lib.eon_ctx_set_serial(self._h, 1 if serial else 0))

    def profile_report(self) -> dict:
        import json

        buf = ctypes.create_string_buffer(1 << 16)
        self.check(self.lib.eon_ctx_profile_report(self._h, buf, len(buf)))
        return json.loads(buf.value.decode())

    def trim(self):
        """Give the context's cached idle device buffers back (eon_ctx_trim)."""
        self.check(self.lib.eon_ctx_trim(self._h))

    def clock_probe(self, launches: int = 160, iters: int = 1024) -> dict:
        """Diagnostic (eon_diag_clock_probe): the in-kernel shader clock under a radix-2^29
        product chain and the product rate at that clock, on this context's stream."""
        r = _lib.eon_clock_probe()
        self.check(self.lib.eon_diag_clock_probe(self._h, int(launches), int(iters), ctypes.byref(r)))
        return {k: getattr(r, k) for k, _ in r._fields_}

    def prod_asm_check(self, n: int = 1 << 20, seed: int = 1) -> list:
        """Diagnostic (eon_diag_prod_asm_check): mismatching cases of the whole-product asm
        statements against the column-block products (mul, sqr, sum2), n random operands each."""
        r = (ctypes.c_uint32 * 3)()
        self.check(self.lib.eon_diag_prod_asm_check(self._h, int(n), int(seed), r))
        return list(r)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.eon_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: dict[int, Context] = {}


def default_context(device: int = 0) -> Context:
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _shape(mat):
    if mat.ndim != 3 or mat.shape[2] != 4:
        raise ValueError("Fr matrix must have shape (height, width, 4) of u64 limbs")
    return int(mat.shape[0]), int(mat.shape[1])


class BitReversedMatrix:
    """BitReversedMatrixView<RowMajorMatrix<Fr>>: `storage` row reverse_bits(k) is logical row k
    (matrix/src/bitrev.rs)."""

    def __init__(self, storage):
        self.storage = storage

    def height(self):
        return int(self.storage.shape[0])

    def width(self):
        return int(self.storage.shape[1])

    def to_row_major_matrix(self):
        h = self.height()
        lg = h.bit_length() - 1
        idx = np.array([int(format(i, f"0{lg}b")[::-1], 2) if lg else 0 for i in range(h)])
        if _is_torch(self.storage):
            import torch

            return self.storage[torch.as_tensor(idx, device=self.storage.device)]
        return self.storage[idx]


class _GpuDft:
    out_order = _lib.EON_ORDER_NATURAL

    def __init__(self, ctx: Context | None = None):
        self.ctx = ctx

    # -- plumbing ----------------------------------------------------------------------------
    def _ctx(self, mat) -> Context:
        if self.ctx is not None:
            return self.ctx
        dev = mat.device.index if _is_torch(mat) else 0
        return default_context(dev or 0)

    def _call(self, name, mat, out_rows_factor, *extra):
        h, w = _shape(mat)
        ctx = self._ctx(mat)
        if _is_torch(mat):
            import torch

            if not mat.is_cuda:
                raise ValueError("torch tensors must be CUDA (device-resident) tensors")
            src = mat.contiguous()
            out = torch.empty((h * out_rows_factor, w, 4), dtype=src.dtype, device=src.device)
            ctx.set_stream(torch.cuda.current_stream(src.device).cuda_stream)
            fn = getattr(ctx.lib, name + "_dev")
            ctx.check(fn(ctx.handle, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                         h, w, *extra))
            return out
        src = np.ascontiguousarray(mat, dtype=np.uint64)
        out = np.empty((h * out_rows_factor, w, 4), dtype=np.uint64)
        fn = getattr(ctx.lib, name)
        ctx.check(fn(ctx.handle, src.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p),
                     h, w, *extra))
        return out

    def _wrap(self, out):
        return BitReversedMatrix(out) if self.out_order == _lib.EON_ORDER_BITREV else out

    # -- TwoAdicSubgroupDft<Fr> (dft/src/traits.rs) -----------------------------------------
    def dft_batch(self, mat):
        return self._wrap(self._call("eon_dft_batch", mat, 1, self.out_order))

    def idft_batch(self, mat):
        return self._call("eon_idft_batch", mat, 1)

    def coset_dft_batch(self, mat, shift):
        s = fr_to_abi(shift)
        return self._wrap(self._call("eon_coset_dft_batch", mat, 1, ctypes.byref(s), self.out_order))

    def coset_idft_batch(self, mat, shift):
        s = fr_to_abi(shift)
        return self._call("eon_coset_idft_batch", mat, 1, ctypes.byref(s))

    def lde_batch(self, mat, added_bits: int):
        return self._wrap(self._call("eon_coset_lde_batch", mat, 1 << added_bits, added_bits, None,
                                     self.out_order))

    def coset_lde_batch(self, mat, added_bits: int, shift):
        s = fr_to_abi(shift)
        return self._wrap(self._call("eon_coset_lde_batch", mat, 1 << added_bits, added_bits,
                                     ctypes.byref(s), self.out_order))

    def coset_dft_padded_batch(self, coeffs, added_bits: int, shift):
        """coset_dft_batch of `coeffs` zero-padded to height << added_bits (coset_lde_batch minus
        its idft; dft/src/traits.rs:226-249)."""
        s = fr_to_abi(shift)
        return self._wrap(self._call("eon_coset_dft_padded_batch", coeffs, 1 << added_bits, added_bits,
                                     ctypes.byref(s), self.out_order))

    # single-column conveniences (dft/src/traits.rs:46,70,100,131,168,207)
    def dft(self, vec):
        return _col(self.dft_batch(_as_col(vec)))

    def idft(self, vec):
        return _col(self.idft_batch(_as_col(vec)))

    def coset_dft(self, vec, shift):
        return _col(self.coset_dft_batch(_as_col(vec), shift))

    def coset_idft(self, vec, shift):
        return _col(self.coset_idft_batch(_as_col(vec), shift))

    def lde(self, vec, added_bits):
        return _col(self.lde_batch(_as_col(vec), added_bits))

    def coset_lde(self, vec, added_bits, shift):
        return _col(self.coset_lde_batch(_as_col(vec), added_bits, shift))


def _as_col(vec):
    return vec.reshape(vec.shape[0], 1, 4)


def _col(m):
    if isinstance(m, BitReversedMatrix):
        m = m.to_row_major_matrix()
    return m.reshape(m.shape[0], 4)


class Radix2Dit(_GpuDft):
    """Natural-order results, as p3_dft::Radix2Dit (dft/src/radix_2_dit.rs)."""

    out_order = _lib.EON_ORDER_NATURAL


class Radix2DitParallel(_GpuDft):
    """Bit-reversed-storage results, as p3_dft::Radix2DitParallel
    (dft/src/radix_2_dit_parallel.rs:146-228)."""

    out_order = _lib.EON_ORDER_BITREV
