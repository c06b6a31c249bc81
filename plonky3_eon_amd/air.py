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

    # --- the same AIR through the generic path: EonAir::eval on a symbolic builder -------------
    def num_public_values(self) -> int:
        return 0

    def eval(self, builder):
        """Poseidon2Air::eval (poseidon2-air/src/air.rs:108-166) on the symbolic builder, lanes in
        order (vectorized.rs:259-274): the initial external layer, full rounds (eval_full_round
        :200-221: add round constant, eval_sbox :253-288 with one committed x^3 register, external
        layer, assert_eq(state, post) then state = post), partial rounds (eval_partial_round
        :224-243: only state[0] through the S-box, internal layer).  The export column is
        unconstrained."""
        from .field import limbs_to_ints
        from .symbolic import SymbolicExpression

        E = SymbolicExpression.lift
        hf, pr = self._b.shape[0], self._p.shape[0]
        begin = [limbs_to_ints(self._b[r]) for r in range(hf)]
        partial = limbs_to_ints(self._p)
        end = [limbs_to_ints(self._e[r]) for r in range(hf)]
        nc = 4 + 12 * hf + 2 * pr
        local = builder.main()[0]

        def ext(s):  # mds_light width 3 (poseidon2/src/external.rs:128-133)
            t = s[0] + s[1] + s[2]
            return [s[0] + t, s[1] + t, s[2] + t]

        def internal(s):  # [2,1,1;1,2,1;1,1,3] (bn254/src/poseidon2.rs:55-63)
            t = s[0] + s[1] + s[2]
            return [s[0] + t, s[1] + t, s[2].double() + t]

        def sbox(x, x3):  # eval_sbox, degree 5 with one register: x3 = x^3, out = x3 * x^2
            x2 = x.square()
            builder.assert_eq(x3, x2 * x)
            return x3 * x2

        for v in range(self.vector_len):
            row = local[v * nc:(v + 1) * nc]
            s = ext([E(row[1]), E(row[2]), E(row[3])])
            k = 4

            def full(s, rc, k):
                s = [sbox(s[i] + rc[i], row[k + i]) for i in range(3)]
                s = ext(s)
                for i in range(3):
                    builder.assert_eq(s[i], row[k + 3 + i])
                return [E(row[k + 3 + i]) for i in range(3)], k + 6

            for rc in begin:
                s, k = full(s, rc, k)
            for rc in partial:
                x = sbox(s[0] + rc, row[k])
                builder.assert_eq(x, row[k + 1])
                s = internal([E(row[k + 1]), s[1], s[2]])
                k += 2
            for rc in end:
                s, k = full(s, rc, k)


class AirProgram:
    """An AIR compiled for the generic quotient path (eon_air_program, include/eon.h): the
    constraint DAG get_symbolic_constraints returns (symbolic.py) -> device program.

    ``air`` is any object with ``width()``, ``num_public_values()`` and ``eval(builder)`` on the
    EonAirBuilder surface (symbolic.SymbolicAirBuilder)."""

    def __init__(self, air, ctx: Context | None = None):
        from . import symbolic

        self.ctx = ctx or default_context(0)
        self.air = air
        self.n_public = int(air.num_public_values())
        self.width = symbolic.air_width(air)
        cs = symbolic.get_symbolic_constraints(air, 0, self.n_public)
        nodes, consts, roots = symbolic.serialize(cs)
        self.num_nodes = len(nodes)
        na = (_lib.eon_sym_node * max(1, len(nodes)))(*[_lib.eon_sym_node(*n) for n in nodes])
        from .field import ints_to_limbs

        ca = np.ascontiguousarray(ints_to_limbs(consts) if consts else np.zeros((1, 4), np.uint64))
        ra = np.ascontiguousarray(np.array(roots if roots else [0], dtype=np.uint32))
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx.lib.eon_air_program_create(
            self.ctx.handle, na, len(nodes), ca.ctypes.data_as(ctypes.c_void_p), len(consts),
            ra.ctypes.data_as(ctypes.c_void_p), len(roots), self.width, self.n_public, ctypes.byref(h)))
        self._h = h
        st = _lib.eon_air_program_stats()
        self.ctx.check(self.ctx.lib.eon_air_program_info(h, ctypes.byref(st)))
        self.stats = {k: int(getattr(st, k)) for k, _ in st._fields_}
        self.max_constraint_degree = self.stats["max_constraint_degree"]
        self.num_constraints = self.stats["num_constraints"]

    @property
    def handle(self):
        return self._h

    def log_quotient_degree(self, is_zk: int = 0) -> int:
        return int(self.ctx.lib.eon_air_program_log_quotient_degree(self._h, is_zk))

    def quotient_values(self, lde, log_n: int, log_qd: int, alpha, publics=()):
        """quotient_values (prover.rs:539-709) on the trace's LDE over GENERATOR * K (natural)."""
        import torch

        from .field import fr_to_abi

        q = 1 << (log_n + log_qd)
        out = torch.empty((q, 4), dtype=torch.int64, device=lde.device)
        a = fr_to_abi(alpha)
        pub = _publics_limbs(publics)
        self.ctx.set_stream(torch.cuda.current_stream(lde.device).cuda_stream)
        self.ctx.check(self.ctx.lib.eon_quotient_values_dev(
            self.ctx.handle, self._h, _dp(lde.contiguous()), log_n, log_qd, ctypes.byref(a),
            pub.ctypes.data_as(ctypes.c_void_p), len(publics), _dp(out)))
        return out

    def close(self):
        if getattr(self, "_h", None):
            self.ctx.lib.eon_air_program_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _publics_limbs(publics) -> np.ndarray:
    """canonical ints (or (n, 4) Montgomery limbs) -> contiguous (max(n,1), 4) u64 limbs"""
    from .field import ints_to_limbs

    if len(publics) == 0:
        return np.zeros((1, 4), np.uint64)
    if isinstance(publics, np.ndarray) and publics.ndim == 2:
        return np.ascontiguousarray(publics, dtype=np.uint64)
    return np.ascontiguousarray(ints_to_limbs([int(x) for x in publics]))


def selectors_on_coset(log_n: int, log_q: int, shift, device=0, ctx: Context | None = None):
    """-> (4, 2^log_q, 4) device tensor: is_first_row, is_last_row, is_transition, inv_vanishing."""
    import torch

    ctx = ctx or default_context(device)
    out = torch.empty((4, 1 << log_q, 4), dtype=torch.int64, device=f"cuda:{device}")
    s = fr_to_abi(shift)
    ctx.set_stream(torch.cuda.current_stream(out.device).cuda_stream)
    ctx.check(ctx.lib.eon_selectors_on_coset_dev(ctx.handle, log_n, log_q, ctypes.byref(s), _dp(out)))
    return out
