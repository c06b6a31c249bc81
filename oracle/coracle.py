"""ctypes binding of the C restatement oracle (oracle/eon_oracle.c -> oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
Matrices are numpy uint64 arrays of shape (h, w, 4): Fr Montgomery limbs, row-major.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"


class fr_t(ctypes.Structure):
    _fields_ = [("v", ctypes.c_uint64 * 4)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        l = ctypes.CDLL(os.fspath(LIB))
        P, U64, U32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        sigs = {
            "or_radix2dit_dft_batch": [P, U64, U64],
            "or_idft_batch": [P, U64, U64],
            "or_coset_dft_batch": [P, U64, U64, fr_t],
            "or_coset_idft_batch": [P, U64, U64, fr_t],
            "or_coset_lde_batch": [P, P, U64, U64, U32, fr_t],
            "or_r2dp_dft_batch": [P, U64, U64],
            "or_r2dp_coset_lde_batch": [P, P, U64, U64, U32, fr_t],
            "or_fr_mul_batch": [P, P, P, U64],
            "or_reverse_matrix_index_bits": [P, U64, U64],
        }
        for k, a in sigs.items():
            getattr(l, k).argtypes = a
            getattr(l, k).restype = None
        l.or_fr_from_u64.argtypes = [U64]
        l.or_fr_from_u64.restype = fr_t
        l.or_two_adic_generator.argtypes = [U32]
        l.or_two_adic_generator.restype = fr_t
        l.or_fr_pow.argtypes = [fr_t, U64]
        l.or_fr_pow.restype = fr_t
        l.or_num_threads.restype = ctypes.c_int
        l.or_set_num_threads.argtypes = [ctypes.c_int]
        l.or_set_num_threads.restype = None
        l.or_eval_poly_col.argtypes = [P, U64, U64, U64, fr_t]
        l.or_eval_poly_col.restype = fr_t
        l.or_kzg_evaluations_on_domain.argtypes = [P, U64, U64, U32, fr_t, P]
        l.or_kzg_evaluations_on_domain.restype = None
        for k, a in {"or_g1_generator": [P], "or_g1_mul": [P, P, P], "or_g1_add": [P, P, P],
                     "or_g1_srs": [U64, P, P], "or_g1_msm": [P, P, U64, P],
                     "or_g1_msm_columns": [P, P, U64, U64, P]}.items():
            getattr(l, k).argtypes = a
            getattr(l, k).restype = None
        for k, a in {"or_p2_generate_trace": [P, U64, U32, U32, U32, P, P, P, P],
                     "or_selectors_on_coset": [U32, U32, fr_t, P, P, P, P],
                     "or_p2_quotient_values": [P, U32, U32, U32, U32, U32, P, P, P, fr_t, P],
                     "or_quotient_and_eval": [P, U64, U64, fr_t, P, P],
                     "or_open_columns": [P, P, U64, U64, fr_t, P, P],
                     "or_bary_eval_cols": [P, U64, U64, P, U32, P]}.items():
            getattr(l, k).argtypes = a
            getattr(l, k).restype = None
        l.or_p2_num_cols.argtypes = [U32, U32]
        l.or_p2_num_cols.restype = U32
        l.or_g1_on_curve.argtypes = [P]
        l.or_g1_on_curve.restype = ctypes.c_int
        _lib = l
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def fr(limbs) -> fr_t:
    s = fr_t()
    for i in range(4):
        s.v[i] = int(limbs[i])
    return s


def fr_from_u64(x: int):
    r = lib().or_fr_from_u64(x)
    return np.array([r.v[i] for i in range(4)], dtype=np.uint64)


def _copy(m):
    return np.ascontiguousarray(m, dtype=np.uint64).copy()


def dft_batch(m):
    x = _copy(m)
    lib().or_radix2dit_dft_batch(_ptr(x), x.shape[0], x.shape[1])
    return x


def idft_batch(m):
    x = _copy(m)
    lib().or_idft_batch(_ptr(x), x.shape[0], x.shape[1])
    return x


def coset_dft_batch(m, shift_limbs):
    x = _copy(m)
    lib().or_coset_dft_batch(_ptr(x), x.shape[0], x.shape[1], fr(shift_limbs))
    return x


def coset_idft_batch(m, shift_limbs):
    x = _copy(m)
    lib().or_coset_idft_batch(_ptr(x), x.shape[0], x.shape[1], fr(shift_limbs))
    return x


def coset_lde_batch(m, added_bits, shift_limbs):
    x = np.ascontiguousarray(m, dtype=np.uint64)
    out = np.empty((x.shape[0] << added_bits, x.shape[1], 4), dtype=np.uint64)
    lib().or_coset_lde_batch(_ptr(x), _ptr(out), x.shape[0], x.shape[1], added_bits, fr(shift_limbs))
    return out


def r2dp_dft_batch(m):
    """Radix2DitParallel::dft_batch storage (bit-reversed)."""
    x = _copy(m)
    lib().or_r2dp_dft_batch(_ptr(x), x.shape[0], x.shape[1])
    return x


def r2dp_coset_lde_batch(m, added_bits, shift_limbs):
    """Radix2DitParallel::coset_lde_batch storage (bit-reversed)."""
    x = np.ascontiguousarray(m, dtype=np.uint64)
    out = np.empty((x.shape[0] << added_bits, x.shape[1], 4), dtype=np.uint64)
    lib().or_r2dp_coset_lde_batch(_ptr(x), _ptr(out), x.shape[0], x.shape[1], added_bits, fr(shift_limbs))
    return out


def bit_reverse_rows(m):
    x = _copy(m)
    lib().or_reverse_matrix_index_bits(_ptr(x), x.shape[0], x.shape[1])
    return x


def eval_poly_col(coeffs, col: int, point_limbs):
    """eval_poly (kzg/src/util.rs:63-68) of column `col` at a point (Montgomery limbs)."""
    x = np.ascontiguousarray(coeffs, dtype=np.uint64)
    r = lib().or_eval_poly_col(_ptr(x), x.shape[0], x.shape[1], col, fr(point_limbs))
    return np.array([r.v[i] for i in range(4)], dtype=np.uint64)


def kzg_evaluations_on_domain(coeffs, log_q: int, shift_limbs):
    """KzgPcs::get_evaluations_on_domain (kzg/src/pcs.rs:267-287): Horner at every point."""
    x = np.ascontiguousarray(coeffs, dtype=np.uint64)
    out = np.empty((1 << log_q, x.shape[1], 4), dtype=np.uint64)
    lib().or_kzg_evaluations_on_domain(_ptr(x), x.shape[0], x.shape[1], log_q, fr(shift_limbs), _ptr(out))
    return out


def fr_pow(base_limbs, e: int):
    r = lib().or_fr_pow(fr(base_limbs), e)
    return np.array([r.v[i] for i in range(4)], dtype=np.uint64)


def fr_mul(a, b):
    a = np.ascontiguousarray(a, dtype=np.uint64).reshape(1, 4)
    b = np.ascontiguousarray(b, dtype=np.uint64).reshape(1, 4)
    r = np.empty_like(a)
    lib().or_fr_mul_batch(_ptr(a), _ptr(b), _ptr(r), 1)
    return r[0]


def two_adic_generator(bits: int):
    r = lib().or_two_adic_generator(bits)
    return np.array([r.v[i] for i in range(4)], dtype=np.uint64)


# --- G1 (points: numpy uint64 (..., 8) = x[4], y[4] Fq Montgomery; identity = zeros) ---------
def g1_generator():
    out = np.zeros(8, dtype=np.uint64)
    lib().or_g1_generator(_ptr(out))
    return out


def g1_mul(p, scalar_limbs):
    p = np.ascontiguousarray(p, dtype=np.uint64)
    s = np.ascontiguousarray(scalar_limbs, dtype=np.uint64)
    out = np.zeros(8, dtype=np.uint64)
    lib().or_g1_mul(_ptr(p), _ptr(s), _ptr(out))
    return out


def g1_add(a, b):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    out = np.zeros(8, dtype=np.uint64)
    lib().or_g1_add(_ptr(a), _ptr(b), _ptr(out))
    return out


def g1_on_curve(p) -> bool:
    return bool(lib().or_g1_on_curve(_ptr(np.ascontiguousarray(p, dtype=np.uint64))))


def g1_srs(n: int, alpha_limbs):
    """init_srs_unsafe g1_powers (kzg/src/params.rs:123-139), affine."""
    out = np.zeros((n, 8), dtype=np.uint64)
    a = np.ascontiguousarray(alpha_limbs, dtype=np.uint64)
    lib().or_g1_srs(n, _ptr(a), _ptr(out))
    return out


def g1_msm(points, scalars):
    """Value of G1::multi_exp (Pippenger restatement)."""
    p = np.ascontiguousarray(points, dtype=np.uint64)
    s = np.ascontiguousarray(scalars, dtype=np.uint64)
    out = np.zeros(8, dtype=np.uint64)
    lib().or_g1_msm(_ptr(p), _ptr(s), p.shape[0], _ptr(out))
    return out


def g1_msm_columns(points, mat):
    """KzgPcs::commit's per-column commit_column (kzg/src/pcs.rs:244-251) of an (n, w, 4) matrix
    against points[:n] -> (w, 8); columns in parallel."""
    p = np.ascontiguousarray(points, dtype=np.uint64)
    m = np.ascontiguousarray(mat, dtype=np.uint64)
    n, w = m.shape[0], m.shape[1]
    out = np.zeros((w, 8), dtype=np.uint64)
    lib().or_g1_msm_columns(_ptr(p), _ptr(m), n, w, _ptr(out))
    return out


def open_columns(points, coeffs, z_limbs):
    """KzgPcs::open of one (n, w, 4) coefficient matrix at one point (kzg/src/pcs.rs:289-335):
    per column quotient_and_eval and commit_column(quotient) over points[:n-1] -> (values (w, 4),
    witnesses (w, 8)); columns in parallel."""
    p = np.ascontiguousarray(points, dtype=np.uint64)
    c = np.ascontiguousarray(coeffs, dtype=np.uint64)
    n, w = c.shape[0], c.shape[1]
    vals = np.zeros((w, 4), dtype=np.uint64)
    wits = np.zeros((w, 8), dtype=np.uint64)
    lib().or_open_columns(_ptr(p), _ptr(c), n, w, fr(z_limbs), _ptr(vals), _ptr(wits))
    return vals, wits


# --- Poseidon2-AIR / quotient / open ----------------------------------------------------------
class P2Constants:
    """Round constants as Montgomery limb arrays: begin (hf, 3, 4), partial (pr, 4), end (hf, 3, 4)."""

    def __init__(self, begin, partial, end):
        self.begin = np.ascontiguousarray(begin, dtype=np.uint64).reshape(-1, 3, 4)
        self.partial = np.ascontiguousarray(partial, dtype=np.uint64).reshape(-1, 4)
        self.end = np.ascontiguousarray(end, dtype=np.uint64).reshape(-1, 3, 4)
        self.hf = self.begin.shape[0]
        self.pr = self.partial.shape[0]

    @property
    def num_cols(self):
        return 1 + 3 + 12 * self.hf + 2 * self.pr


def p2_generate_trace(inputs, vl: int, k: P2Constants):
    x = np.ascontiguousarray(inputs, dtype=np.uint64).reshape(-1, 3, 4)
    n = x.shape[0]
    out = np.zeros((n // vl, k.num_cols * vl, 4), dtype=np.uint64)
    lib().or_p2_generate_trace(_ptr(x), n, vl, k.hf, k.pr, _ptr(k.begin), _ptr(k.partial), _ptr(k.end), _ptr(out))
    return out


def selectors_on_coset(log_n: int, log_q: int, shift_limbs):
    q = 1 << log_q
    out = np.zeros((4, q, 4), dtype=np.uint64)
    lib().or_selectors_on_coset(log_n, log_q, fr(shift_limbs), _ptr(out[0]), _ptr(out[1]), _ptr(out[2]), _ptr(out[3]))
    return out


def p2_quotient_values(lde, log_n: int, log_qd: int, vl: int, k: P2Constants, alpha_limbs):
    x = np.ascontiguousarray(lde, dtype=np.uint64)
    out = np.zeros((1 << (log_n + log_qd), 4), dtype=np.uint64)
    lib().or_p2_quotient_values(_ptr(x), log_n, log_qd, vl, k.hf, k.pr, _ptr(k.begin), _ptr(k.partial),
                                _ptr(k.end), fr(alpha_limbs), _ptr(out))
    return out


def quotient_and_eval(coeffs_col, point_limbs):
    """quotient_and_eval (kzg/src/util.rs:100-111) on one coefficient column."""
    c = np.ascontiguousarray(coeffs_col, dtype=np.uint64).reshape(-1, 4)
    n = c.shape[0]
    q = np.zeros((max(n - 1, 0), 4), dtype=np.uint64)
    v = np.zeros(4, dtype=np.uint64)
    lib().or_quotient_and_eval(_ptr(c), n, 1, fr(point_limbs), _ptr(q) if n > 1 else None, _ptr(v))
    return q, v


def bary_eval_cols(evals, points):
    """Every column polynomial of `evals` (n x w natural order over H) at each point (Montgomery
    limbs (npts, 4)): (npts, w, 4) -- the values quotient_and_eval returns, from the evaluations."""
    e = np.ascontiguousarray(evals, dtype=np.uint64)
    n, w = e.shape[0], e.shape[1]
    pts = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1, 4)
    out = np.zeros((pts.shape[0], w, 4), dtype=np.uint64)
    lib().or_bary_eval_cols(_ptr(e), n, w, _ptr(pts), pts.shape[0], _ptr(out))
    return out


def num_threads() -> int:
    return lib().or_num_threads()


class threads:
    """`with threads(n):` -- OpenMP threads of the C restatement inside the block."""

    def __init__(self, n: int):
        self.n = n

    def __enter__(self):
        self.prev = num_threads()
        lib().or_set_num_threads(self.n)
        return self

    def __exit__(self, *exc):
        lib().or_set_num_threads(self.prev)
        return False


def random_fr(seed: int, n: int) -> np.ndarray:
    """n uniform canonical Montgomery residues (rejection sampling as bn254/src/field.rs:534-551),
    numpy PCG64 stream -- deterministic test inputs."""
    rng = np.random.Generator(np.random.PCG64(seed))
    P = [0x43E1F593F0000001, 0x2833E84879B97091, 0xB85045B68181585D, 0x30644E72E131A029]
    out = np.empty((0, 4), dtype=np.uint64)
    while out.shape[0] < n:
        c = rng.integers(0, 2**64, size=(2 * (n - out.shape[0]) + 16, 4), dtype=np.uint64)
        c[:, 3] &= np.uint64((1 << 62) - 1)
        # accept if c < P (compare limbs from the top)
        lt = np.zeros(c.shape[0], dtype=bool)
        eq = np.ones(c.shape[0], dtype=bool)
        for i in (3, 2, 1, 0):
            lt |= eq & (c[:, i] < np.uint64(P[i]))
            eq &= c[:, i] == np.uint64(P[i])
        out = np.concatenate([out, c[lt]])
    return out[:n]
