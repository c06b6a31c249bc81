"""Fr / Fq value formatting for the C ABI (host side, not a compute path).

An Fr element crosses the boundary as 4 little-endian u64 limbs of its Montgomery residue
a*2^256 mod r (bn254/src/field.rs:98-105); these helpers convert Python ints and numpy limb
arrays.  Field arithmetic itself only runs in the HIP kernels.
"""

from __future__ import annotations

import numpy as np

from . import _lib

FR_MODULUS = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
FQ_MODULUS = 21888242871839275222246405745257275088696311157297823662689037894645226208583
_R = 1 << 256
_MASK64 = (1 << 64) - 1


def fr_mont(x: int) -> int:
    return (x % FR_MODULUS) * (_R % FR_MODULUS) % FR_MODULUS


def fr_unmont(m: int) -> int:
    return m * pow(_R, -1, FR_MODULUS) % FR_MODULUS


def _limbs(v: int):
    return [(v >> (64 * i)) & _MASK64 for i in range(4)]


def fr_to_abi(x) -> _lib.eon_fr:
    """canonical int -> eon_fr (Montgomery).  A 4-tuple/array is taken as Montgomery limbs."""
    s = _lib.eon_fr()
    if isinstance(x, (int, np.integer)):
        limbs = _limbs(fr_mont(int(x)))
    else:
        limbs = [int(v) for v in x]
    for i in range(4):
        s.l[i] = limbs[i]
    return s


def ints_to_limbs(values, mont: bool = True) -> np.ndarray:
    """Iterable of canonical ints -> (n, 4) u64 Montgomery limbs."""
    vals = list(values)
    out = np.empty((len(vals), 4), dtype=np.uint64)
    for i, x in enumerate(vals):
        v = fr_mont(x) if mont else int(x)
        out[i] = _limbs(v)
    return out


def limbs_to_ints(arr, mont: bool = True):
    """(..., 4) u64 limbs -> flat list of canonical ints."""
    a = np.asarray(arr, dtype=np.uint64).reshape(-1, 4)
    out = []
    for row in a:
        v = int(row[0]) | int(row[1]) << 64 | int(row[2]) << 128 | int(row[3]) << 192
        out.append(fr_unmont(v) if mont else v)
    return out
