"""Generates tests/golden/*.npz from the Python big-integer oracle (oracle/pyoracle.py).

Fixtures are data only: inputs and expected outputs as Fr / G1 Montgomery limbs (the C-ABI
layout).  Regenerate with `python tests/golden/make_golden.py`.  Contents:
  dft_kat.npz     the reference NaiveDft KAT (dft/src/naive.rs:49-85) and seeded DFT cases
                  (dft / idft / coset_dft / coset_idft / coset_lde natural and bit-reversed)
  msm_kat.npz     G1::multi_exp identities (bn254/src/curve.rs:598-628) and seeded MSMs
"""

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import pyoracle as O  # noqa: E402


def mat(m):
    h = len(m)
    w = len(m[0]) if h else 0
    return np.array([[O.int_to_limbs(O.to_mont(x)) for x in row] for row in m], dtype=np.uint64).reshape(h, w, 4)


def pt(p):
    return np.frombuffer(O.g1_to_bytes(p), dtype=np.uint64).copy()


def main():
    d = {}
    kat_in = [[5, 2, 0], [4, 3, 0]]
    d["kat_in"] = mat(kat_in)
    d["kat_dft"] = mat(O.dft(kat_in))
    s = O.GENERATOR
    d["shift"] = np.array(O.int_to_limbs(O.to_mont(s)), dtype=np.uint64)
    cases = [(0, 1), (1, 2), (2, 3), (3, 1), (4, 3), (5, 2), (6, 3), (7, 1)]
    for log_h, w in cases:
        m = O.random_matrix(1000 + 10 * log_h + w, 1 << log_h, w)
        k = f"{log_h}_{w}"
        d[f"in_{k}"] = mat(m)
        d[f"dft_{k}"] = mat(O.dft(m))
        d[f"dft_bitrev_{k}"] = mat(O.bit_reverse_rows(O.dft(m)))
        d[f"idft_{k}"] = mat(O.idft(m))
        d[f"coset_dft_{k}"] = mat(O.coset_dft(m, s))
        d[f"coset_idft_{k}"] = mat(O.coset_idft(m, s))
        for b in (1, 2):
            lde = O.coset_lde(m, b, s)
            d[f"coset_lde{b}_{k}"] = mat(lde)
            d[f"coset_lde{b}_bitrev_{k}"] = mat(O.bit_reverse_rows(lde))
    np.savez_compressed(HERE / "dft_kat.npz", **d)

    g = O.G1_GEN
    m = {}
    m["g"] = pt(g)
    m["five_g"] = pt(O.g1_mul(g, 5))
    m["g7"] = pt(O.g1_mul(g, 7))
    m["g11"] = pt(O.g1_mul(g, 11))
    m["g76"] = pt(O.g1_mul(g, 76))
    rng = O.SplitMix64(4242)
    for n in (1, 3, 8, 33):
        pts = [O.g1_mul(g, rng.next() % (1 << 40) + 1) for _ in range(n)]
        sc = [O.from_mont(rng.fr_mont()) for _ in range(n)]
        m[f"pts_{n}"] = np.stack([pt(p) for p in pts])
        m[f"scalars_{n}"] = np.stack([np.array(O.int_to_limbs(O.to_mont(x)), dtype=np.uint64) for x in sc])
        m[f"msm_{n}"] = pt(O.msm(pts, sc))
    srs = O.init_srs_g1(15, 12345)
    m["srs16"] = np.stack([pt(p) for p in srs])
    coeffs = [O.from_mont(rng.fr_mont()) for _ in range(16)]
    m["commit_coeffs16"] = np.stack([np.array(O.int_to_limbs(O.to_mont(x)), dtype=np.uint64) for x in coeffs])
    m["commit16"] = pt(O.commit_column(srs, coeffs))
    np.savez_compressed(HERE / "msm_kat.npz", **m)
    print("wrote", HERE / "dft_kat.npz", HERE / "msm_kat.npz")


if __name__ == "__main__":
    main()
