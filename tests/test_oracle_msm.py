"""The C restatement's Pippenger (signed windows, XYZZ buckets, parallel over window x chunk) and
its column-parallel commit / open helpers, against the per-column reference loops and the
group-law identities (bn254/src/curve.rs:598-628, kzg/src/util.rs:37-40,100-111)."""

import numpy as np
import pytest

from oracle import coracle as C
from oracle import pyoracle as O


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 1000, 4096])
def test_msm_equals_kzg_identity(n):
    alpha = C.fr_from_u64(4242)
    pts = C.g1_srs(n, alpha)
    s = C.random_fr(n + 7, n).reshape(n, 4)
    f = C.eval_poly_col(s.reshape(n, 1, 4), 0, alpha)
    np.testing.assert_array_equal(C.g1_msm(pts, s), C.g1_mul(C.g1_generator(), f))


def test_msm_edge_scalars_and_bases():
    """zero / one / p - 1 scalars, identity bases, P and -P, duplicates: against double-and-add."""
    g = C.g1_generator()
    p7 = C.g1_mul(g, C.fr_from_u64(7))
    neg7 = p7.copy()
    y = O.fq_from_mont(O.limbs_to_int([int(v) for v in p7[4:]]))
    neg7[4:] = np.array(O.int_to_limbs(O.fq_to_mont(O.Q - y)), dtype=np.uint64)
    pts = np.stack([p7, neg7, p7, np.zeros(8, np.uint64), g])
    pm1 = np.array(O.int_to_limbs(O.to_mont(O.P - 1)), dtype=np.uint64)
    one = C.fr_from_u64(1)
    zero = np.zeros(4, np.uint64)
    for sc in ([one, one, one, one, one], [pm1, pm1, zero, one, pm1], [zero] * 5, [one, pm1, one, pm1, zero]):
        s = np.stack(sc)
        acc = np.zeros(8, np.uint64)
        for i in range(5):
            acc = C.g1_add(acc, C.g1_mul(pts[i], s[i]))
        np.testing.assert_array_equal(C.g1_msm(pts, s), acc)


def test_columns_helpers_equal_the_per_column_loops():
    n, w = 300, 5
    pts = C.g1_srs(n, C.fr_from_u64(99))
    m = C.random_fr(5, n * w).reshape(n, w, 4)
    cols = C.g1_msm_columns(pts, m)
    z = C.random_fr(6, 1)[0]
    vals, wits = C.open_columns(pts[:n - 1], m, z)
    for j in range(w):
        np.testing.assert_array_equal(cols[j], C.g1_msm(pts, m[:, j]))
        q, v = C.quotient_and_eval(m[:, j], z)
        np.testing.assert_array_equal(vals[j], v)
        np.testing.assert_array_equal(wits[j], C.g1_msm(pts[:n - 1], q))
