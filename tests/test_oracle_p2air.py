"""CPU: the two restatements of the Poseidon2-AIR / quotient path agree (Python: explicit
constraint list + explicit reversed alpha powers; C: Horner fold), and a generated trace
satisfies every constraint (check_constraints, eon-uni-stark/src/check_constraints.rs)."""

import numpy as np
import pytest

from oracle import coracle as C
from oracle import pyoracle as O

HF, PR = 4, 56


def lim(x):
    return np.array(O.int_to_limbs(O.to_mont(x)), dtype=np.uint64)


@pytest.fixture(scope="module")
def consts():
    py = O.p2_constants(77, HF, PR)
    c = C.P2Constants([[lim(x) for x in r] for r in py[0]], [lim(x) for x in py[1]], [[lim(x) for x in r] for r in py[2]])
    return py, c


def test_trace_and_constraints(consts):
    py, c = consts
    assert O.p2_num_cols(HF, PR) == 164 == c.num_cols
    rng = O.SplitMix64(5)
    inputs = [[O.from_mont(rng.fr_mont()) for _ in range(3)] for _ in range(4)]
    rows = [O.p2_trace_row(i, py) for i in inputs]
    for r in rows:
        cs = O.p2_constraints(r, py)
        assert len(cs) == 160 and all(x == 0 for x in cs)
    tr = C.p2_generate_trace(np.array([[lim(x) for x in i] for i in inputs]), 2, c)
    assert tr.shape == (2, 328, 4)
    flat = [O.from_mont(O.limbs_to_int(e)) for e in tr.reshape(-1, 4)]
    assert flat == rows[0] + rows[1] + rows[2] + rows[3]


def test_selectors(consts):
    sel = C.selectors_on_coset(3, 5, lim(5))
    want = O.selectors_on_coset(3, 5, 5)
    for a, b in zip(sel, want):
        assert [O.from_mont(O.limbs_to_int(e)) for e in a] == b


@pytest.mark.parametrize("vl", [1, 2])
def test_quotient_values_c_vs_python(consts, vl):
    py, c = consts
    log_n, log_qd = 2, 1
    rng = O.SplitMix64(9 + vl)
    n = 1 << log_n
    inputs = [[O.from_mont(rng.fr_mont()) for _ in range(3)] for _ in range(n * vl)]
    rows = [sum((O.p2_trace_row(inputs[r * vl + v], py) for v in range(vl)), []) for r in range(n)]
    lde = O.coset_lde(rows, log_qd, O.GENERATOR)
    alpha = 123456789
    want = O.p2_quotient_values(lde, log_n, log_qd, vl, py, alpha)
    lde_np = np.array([[lim(x) for x in row] for row in lde], dtype=np.uint64)
    got = C.p2_quotient_values(lde_np, log_n, log_qd, vl, c, lim(alpha))
    assert [O.from_mont(O.limbs_to_int(e)) for e in got] == want


def test_quotient_and_eval():
    rng = O.SplitMix64(3)
    coeffs = [O.from_mont(rng.fr_mont()) for _ in range(9)]
    z = 987654321
    q, v = C.quotient_and_eval(np.array([lim(x) for x in coeffs]), lim(z))
    fz = sum(c * pow(z, i, O.P) for i, c in enumerate(coeffs)) % O.P
    assert O.from_mont(O.limbs_to_int(v)) == fz
    # (f(X) - f(z)) = q(X) (X - z)
    qs = [O.from_mont(O.limbs_to_int(e)) for e in q]
    prod = [0] * 9
    for i, a in enumerate(qs):
        prod[i + 1] = (prod[i + 1] + a) % O.P
        prod[i] = (prod[i] - z * a) % O.P
    assert prod == [(coeffs[0] - fz) % O.P] + coeffs[1:]
