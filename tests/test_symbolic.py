"""CPU tests of the symbolic layer (plonky3_eon_amd.symbolic) against the reference's own unit
tests (eon-uni-stark/src/symbolic_builder.rs:393-541, symbolic_expression.rs:350-854) and against
the oracle's direct constraint restatements (FibonacciAir, Poseidon2-AIR)."""

import random

import pytest

from oracle import pyoracle as O
from plonky3_eon_amd import symbolic as S

from airs import FibonacciAir, MixedAir, MockAir

P = O.P


def eval_serialized(nodes, consts, roots, local, nxt, sels, publics):
    """Evaluate the eon_sym_node array (the ABI form) directly."""
    v = []
    for kind, a, b in nodes:
        if kind == S.SYM_CONSTANT:
            x = consts[a]
        elif kind == S.SYM_MAIN:
            x = (nxt if b else local)[a]
        elif kind == S.SYM_PUBLIC:
            x = publics[a]
        elif kind in (S.SYM_IS_FIRST_ROW, S.SYM_IS_LAST_ROW, S.SYM_IS_TRANSITION):
            x = sels[kind - S.SYM_IS_FIRST_ROW]
        elif kind == S.SYM_ADD:
            x = v[a] + v[b]
        elif kind == S.SYM_SUB:
            x = v[a] - v[b]
        elif kind == S.SYM_NEG:
            x = -v[a]
        elif kind == S.SYM_MUL:
            x = v[a] * v[b]
        else:
            raise AssertionError(kind)
        v.append(x % P)
    return [v[r] for r in roots]


# --- reference unit tests (symbolic_builder.rs) ------------------------------------------------
def test_log_quotient_degree_no_constraints():
    assert S.get_log_quotient_degree(MockAir([], 4), 3, 2, 0) == 0


def test_log_quotient_degree_single_constraint():
    assert S.get_log_quotient_degree(MockAir([(0, 0)], 4), 3, 2, 0) == S.log2_ceil(1)


def test_log_quotient_degree_multiple_constraints():
    assert S.get_log_quotient_degree(MockAir([(0, 0), (1, 1), (0, 2)], 4), 3, 2, 0) == S.log2_ceil(1)


def test_max_constraint_degree():
    assert S.get_max_constraint_degree(MockAir([], 4), 3, 2) == 0
    assert S.get_max_constraint_degree(MockAir([(0, 0), (1, 1), (0, 2)], 4), 3, 2) == 1


def test_get_symbolic_constraints():
    cs = S.get_symbolic_constraints(MockAir([(0, 0), (1, 1)], 4), 3, 2)
    assert len(cs) == 2
    got = {(c.var.entry, c.var.index) for c in cs}
    assert got == {(S.Entry("main", 0), 0), (S.Entry("main", 1), 1)}


def test_builder_initialization():
    b = S.SymbolicAirBuilder(2, 4, 0, 0, 3)
    flat = [v for row in b.main() for v in row]
    assert [(v.entry, v.index) for v in flat] == [(S.Entry("main", o), i) for o in (0, 1) for i in range(4)]
    assert b.is_first_row() is S.IS_FIRST_ROW and b.is_last_row() is S.IS_LAST_ROW
    with pytest.raises(ValueError):
        b.is_transition_window(3)


def test_builder_assert_zero_constant():
    b = S.SymbolicAirBuilder(2, 4, 0, 0, 3)
    b.assert_zero(S.SymbolicExpression.constant(5))
    assert len(b.constraints) == 1 and b.constraints[0].op == "const" and b.constraints[0].value == 5


# --- symbolic_expression.rs tests ------------------------------------------------------------
def test_degree_multiples():
    var = S.SymbolicVariable(S.Entry("main", 0), 1)
    pre = S.SymbolicVariable(S.Entry("preprocessed", 0), 2)
    assert S.SymbolicExpression.lift(var).degree_multiple == 1
    assert S.SymbolicExpression.lift(pre).degree_multiple == 1
    assert S.SymbolicExpression.lift(S.SymbolicVariable(S.Entry("permutation", 0), 3)).degree_multiple == 1
    assert S.SymbolicExpression.lift(S.SymbolicVariable(S.Entry("public"), 4)).degree_multiple == 0
    assert S.SymbolicExpression.lift(S.SymbolicVariable(S.Entry("challenge"), 5)).degree_multiple == 0
    assert (S.IS_FIRST_ROW.degree_multiple, S.IS_LAST_ROW.degree_multiple, S.IS_TRANSITION.degree_multiple) == (1, 1, 0)
    assert (var + pre).degree_multiple == 1 and (var - pre).degree_multiple == 1
    assert (-S.SymbolicExpression.lift(var)).degree_multiple == 1 and (var * pre).degree_multiple == 2
    c = S.SymbolicVariable(S.Entry("main", 0), 2)
    assert ((var * pre) * c).degree_multiple == 3
    assert (S.SymbolicExpression.constant(5) + var).degree_multiple == 1


def test_constant_folding():
    C = S.SymbolicExpression.constant
    assert (C(3) + C(4)).value == 7 and (C(10) - C(4)).value == 6 and (C(3) * C(5)).value == 15
    assert (-C(7)).value == P - 7
    x = C(5)
    x = x + C(3)
    assert x.op == "const" and x.value == 8
    v = S.SymbolicVariable(S.Entry("main", 0), 0)
    assert (v - S.SymbolicVariable(S.Entry("main", 0), 1)).op == "sub" and (-v).op == "neg"


def test_fibonacci_degree_and_count():
    cs = S.get_symbolic_constraints(FibonacciAir())
    assert len(cs) == 5
    assert [c.degree_multiple for c in cs] == [2, 2, 1, 1, 2]
    assert S.get_log_quotient_degree(FibonacciAir()) == 0  # constraint degree 2 -> 1 quotient chunk


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fibonacci_matches_oracle(seed):
    rng = random.Random(seed)
    nodes, consts, roots = S.serialize(S.get_symbolic_constraints(FibonacciAir()))
    for _ in range(20):
        loc, nxt = [rng.randrange(P) for _ in range(2)], [rng.randrange(P) for _ in range(2)]
        sels, pub = [rng.randrange(P) for _ in range(3)], [rng.randrange(P) for _ in range(3)]
        assert eval_serialized(nodes, consts, roots, loc, nxt, sels, pub) == O.fib_constraints(loc, nxt, sels, pub)


def test_poseidon2_symbolic_matches_oracle():
    """The symbolic Poseidon2-AIR (air.Poseidon2Air.eval) reproduces the oracle's constraint list,
    itself pinned to poseidon2-air/src/air.rs:108-288 (tests/test_oracle_p2air.py)."""
    import numpy as np

    from plonky3_eon_amd.air import Poseidon2Air

    py = O.p2_constants(2024, 4, 56)

    def lim(v):
        return np.array(O.int_to_limbs(O.to_mont(v)), dtype=np.uint64)

    class _NoDevice(Poseidon2Air):  # the symbolic eval only needs the constants
        def __init__(self, vl):
            self._b = np.array([[lim(v) for v in r] for r in py[0]])
            self._p = np.array([lim(v) for v in py[1]])
            self._e = np.array([[lim(v) for v in r] for r in py[2]])
            self.vector_len = vl
            self.width = O.p2_num_cols(4, 56) * vl

        def __del__(self):
            pass

    for vl in (1, 2):
        air = _NoDevice(vl)
        cs = S.get_symbolic_constraints(air)
        assert len(cs) == 160 * vl
        assert max(c.degree_multiple for c in cs) == 3 and S.get_log_quotient_degree(air) == 1
        nodes, consts, roots = S.serialize(cs)
        rng = random.Random(vl)
        rows = [O.p2_trace_row([rng.randrange(P) for _ in range(3)], py) for _ in range(vl)]
        row = [x for r in rows for x in r]
        want = [c for r in rows for c in O.p2_constraints(r, py)]
        assert eval_serialized(nodes, consts, roots, row, row, [0, 0, 0], []) == want
        # a satisfied row: every constraint vanishes
        assert not any(want)
        bad = list(row)
        bad[10] = (bad[10] + 1) % P
        assert any(eval_serialized(nodes, consts, roots, bad, bad, [0, 0, 0], []))


def test_serialize_shares_nodes_and_orders_operands():
    nodes, consts, roots = S.serialize(S.get_symbolic_constraints(MixedAir()))
    for i, (kind, a, b) in enumerate(nodes):
        if kind in (S.SYM_ADD, S.SYM_SUB, S.SYM_MUL):
            assert a < i and b < i
        if kind == S.SYM_NEG:
            assert a < i
    # the shared `s` is emitted once: roots 0 (s*s - next) and 7 (s itself) point into one node
    s_idx = roots[7]
    assert nodes[roots[0]][0] == S.SYM_SUB and nodes[nodes[roots[0]][1]][1] == s_idx
    rng = random.Random(9)
    loc, nxt = [rng.randrange(P) for _ in range(5)], [rng.randrange(P) for _ in range(5)]
    sels, pub = [rng.randrange(P) for _ in range(3)], [rng.randrange(P) for _ in range(2)]
    got = eval_serialized(nodes, consts, roots, loc, nxt, sels, pub)
    s = (loc[0] + 3 * loc[1]) % P
    want = [(s * s - nxt[2]) % P, sels[0] * (loc[3] - pub[0]) % P, sels[1] * ((-loc[4] + pub[1]) - 1) % P,
            sels[2] * (nxt[0] - (pow(s, 5, P) - pow(loc[2], 7, P))) % P, (1 - loc[1]) * loc[1] % P,
            (loc[2] - 7) * loc[3] * nxt[4] % P, (loc[2] - 7) * (-(nxt[1] - 11)) % P, s, loc[4]]
    assert got == want


def test_deep_chain_serializes_without_recursion():
    """A 20000-deep left-leaning chain (sums over many columns build these) flattens iteratively."""
    v = S.SymbolicVariable(S.Entry("main", 0), 0)
    e = S.SymbolicExpression.lift(v)
    for _ in range(20000):
        e = e + v
    nodes, consts, roots = S.serialize([e])
    assert len(nodes) == 40001 and roots == [40000]  # each `+ v` lifts v into a fresh leaf, as From<SymbolicVariable> does
