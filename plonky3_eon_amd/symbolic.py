"""Symbolic constraint capture for any AIR: the host side of the generic quotient path.

Mirrors eon-uni-stark's symbolic layer so an AIR written against the reference's builder surface
(eon-air/src/builder.rs) yields the same constraint list, in the same order, that
``get_symbolic_constraints`` returns (eon-uni-stark/src/symbolic_builder.rs:72-126):

* ``Entry`` / ``SymbolicVariable``       symbolic_variable.rs:8-40
* ``SymbolicExpression``                 symbolic_expression.rs:78-338 (constant folding on
                                         + - * and negation, cached degree_multiple)
* ``SymbolicAirBuilder``                 symbolic_builder.rs:117-249 (main = 2 rows, publics,
                                         is_first_row / is_last_row / is_transition_window(2))
* ``FilteredAirBuilder``                 eon-air/src/filtered_builder.rs:25-70 (cond * x)
* ``assert_eq / assert_one / assert_bool / when*``   eon-air/src/builder.rs:109-182
* ``get_max_constraint_degree`` / ``get_log_quotient_degree``   symbolic_builder.rs:15-69

``serialize`` flattens the constraint DAG into the ``eon_sym_node`` array that
``eon_air_program_create`` (include/eon.h) compiles into a device program -- the same array a Rust
shim would emit from the reference's own ``Vec<SymbolicExpression<Fr>>`` (shared ``Arc`` nodes
once, operands before users).  Field constants are canonical ints mod r.
"""

from __future__ import annotations

from dataclasses import dataclass

P = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001

# eon_sym_node kinds (include/eon.h)
SYM_CONSTANT = 0
SYM_MAIN = 1
SYM_PUBLIC = 2
SYM_IS_FIRST_ROW = 3
SYM_IS_LAST_ROW = 4
SYM_IS_TRANSITION = 5
SYM_ADD = 6
SYM_SUB = 7
SYM_NEG = 8
SYM_MUL = 9
SYM_PREPROCESSED = 10
SYM_PERMUTATION = 11
SYM_CHALLENGE = 12


@dataclass(frozen=True)
class Entry:
    """symbolic_variable.rs:8-15: kind in {"preprocessed", "main", "permutation", "public",
    "challenge"}; offset for the row-window kinds (0 = local, 1 = next)."""

    kind: str
    offset: int = 0


class SymbolicExpression:
    __slots__ = ("op", "x", "y", "value", "var", "degree_multiple")

    def __init__(self, op, x=None, y=None, value=None, var=None, degree_multiple=0):
        self.op = op  # "var" "const" "first" "last" "trans" "add" "sub" "neg" "mul"
        self.x = x
        self.y = y
        self.value = value
        self.var = var
        self.degree_multiple = degree_multiple

    # --- constructors (symbolic_expression.rs:198-222) --------------------------------------------
    @staticmethod
    def constant(v: int) -> "SymbolicExpression":
        return SymbolicExpression("const", value=v % P)

    @staticmethod
    def lift(v) -> "SymbolicExpression":
        if isinstance(v, SymbolicExpression):
            return v
        if isinstance(v, SymbolicVariable):
            return SymbolicExpression("var", var=v, degree_multiple=v.degree_multiple())
        if isinstance(v, int):
            return SymbolicExpression.constant(v)
        raise TypeError(f"cannot lift {type(v).__name__} into a SymbolicExpression")

    def is_const(self) -> bool:
        return self.op == "const"

    # --- ring operations with the reference's constant folding (symbolic_expression.rs:232-330) -
    def __add__(self, rhs):
        rhs = SymbolicExpression.lift(rhs)
        if self.is_const() and rhs.is_const():
            return SymbolicExpression.constant(self.value + rhs.value)
        return SymbolicExpression("add", self, rhs, degree_multiple=max(self.degree_multiple, rhs.degree_multiple))

    def __radd__(self, lhs):
        return SymbolicExpression.lift(lhs) + self

    def __sub__(self, rhs):
        rhs = SymbolicExpression.lift(rhs)
        if self.is_const() and rhs.is_const():
            return SymbolicExpression.constant(self.value - rhs.value)
        return SymbolicExpression("sub", self, rhs, degree_multiple=max(self.degree_multiple, rhs.degree_multiple))

    def __rsub__(self, lhs):
        return SymbolicExpression.lift(lhs) - self

    def __neg__(self):
        if self.is_const():
            return SymbolicExpression.constant(-self.value)
        return SymbolicExpression("neg", self, degree_multiple=self.degree_multiple)

    def __mul__(self, rhs):
        rhs = SymbolicExpression.lift(rhs)
        if self.is_const() and rhs.is_const():
            return SymbolicExpression.constant(self.value * rhs.value)
        return SymbolicExpression("mul", self, rhs, degree_multiple=self.degree_multiple + rhs.degree_multiple)

    def __rmul__(self, lhs):
        return SymbolicExpression.lift(lhs) * self

    def square(self):
        return self * self

    def cube(self):
        return self.square() * self

    def exp_const_u64(self, e: int):
        """PrimeCharacteristicRing::exp_const_u64 (field/src/field.rs:239-253): the reference's
        addition chains for 0..=7, so the DAG (and its degree) is the reference's."""
        if e == 0:
            return SymbolicExpression.constant(1)
        if e == 1:
            return self
        if e == 2:
            return self.square()
        if e == 3:
            return self.cube()
        if e == 4:
            return self.square().square()
        if e == 5:
            return self.square().square() * self
        if e == 6:
            return self.square().cube()
        if e == 7:
            x2 = self.square()
            return (x2 * self) * x2.square()
        acc = self
        for _ in range(e - 1):
            acc = acc * self
        return acc

    def double(self):
        return self + self

    def bool_check(self):
        """andn(x, x) = (1 - x) * x (field/src/field.rs:196-209)."""
        return (SymbolicExpression.constant(1) - self) * self

    def __repr__(self):
        if self.op == "const":
            return f"C({self.value})"
        if self.op == "var":
            return repr(self.var)
        if self.op in ("first", "last", "trans"):
            return self.op
        if self.op == "neg":
            return f"-({self.x!r})"
        return f"({self.x!r} {dict(add='+', sub='-', mul='*')[self.op]} {self.y!r})"


IS_FIRST_ROW = SymbolicExpression("first", degree_multiple=1)
IS_LAST_ROW = SymbolicExpression("last", degree_multiple=1)
IS_TRANSITION = SymbolicExpression("trans", degree_multiple=0)


class SymbolicVariable:
    """symbolic_variable.rs:17-40; arithmetic lifts into SymbolicExpression (:42-73)."""

    __slots__ = ("entry", "index")

    def __init__(self, entry: Entry, index: int):
        self.entry = entry
        self.index = index

    def degree_multiple(self) -> int:
        return 1 if self.entry.kind in ("preprocessed", "main", "permutation") else 0

    def _e(self):
        return SymbolicExpression.lift(self)

    def __add__(self, o):
        return self._e() + o

    def __radd__(self, o):
        return SymbolicExpression.lift(o) + self._e()

    def __sub__(self, o):
        return self._e() - o

    def __rsub__(self, o):
        return SymbolicExpression.lift(o) - self._e()

    def __mul__(self, o):
        return self._e() * o

    def __rmul__(self, o):
        return SymbolicExpression.lift(o) * self._e()

    def __neg__(self):
        return -self._e()

    def square(self):
        return self._e().square()

    def cube(self):
        return self._e().cube()

    def exp_const_u64(self, e: int):
        return self._e().exp_const_u64(e)

    def bool_check(self):
        return self._e().bool_check()

    def double(self):
        return self._e().double()

    def __repr__(self):
        if self.entry.kind in ("public", "challenge"):
            return f"{self.entry.kind}[{self.index}]"
        return f"{self.entry.kind}{self.entry.offset}[{self.index}]"


class _Builder:
    """The shared surface of EonAirBuilder (eon-air/src/builder.rs:36-224)."""

    def assert_zero(self, x):  # pragma: no cover - abstract
        raise NotImplementedError

    def assert_zeros(self, xs):
        for x in xs:
            self.assert_zero(x)

    def assert_eq(self, x, y):
        self.assert_zero(SymbolicExpression.lift(x) - y)

    def assert_one(self, x):
        self.assert_zero(SymbolicExpression.lift(x) - 1)

    def assert_bool(self, x):
        self.assert_zero(SymbolicExpression.lift(x).bool_check())

    def assert_bools(self, xs):
        self.assert_zeros([SymbolicExpression.lift(x).bool_check() for x in xs])

    def when(self, condition) -> "FilteredAirBuilder":
        return FilteredAirBuilder(self, SymbolicExpression.lift(condition))

    def when_ne(self, x, y) -> "FilteredAirBuilder":
        return self.when(SymbolicExpression.lift(x) - y)

    def when_first_row(self):
        return self.when(self.is_first_row())

    def when_last_row(self):
        return self.when(self.is_last_row())

    def when_transition(self):
        return self.when(self.is_transition())

    def when_transition_window(self, size: int):
        return self.when(self.is_transition_window(size))

    def is_transition(self):
        return self.is_transition_window(2)


class FilteredAirBuilder(_Builder):
    """eon-air/src/filtered_builder.rs: assert_zero(x) -> inner.assert_zero(condition * x)."""

    def __init__(self, inner: _Builder, condition: SymbolicExpression):
        self.inner = inner
        self.condition = condition

    def main(self):
        return self.inner.main()

    def public_values(self):
        return self.inner.public_values()

    def is_first_row(self):
        return self.inner.is_first_row()

    def is_last_row(self):
        return self.inner.is_last_row()

    def is_transition_window(self, size: int):
        return self.inner.is_transition_window(size)

    def assert_zero(self, x):
        self.inner.assert_zero(self.condition * SymbolicExpression.lift(x))


class SymbolicAirBuilder(_Builder):
    """symbolic_builder.rs:117-249.  ``main()`` returns the 2-row window: main()[0] = local row,
    main()[1] = next row, each a list of SymbolicVariable (RowMajorMatrix of width `width`)."""

    def __init__(self, preprocessed_width: int, width: int, num_public_values: int,
                 permutation_width: int = 0, num_permutation_challenges: int = 0):
        self._main = [[SymbolicVariable(Entry("main", off), i) for i in range(width)] for off in (0, 1)]
        self._preprocessed = [[SymbolicVariable(Entry("preprocessed", off), i) for i in range(preprocessed_width)]
                              for off in (0, 1)]
        self._permutation = ([[SymbolicVariable(Entry("permutation", off), i) for i in range(permutation_width)]
                              for off in (0, 1)] if permutation_width > 0 else None)
        self._challenges = [SymbolicVariable(Entry("challenge"), i) for i in range(num_permutation_challenges)]
        self._publics = [SymbolicVariable(Entry("public"), i) for i in range(num_public_values)]
        self.constraints: list[SymbolicExpression] = []

    def main(self):
        return self._main

    def preprocessed(self):
        return self._preprocessed

    def permutation(self):
        if self._permutation is None:
            raise RuntimeError("permutation called but aux trace is None")
        return self._permutation

    def permutation_randomness(self):
        return self._challenges

    def public_values(self):
        return self._publics

    def is_first_row(self):
        return IS_FIRST_ROW

    def is_last_row(self):
        return IS_LAST_ROW

    def is_transition_window(self, size: int):
        if size != 2:
            raise ValueError("uni-stark only supports a window size of 2")  # symbolic_builder.rs:215-221
        return IS_TRANSITION

    def assert_zero(self, x):
        self.constraints.append(SymbolicExpression.lift(x))


def air_width(air) -> int:
    """EonAir::width (a method on the reference's trait; an int attribute on Poseidon2Air)."""
    w = air.width
    return int(w() if callable(w) else w)


def get_symbolic_constraints(air, preprocessed_width: int = 0, num_public_values: int | None = None,
                             permutation_width: int = 0, num_permutation_challenges: int = 0):
    """symbolic_builder.rs:72-115 (no lookups: AirLookupHandler::eval is Air::eval,
    lookup/src/lookup_traits.rs:257-269)."""
    if num_public_values is None:
        num_public_values = air.num_public_values()
    b = SymbolicAirBuilder(preprocessed_width, air_width(air), num_public_values, permutation_width,
                           num_permutation_challenges)
    air.eval(b)
    return b.constraints


def get_max_constraint_degree(air, preprocessed_width: int = 0, num_public_values: int | None = None) -> int:
    """symbolic_builder.rs:46-69."""
    cs = get_symbolic_constraints(air, preprocessed_width, num_public_values)
    return max((c.degree_multiple for c in cs), default=0)


def log2_ceil(n: int) -> int:
    """p3_util::log2_ceil_usize."""
    return 0 if n <= 1 else (n - 1).bit_length()


def log_quotient_degree_of(max_degree: int, is_zk: int = 0) -> int:
    """get_log_quotient_degree's arithmetic (symbolic_builder.rs:28-42)."""
    assert is_zk <= 1, "is_zk must be either 0 or 1"
    d = max(max_degree + is_zk, 2)
    return log2_ceil(d - 1)


def get_log_quotient_degree(air, preprocessed_width: int = 0, num_public_values: int | None = None,
                            is_zk: int = 0) -> int:
    """symbolic_builder.rs:15-43."""
    return log_quotient_degree_of(get_max_constraint_degree(air, preprocessed_width, num_public_values), is_zk)


_KINDS = {"main": SYM_MAIN, "public": SYM_PUBLIC, "preprocessed": SYM_PREPROCESSED,
          "permutation": SYM_PERMUTATION, "challenge": SYM_CHALLENGE}


def serialize(constraints):
    """Flatten the DAG: returns (nodes [(kind, a, b)], consts [int], roots [node index]).
    Shared sub-expressions (the same Python object, as a shared Arc) are emitted once; operands
    precede their users.  Iterative post-order (deep Horner-like chains must not recurse)."""
    nodes, consts, index = [], [], {}
    const_idx = {}

    def emit(root):
        stack = [(root, False)]
        while stack:
            e, ready = stack.pop()
            if id(e) in index:
                continue
            kids = [k for k in (e.x, e.y) if k is not None]
            if not ready and any(id(k) not in index for k in kids):
                stack.append((e, True))
                for k in reversed(kids):
                    if id(k) not in index:
                        stack.append((k, False))
                continue
            if e.op == "const":
                if e.value not in const_idx:
                    const_idx[e.value] = len(consts)
                    consts.append(e.value)
                node = (SYM_CONSTANT, const_idx[e.value], 0)
            elif e.op == "var":
                v = e.var
                node = (_KINDS[v.entry.kind], v.index, v.entry.offset)
            elif e.op == "first":
                node = (SYM_IS_FIRST_ROW, 0, 0)
            elif e.op == "last":
                node = (SYM_IS_LAST_ROW, 0, 0)
            elif e.op == "trans":
                node = (SYM_IS_TRANSITION, 0, 0)
            elif e.op == "neg":
                node = (SYM_NEG, index[id(e.x)], 0)
            else:
                node = ({"add": SYM_ADD, "sub": SYM_SUB, "mul": SYM_MUL}[e.op], index[id(e.x)], index[id(e.y)])
            index[id(e)] = len(nodes)
            nodes.append(node)
        return index[id(root)]

    roots = [emit(c) for c in constraints]
    return nodes, consts, roots
