"""Test AIRs written against the EonAirBuilder surface (plonky3_eon_amd.symbolic), as the
reference's own tests define them."""


class FibonacciAir:
    """eon-uni-stark/tests/fib_air.rs:15-52: two columns (left, right), public values (a, b, x)."""

    def width(self):
        return 2

    def num_public_values(self):
        return 3

    def eval(self, builder):
        main = builder.main()
        a, b, x = builder.public_values()
        local, nxt = main[0], main[1]
        when_first_row = builder.when_first_row()
        when_first_row.assert_eq(local[0], a)
        when_first_row.assert_eq(local[1], b)
        when_transition = builder.when_transition()
        when_transition.assert_eq(local[1], nxt[0])  # a' <- b
        when_transition.assert_eq(local[0] + local[1], nxt[1])  # b' <- a + b
        builder.when_last_row().assert_eq(local[1], x)


class MockAir:
    """symbolic_builder.rs:308-354 MockAir: one assert_zero(main[offset][index]) per spec."""

    def __init__(self, specs, width):
        self.specs = specs
        self._w = width

    def width(self):
        return self._w

    def num_public_values(self):
        return 0

    def eval(self, builder):
        main = builder.main()
        for offset, index in self.specs:
            builder.assert_zero(main[offset][index])


class MixedAir:
    """Exercises every node kind the generic program supports: selectors, publics, next row,
    negation, constants, shared sub-expressions, bool checks and x^5 / x^7 chains."""

    def width(self):
        return 5

    def num_public_values(self):
        return 2

    def eval(self, builder):
        m = builder.main()
        loc, nxt = m[0], m[1]
        p0, p1 = builder.public_values()
        s = loc[0] + loc[1] * 3  # shared below
        builder.assert_zero(s * s - nxt[2])
        builder.when_first_row().assert_eq(loc[3], p0)
        builder.when_last_row().assert_one(-loc[4] + p1)
        builder.when_transition().assert_eq(nxt[0], s.exp_const_u64(5) - loc[2].exp_const_u64(7))
        builder.assert_bool(loc[1])
        builder.when(loc[2] - 7).assert_zeros([loc[3] * nxt[4], -(nxt[1] - 11)])
        builder.assert_zero(s)  # a constraint that is a shared value
        builder.assert_zero(loc[4])  # a constraint that is a leaf


class MulAir:
    """MulAir of uni-stark/tests/mul_air.rs:37-118 (degree 3, boundary and transition constraints
    on): REPETITIONS = 20 triples (a, b, c) per row; assert_zero(a^2 b - c); when_first_row
    assert_eq(a a + 1, b); when_transition assert_eq(a + 20, next a)."""

    REPETITIONS = 20

    def width(self):
        return 3 * self.REPETITIONS

    def num_public_values(self):
        return 0

    def eval(self, builder):
        m = builder.main()
        loc, nxt = m[0], m[1]
        for i in range(self.REPETITIONS):
            a, b, c = loc[3 * i], loc[3 * i + 1], loc[3 * i + 2]
            builder.assert_zero(a.exp_const_u64(2) * b - c)
            builder.when_first_row().assert_eq(a * a + 1, b)
            builder.when_transition().assert_eq(a + self.REPETITIONS, nxt[3 * i])
