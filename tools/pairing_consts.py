"""Generate the constant tables of csrc/pairing.h (BN254 optimal-ate pairing) from their
definitions, with Python integers (run once, output pasted into pairing.h; the GPU tests compare
the kernels with oracle/pairing.py, which derives the same values independently).

Tower: Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3 - xi), Fq12 = Fq6[w]/(w^2 - v), xi = 9 + u, so
w^6 = xi.  Frobenius: (a w^k)^(q^j) = frob_j(a) w^k xi^(k (q^j - 1) / 6).
"""

Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
X_BN = 4965661367192848881


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % Q, (a[0] * b[1] + a[1] * b[0]) % Q)


def f2_pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_mul(a, a)
        e >>= 1
    return r


def mont_limbs32(x):
    m = x * (1 << 256) % Q
    return [(m >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def fq_lit(x):
    return "{" + ", ".join(f"0x{v:08x}u" for v in mont_limbs32(x)) + "}"


def f2_lit(a):
    return "{" + fq_lit(a[0]) + ", " + fq_lit(a[1]) + "}"


XI = (9, 1)


def main():
    assert (Q - 1) % 6 == 0
    out = []
    for j in (1, 2, 3):
        ks = []
        for k in range(6):
            g = f2_pow(XI, k * (Q ** j - 1) // 6)
            ks.append(f2_lit(g))
        out.append(f"// xi^(k (q^{j} - 1) / 6), k = 0..5\nconstexpr uint32_t FROB{j}[6][2][8] = {{\n    " + ",\n    ".join(ks) + "};")
    # twist Frobenius: pi(x, y) = (conj(x) xi^((q-1)/3), conj(y) xi^((q-1)/2))
    g13 = f2_pow(XI, (Q - 1) // 3)
    g12 = f2_pow(XI, (Q - 1) // 2)
    g23 = f2_pow(XI, (Q * Q - 1) // 3)
    g22 = f2_pow(XI, (Q * Q - 1) // 2)
    assert g23[1] == 0 and g22 == (Q - 1, 0)
    out.append(f"constexpr uint32_t TWIST_FROB_X[2][8] = {f2_lit(g13)};")
    out.append(f"constexpr uint32_t TWIST_FROB_Y[2][8] = {f2_lit(g12)};")
    out.append(f"constexpr uint32_t TWIST_FROB2_X[8] = {fq_lit(g23[0])};  // xi^((q^2-1)/3) (in Fq); xi^((q^2-1)/2) = -1")
    inv_xi = f2_pow(XI, Q * Q - 2)
    b2 = f2_mul((3, 0), inv_xi)
    out.append(f"constexpr uint32_t TWIST_B[2][8] = {f2_lit(b2)};  // 3 / xi")
    hard = (Q ** 4 - Q ** 2 + 1)
    assert hard % R == 0
    # the hard part (q^4 - q^2 + 1) / r = l0 + l1 q + l2 q^2 + l3 q^3 exactly, with the l_i
    # polynomials in x (Scott et al., "On the final exponentiation for calculating pairings on
    # ordinary elliptic curves", 2009): pairing.hip computes it from f^x, f^(x^2), f^(x^3)
    x = X_BN
    l3, l2 = 1, 6 * x * x + 1
    l1 = -36 * x ** 3 - 18 * x * x - 12 * x + 1
    l0 = -36 * x ** 3 - 30 * x * x - 18 * x - 2
    assert l0 + l1 * Q + l2 * Q * Q + l3 * Q ** 3 == hard // R
    # the addition chain of final_exponentiation (y_i exponents, then T0 / T1 as in the kernel)
    y0, y1, y2, y3 = Q + Q * Q + Q ** 3, -1, x * x * Q * Q, -x * Q
    y4, y5, y6 = -(x + x * x * Q), -x * x, -(x ** 3 + x ** 3 * Q)
    t0 = 2 * y6 + y4 + y5
    t1 = y3 + y5 + t0
    t0 = t0 + y2
    t1 = 4 * t1 + 2 * t0
    t0, t1 = 2 * (t1 + y1), t1 + y0
    assert t0 + t1 == hard // R
    out.append(f"constexpr uint64_t BN_X = 0x{x:x}ull;  // the BN parameter x (q, r are polynomials in x)")
    # x in non-adjacent form: x = sum of 2^i over NAF_POS's bits minus 2^i over NAF_NEG's (24 digits
    # against x's 28 set bits); the top digit is bit 62
    pos = neg = 0
    k, i = x, 0
    while k:
        if k & 1:
            d = 2 - (k % 4)
            k -= d
            if d == 1:
                pos |= 1 << i
            else:
                neg |= 1 << i
        k //= 2
        i += 1
    assert pos - neg == x and pos >> 62 == 1 and (pos | neg) >> 63 == 0
    out.append(f"constexpr uint64_t BN_X_NAF_POS = 0x{pos:x}ull, BN_X_NAF_NEG = 0x{neg:x}ull;")
    # the standard BN254 G2 generator (EIP-197; halo2curves' G2::generator)
    gx = (10857046999023057135944570762232829481370756359578518086990519993285655852781,
          11559732032986387107991004021392285783925812861821192530917403151452391805634)
    gy = (8495653923123431417604973247489272438418190587263600148770280649306958101930,
          4082367875863433681332203403145435568316851327593401208105741076214120093531)
    lhs = f2_mul(gy, gy)
    rhs = f2_mul(f2_mul(gx, gx), gx)
    rhs = ((rhs[0] + b2[0]) % Q, (rhs[1] + b2[1]) % Q)
    assert lhs == rhs
    out.append(f"constexpr uint32_t G2_GEN_X[2][8] = {f2_lit(gx)};")
    out.append(f"constexpr uint32_t G2_GEN_Y[2][8] = {f2_lit(gy)};")
    # 2^i G2 (affine), i = 0..255: [z] G2 for verify_batch by additions only (fixed base)
    def f2_inv(a):
        return f2_pow(a, Q * Q - 2)

    def g2_dbl(p):
        x, y = p
        x2 = f2_mul(x, x)
        lam = f2_mul((3 * x2[0] % Q, 3 * x2[1] % Q), f2_inv(((2 * y[0]) % Q, (2 * y[1]) % Q)))
        l2 = f2_mul(lam, lam)
        x3 = ((l2[0] - 2 * x[0]) % Q, (l2[1] - 2 * x[1]) % Q)
        t = f2_mul(lam, ((x[0] - x3[0]) % Q, (x[1] - x3[1]) % Q))
        return x3, ((t[0] - y[0]) % Q, (t[1] - y[1]) % Q)

    p, rows = (gx, gy), []
    for _ in range(256):
        rows.append("{" + f2_lit(p[0]) + ", " + f2_lit(p[1]) + "}")
        p = g2_dbl(p)
    out.append("constexpr uint32_t G2_POW2[256][2][2][8] = {  // 2^i G2, i = 0..255 (x, y)\n    "
               + ",\n    ".join(rows) + "};")
    # 2^i G1 (affine, G1 = (1, 2) on y^2 = x^3 + 3), i = 0..255: [sum v] G1 by additions only
    def g1_dbl(p):
        x, y = p
        lam = 3 * x * x * pow(2 * y, Q - 2, Q) % Q
        x3 = (lam * lam - 2 * x) % Q
        return x3, (lam * (x - x3) - y) % Q

    p, rows = (1, 2), []
    for _ in range(256):
        rows.append("{" + fq_lit(p[0]) + ", " + fq_lit(p[1]) + "}")
        p = g1_dbl(p)
    out.append("constexpr uint32_t G1_POW2[256][2][8] = {  // 2^i G1, i = 0..255 (x, y)\n    "
               + ",\n    ".join(rows) + "};")
    ate = 6 * X_BN + 2
    assert ate.bit_length() == 65
    out.append(f"constexpr uint64_t ATE_LOOP_LOW = 0x{ate & ((1 << 64) - 1):x}ull;  // 6x + 2 below its top bit (bit 64)")
    # 6x + 2 in non-adjacent form for the Miller loop: 22 nonzero digits against 37 set bits; the
    # top digit is 65 and digit 64 is zero, so the loop runs bits 64..0 from the masks
    pos = neg = 0
    k, i = ate, 0
    while k:
        if k & 1:
            d = 2 - (k % 4)
            k -= d
            if d == 1:
                pos |= 1 << i
            else:
                neg |= 1 << i
        k //= 2
        i += 1
    assert pos - neg == ate and pos >> 65 == 1 and (pos | neg) >> 64 == 2
    low = (1 << 64) - 1
    out.append(f"constexpr uint64_t ATE_NAF_POS = 0x{pos & low:x}ull, ATE_NAF_NEG = 0x{neg & low:x}ull;"
               "  // 6x + 2 = 2^65 + POS - NEG")
    print("\n".join(out))


if __name__ == "__main__":
    main()
