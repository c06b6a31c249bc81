#!/usr/bin/env python3
"""Generate plonky3_eon_amd/csrc/prod_asm.h: whole radix-2^29 Montgomery products as ONE asm
statement each -- mul29, sqr29 (doubled cross terms) and mul29_sum2 of field29.h with the same
column schedule, the same unmasked multipliers and therefore the same results.

Why: hipcc pads every inline-asm statement with one wait state (`s_nop 0`) before the next VALU
instruction that reads one of its outputs (its hazard recognizer cannot see inside the string).
With one statement per column (mad_blocks.h) a product carries ~20 such pads, ~200 per XYZZ mixed
addition of the MSM piece sums.  The compiler's own code for these chains has no wait state
between the instructions (v_mad_u64_u32 -> v_mul_lo_u32 -> v_mad_u64_u32 -> v_lshrrev_b64 ->
v_and_b32 need none on gfx950), so a product in one statement needs none inside it.

Operands: the limbs of the inputs in VGPRs, the modulus limbs and -p^-1 mod 2^32 in SGPRs (the
compiler materialises the constants).  The 64-bit column accumulator is the fixed pair v[0:1]
(declared clobbered): AMDGPU inline asm cannot name the low half of a 64-bit operand, which the
multiplier (v_mul_lo_u32) and the output limbs (v_and_b32) read.  The carry-out of every
v_mad_u64_u32 goes to vcc (clobbered, never read).

Where the result goes (no register is written before its last read, because limb j of an operand
and multiplier m_j are last read in column j + 8, and output limb r_j is written in column j + 9):
  * `_asm`:     r_j takes multiplier m_j's register (9 early-clobber outputs, no other temporary);
  * `_asm_ip`:  r_j overwrites limb j of the first operand (mul29: a, mul29_sum2: c) in place --
    for `acc = acc * x` updates of a loop-carried accumulator, whose registers then need no copy
    at the back edge; the multipliers are 9 early-clobber temporaries.

usage: python3 tools/gen_prod_asm.py > plonky3_eon_amd/csrc/prod_asm.h
"""

ACC, ACC_LO = "v[0:1]", "v0"


def product(kind: str, U: int, inplace: bool):
    """The asm lines and operand lists of one product.  kind: mul (a b), sqr (a a, cross terms
    against 2 a_i), sum2 (a b + c d)."""
    outs, ins = [], []

    def operand(lst, c, e):
        lst.append('"%s"(%s)' % (c, e))

    # outputs first: %0 ..
    if inplace:
        dest = "a" if kind == "mul" else "c"
        for i in range(9):
            operand(outs, "+v", "%s.l[%d]" % (dest, i))
        R = ["%%%d" % i for i in range(9)]
        for i in range(9):
            operand(outs, "=&v", "m[%d]" % i)
        M = ["%%%d" % (9 + i) for i in range(9)]
        n = 18
    else:
        for i in range(9):
            operand(outs, "=&v", "r[%d]" % i)
        R = M = ["%%%d" % i for i in range(9)]
        n = 9
    DD = None
    if kind == "sqr":
        for i in range(8):
            operand(outs, "=&v", "dd[%d]" % i)
        DD = ["%%%d" % (n + i) for i in range(8)]
        n += 8
    nxt = [n]

    def add(c, e):
        operand(ins, c, e)
        nxt[0] += 1
        return "%%%d" % (nxt[0] - 1)

    A = R if (inplace and kind == "mul") else [add("v", "a.l[%d]" % i) for i in range(9)]
    B = C = D = None
    if kind in ("mul", "sum2"):
        B = [add("v", "b.l[%d]" % i) for i in range(9)]
    if kind == "sum2":
        C = R if inplace else [add("v", "c.l[%d]" % i) for i in range(9)]
        D = [add("v", "d.l[%d]" % i) for i in range(9)]
    P = [add("s", "P[%d]" % i) for i in range(9)]
    INV = add("s", "inv")
    lines = []
    first = [True]

    def mad(x, y):
        addend = "0" if first[0] else ACC
        first[0] = False
        lines.append("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (ACC, x, y, addend))

    if kind == "sqr":
        for i in range(8):
            lines.append("v_lshlrev_b32 %s, 1, %s" % (DD[i], A[i]))
    for k in range(17):
        lo, hi = max(0, k - 8), min(k, 8)
        for i in range(lo, hi + 1):
            j = k - i
            if kind == "sqr":
                if i < j:
                    mad(DD[i], A[j])
                elif i == j:
                    mad(A[i], A[i])
            else:
                mad(A[i], B[j])
        if kind == "sum2":
            for i in range(lo, hi + 1):
                mad(C[i], D[k - i])
        for i in range(lo, min(k, 9)):  # reduction terms m_i p_(k-i), i < k
            mad(M[i], P[k - i])
        if k < 9:
            lines.append("v_mul_lo_u32 %s, %s, %s" % (M[k], ACC_LO, INV))
            if k >= U:
                lines.append("v_and_b32 %s, 0x1fffffff, %s" % (M[k], M[k]))
            mad(M[k], P[0])
            lines.append("v_lshrrev_b64 %s, 29, %s" % (ACC, ACC))
        elif k < 16:
            lines.append("v_and_b32 %s, 0x1fffffff, %s" % (R[k - 9], ACC_LO))
            lines.append("v_lshrrev_b64 %s, 29, %s" % (ACC, ACC))
        else:  # r_7, and r_8 = acc >> 29 (< 2^32) straight from the pair
            lines.append("v_and_b32 %s, 0x1fffffff, %s" % (R[7], ACC_LO))
            lines.append("v_alignbit_b32 %s, v1, v0, 29" % R[8])
    return lines, outs, ins


def emit(name: str, kind: str, U: int, inplace: bool, params: str, doc: str) -> str:
    lines, outs, ins = product(kind, U, inplace)
    body = "\n            ".join('"%s\\n\\t"' % ln for ln in lines[:-1]) + '\n            "%s"' % lines[-1]
    temps = []
    if inplace:
        temps.append("uint32_t m[9];")
    else:
        temps.append("F29 res;")
        temps.append("uint32_t* r = res.l;")
    if kind == "sqr":
        temps.append("uint32_t dd[8];")
    ret = "" if inplace else "\n    return res;"
    rtype = "void" if inplace else "F29"
    return """// %s
template <class M>
__device__ __forceinline__ %s %s(%s) {
    constexpr uint32_t inv = R29<M>::INV;
    const uint32_t* P = R29<M>::P;
    %s
    asm(%s
            : %s
            : %s
            : "v0", "v1", "vcc");%s
}
""" % (doc, rtype, name, params, "\n    ".join(temps), body, ",\n              ".join(outs),
       ",\n              ".join(ins), ret)


def main() -> None:
    out = [
        "// GENERATED by tools/gen_prod_asm.py -- do not edit.  Whole radix-2^29 Montgomery products,",
        "// one asm statement each (see the generator's docstring): mul29 / sqr29 / mul29_sum2 of",
        "// field29.h with the same column schedule and results.  Device code only.",
        "#pragma once",
        "",
        "namespace eon {",
        "",
        emit("mul29_asm", "mul", 8, False, "const F29& a, const F29& b",
             "a b 2^-261 mod p (mul29's contract; multipliers m_0..m_7 unmasked)"),
        emit("mul29_asm_ip", "mul", 8, True, "F29& a, const F29& b", "a = a b 2^-261 mod p in place (as mul29_asm)"),
        emit("sqr29_asm", "sqr", 8, False, "const F29& a",
             "a^2 2^-261 mod p (sqr29's contract; cross terms against 2 a_i)"),
        emit("mul29_sum2_asm", "sum2", 6, False, "const F29& a, const F29& b, const F29& c, const F29& d",
             "(a b + c d) 2^-261 mod p (mul29_sum2's contract; m_0..m_5 unmasked)"),
        emit("mul29_sum2_asm_ip", "sum2", 6, True, "const F29& a, const F29& b, F29& c, const F29& d",
             "c = (a b + c d) 2^-261 mod p in place (as mul29_sum2_asm)"),
        "}  // namespace eon",
    ]
    print("\n".join(out))


if __name__ == "__main__":
    main()
