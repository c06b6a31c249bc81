"""Round constants of the HorizenLabs Poseidon2 instance for BN254 (t = 3, x^5, R_F = 8, R_P = 56)
from their published generation procedure (the Grain LFSR of the Poseidon paper's parameter
script).  TEST INFRASTRUCTURE ONLY.

The reference tests its Poseidon2Bn254<3> against zkhash's Poseidon2 with these constants
(bn254/src/poseidon2.rs:148-201, `RC3` from the git dependency zkhash, absent here).  Restating the
generation lets the permutation (pyoracle.p2_permute and the driver's host transcript) be checked
against the instance's known-answer vector perm([0, 1, 2]).

Grain LFSR: an 80-bit state initialised with the field type (2 bits: 1 = prime field), the S-box
type (4 bits: 0 = x^alpha), the field size n (12 bits), t (12 bits), R_F (10 bits), R_P (10 bits)
and 30 ones; the feedback bit is s[62] ^ s[51] ^ s[38] ^ s[23] ^ s[13] ^ s[0]; the first 160
bits are discarded; output bits are taken in pairs (a, b): b is emitted when a = 1, the pair is
dropped otherwise.  A constant is n output bits, most significant first, rejected while >= p.
Poseidon2 draws R_F * t + R_P constants: t per full round, one per partial round, in round order.
"""

from __future__ import annotations

from . import pyoracle as O


def _grain(n: int, t: int, r_f: int, r_p: int):
    bits = []
    for v, w in ((1, 2), (0, 4), (n, 12), (t, 12), (r_f, 10), (r_p, 10)):
        bits += [int(c) for c in bin(v)[2:].zfill(w)]
    bits += [1] * 30
    assert len(bits) == 80

    def step():
        nb = bits[62] ^ bits[51] ^ bits[38] ^ bits[23] ^ bits[13] ^ bits[0]
        bits.pop(0)
        bits.append(nb)
        return nb

    for _ in range(160):
        step()
    while True:
        a = step()
        b = step()
        if a:
            yield b


def round_constants(t: int = 3, r_f: int = 8, r_p: int = 56, n: int = 254, p: int = O.P):
    """(begin[r_f/2][t], partial[r_p], end[r_f/2][t]) as canonical ints."""
    g = _grain(n, t, r_f, r_p)

    def draw():
        while True:
            v = 0
            for _ in range(n):
                v = (v << 1) | next(g)
            if v < p:
                return v

    half = r_f // 2
    begin = [[draw() for _ in range(t)] for _ in range(half)]
    partial = [draw() for _ in range(r_p)]
    end = [[draw() for _ in range(t)] for _ in range(half)]
    return begin, partial, end


# perm([0, 1, 2]) of the HorizenLabs Poseidon2 BN254 t = 3 instance (its known-answer test)
KAT_IN = [0, 1, 2]
KAT_OUT = [0x0BB61D24DACA55EEBCB1929A82650F328134334DA98EA4F847F760054F4A3033,
           0x303B6F7C86D043BFCBCC80214F26A30277A15D3F74CA654992DEFE7FF8D03570,
           0x1ED25194542B12EEF8617361C3BA7C52E660B145994427CC86296242CF766EC8]
