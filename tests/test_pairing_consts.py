"""csrc/pairing_consts.h is exactly what tools/pairing_consts.py generates from the definitions
(the generator also asserts the exact base-q decomposition of the final exponentiation's hard part
and the exponent of the addition chain pairing.hip evaluates), and its 2^i G2 table agrees with the
pairing oracle's G2 arithmetic."""

import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_header_matches_generator():
    body = subprocess.run([sys.executable, str(ROOT / "tools" / "pairing_consts.py")], capture_output=True,
                          text=True, check=True).stdout
    header = (ROOT / "plonky3_eon_amd" / "csrc" / "pairing_consts.h").read_text()
    assert body.strip() in header


def test_g2_pow2_table_matches_oracle():
    from oracle import pairing as PO
    from oracle import pyoracle as O

    header = (ROOT / "plonky3_eon_amd" / "csrc" / "pairing_consts.h").read_text()
    table = header.split("G2_POW2[256][2][2][8] = {")[1].split("};")[0]
    words = [int(w.rstrip("u"), 16) for w in table.replace("{", " ").replace("}", " ").replace(",", " ").split()
             if w.startswith("0x")]
    assert len(words) == 256 * 32

    def fq(ws):  # 8 little-endian Montgomery words -> integer
        m = sum(w << (32 * i) for i, w in enumerate(ws))
        return m * pow(1 << 256, -1, O.Q) % O.Q

    p = PO.G2_GEN
    for i in (0, 1, 2, 77, 254, 255):
        ws = words[32 * i:32 * (i + 1)]
        got = ((fq(ws[0:8]), fq(ws[8:16])), (fq(ws[16:24]), fq(ws[24:32])))
        assert got == PO.g2_mul(p, 1 << i), i


def test_g1_pow2_table_matches_oracle():
    from oracle import pyoracle as O

    header = (ROOT / "plonky3_eon_amd" / "csrc" / "pairing_consts.h").read_text()
    table = header.split("G1_POW2[256][2][8] = {")[1].split("};")[0]
    words = [int(w.rstrip("u"), 16) for w in table.replace("{", " ").replace("}", " ").replace(",", " ").split()
             if w.startswith("0x")]
    assert len(words) == 256 * 16

    def fq(ws):
        m = sum(w << (32 * i) for i, w in enumerate(ws))
        return m * pow(1 << 256, -1, O.Q) % O.Q

    for i in (0, 1, 3, 128, 255):
        ws = words[16 * i:16 * (i + 1)]
        assert (fq(ws[0:8]), fq(ws[8:16])) == O.g1_mul((1, 2), 1 << i), i
