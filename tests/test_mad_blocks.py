"""CPU: plonky3_eon_amd/csrc/mad_blocks.h is exactly what tools/gen_mad_blocks.py generates (the
multiply-add column blocks of field29.h's madcol are generated code, never edited by hand)."""

import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_mad_blocks_header_is_generated():
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "gen_mad_blocks.py")], check=True,
                         capture_output=True, text=True).stdout
    assert out == (ROOT / "plonky3_eon_amd" / "csrc" / "mad_blocks.h").read_text()


def test_mad_blocks_early_clobber_outputs():
    # the accumulator and the carry-out pair are written before the block's last inputs are read
    text = (ROOT / "plonky3_eon_amd" / "csrc" / "mad_blocks.h").read_text()
    assert '"=s"(c)' not in text and text.count('"=&s"(c)') == text.count("struct MadAsm<")
    assert '"=v"(acc)' not in text
