"""The C restatement (oracle/eon_oracle.c) under AddressSanitizer + UBSan:
oracle/asan_check.c drives every entry point the tests and the bench's CPU baseline use on small,
ragged and edge shapes with self-consistency checks; any sanitizer report or failed check fails."""

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ORACLE = Path(__file__).resolve().parent.parent / "oracle"


def test_oracle_under_asan_and_ubsan():
    if shutil.which("gcc") is None or shutil.which("make") is None:
        pytest.skip("no host C toolchain")
    b = subprocess.run(["make", "-s", "-C", str(ORACLE), "asan_check"], capture_output=True, text=True)
    assert b.returncode == 0, b.stderr[-3000:]
    # the harness may preload a library ahead of the ASan runtime: do not insist on link order
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="4")
    r = subprocess.run([str(ORACLE / "asan_check")], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "asan_check: ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
