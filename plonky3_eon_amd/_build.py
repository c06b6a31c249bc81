"""Builds libeonhip.so (the C-ABI shared library, include/eon.h) in-tree for gfx950.

Each translation unit is compiled with hipcc --offload-arch=gfx950 into build/, then linked
into plonky3_eon_amd/libeonhip.so.  Objects are rebuilt only when a source or header is newer.
"""

from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = ROOT / "build" / "eonhip"
LIB = PKG / "libeonhip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
         "-I" + str(ROOT / "include")]


def sources():
    return sorted(CSRC.glob("*.hip"))


def _headers_mtime() -> float:
    hs = list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path) -> Path:
    obj = BUILD / (src.stem + ".o")
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _headers_mtime()):
        return obj
    cmd = [HIPCC, *FLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    return obj


def build(verbose: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if not LIB.exists() or LIB.stat().st_mtime < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(LIB)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    if verbose:
        print(f"built {LIB}")
    return LIB


def build_variant(name: str, defines: list[str]) -> Path:
    """Tuning builds: every source with extra -D flags -> build/variants/libeonhip_<name>.so, loaded
    instead of the default library when EON_LIB points at it (plonky3_eon_amd/_lib.py)."""
    out_dir = ROOT / "build" / "variants" / name
    out_dir.mkdir(parents=True, exist_ok=True)

    def comp(src: Path) -> Path:
        obj = out_dir / (src.stem + ".o")
        cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines], "-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(comp, sources()))
    lib = ROOT / "build" / "variants" / f"libeonhip_{name}.so"
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(lib)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    return lib


if __name__ == "__main__":
    import sys

    if len(sys.argv) > 2 and sys.argv[1] == "variant":
        print(build_variant(sys.argv[2], sys.argv[3:]))
    else:
        build(verbose=True)
