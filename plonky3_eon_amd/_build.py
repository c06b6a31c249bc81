"""Builds the two in-tree shared libraries for gfx950:

* libeonhip.so   -- the C-ABI hot path (include/eon.h): the HIP kernels in csrc/*.hip;
* libeonprove.so -- the native prove driver above it (include/eon_prove.h): host C++ in
                    host/*.cpp that calls only eon.h (linked against libeonhip.so, $ORIGIN rpath)
                    and RCCL for the sharded prove's all-gathers.

Each translation unit is compiled with hipcc into build/, then linked.  Objects are rebuilt only
when a source or header is newer.
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
HOST = PKG / "host"
BUILD_HOST = ROOT / "build" / "eonprove"
PROVE_LIB = PKG / "libeonprove.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
         "-I" + str(ROOT / "include")]


def sources():
    return sorted(CSRC.glob("*.hip"))


def _headers_mtime() -> float:
    hs = list(CSRC.glob("*.h")) + list(HOST.glob("*.h")) + list((ROOT / "include").glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, out_dir: Path = BUILD, extra=()) -> Path:
    obj = out_dir / (src.stem + ".o")
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _headers_mtime()):
        return obj
    cmd = [HIPCC, *FLAGS, *extra, "-c", str(src), "-o", str(obj)]
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
    _build_prove_driver()
    if verbose:
        print(f"built {LIB} and {PROVE_LIB}")
    return LIB


def _build_prove_driver() -> Path:
    """libeonprove.so: host C++ only (no kernels); hipcc supplies the HIP runtime headers."""
    BUILD_HOST.mkdir(parents=True, exist_ok=True)
    srcs = sorted(HOST.glob("*.cpp"))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda p: _compile(p, BUILD_HOST, ("-I" + str(HOST),)), srcs))
    newest = max([o.stat().st_mtime for o in objs] + [LIB.stat().st_mtime])
    if not PROVE_LIB.exists() or PROVE_LIB.stat().st_mtime < newest:
        cmd = [HIPCC, "-shared", "-fPIC", *map(str, objs), "-o", str(PROVE_LIB), "-L" + str(PKG), "-leonhip",
               "-lrccl", "-pthread", "-Wl,-rpath,$ORIGIN"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed (libeonprove.so):\n{r.stderr[-6000:]}")
    return PROVE_LIB


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
