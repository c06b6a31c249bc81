"""CPU-side checks of the drop-in boundary: libeonhip.so loads and exports every entry point
include/eon.h declares (no device calls), and the Python mirror declares the same surface."""

import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_functions(header="eon.h"):
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(eon_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["eon_ctx_create", "eon_dft_batch", "eon_idft_batch", "eon_coset_dft_batch",
                 "eon_coset_idft_batch", "eon_coset_lde_batch", "eon_msm_bases_create", "eon_msm_g1",
                 "eon_g1_multi_exp"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    from plonky3_eon_amd import _lib

    if not _lib.LIB_PATH.exists():
        pytest.skip("libeonhip.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.eon_abi_version() >= 1


def test_python_binding_covers_header():
    from plonky3_eon_amd import _lib

    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_context_create_without_gpu_fails_cleanly():
    import ctypes

    from conftest import gpu_available
    from plonky3_eon_amd import _lib

    if gpu_available() or not _lib.LIB_PATH.exists():
        pytest.skip("only meaningful on a host without a GPU")
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.eon_ctx_create(0, ctypes.byref(h)) == _lib.EON_E_DEVICE


def test_no_oracle_in_product_path():
    """The product package never imports or links the oracle."""
    for p in (ROOT / "plonky3_eon_amd").rglob("*"):
        if p.suffix in (".py", ".hip", ".h", ".cpp"):
            assert "oracle" not in p.read_text().replace("no CPU fallback", ""), p


def test_prove_driver_exports_every_declared_symbol():
    """libeonprove.so (the C++ host side above eon.h) loads without a GPU and exports
    include/eon_prove.h; the ctypes table covers the header."""
    from plonky3_eon_amd import _lib, native

    if not _lib.LIB_PATH.exists() or not native.PROVE_LIB_PATH.exists():
        pytest.skip("libraries not built (run __graft_entry__.build())")
    lib = native.load()
    names = declared_functions("eon_prove.h")
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(native.SIGNATURES) == names
    assert lib.eon_prove_abi_version() >= 1


def test_prove_driver_calls_only_the_c_abi():
    """The driver is above the boundary: it includes eon.h / eon_prove.h and its own headers,
    never the kernel sources."""
    for p in (ROOT / "plonky3_eon_amd" / "host").glob("*"):
        text = p.read_text()
        assert "csrc/" not in text and '#include "field.h"' not in text and '#include "context.h"' not in text, p


def test_collective_struct_layout():
    """eon_collective (include/eon.h) as the Python binding lays it out: a Rust / C caller's struct
    must match (rank, world, all_gather, user, all_to_all)."""
    import ctypes

    from plonky3_eon_amd.collective import eon_collective

    offs = [getattr(eon_collective, f).offset for f, _ in eon_collective._fields_]
    assert offs == [0, 4, 8, 16, 24] and ctypes.sizeof(eon_collective) == 32
