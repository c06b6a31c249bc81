"""ctypes binding of libeonhip.so (include/eon.h).

The product path is native: if the shared library is missing or fails to load this module
raises -- there is no CPU fallback anywhere in plonky3_eon_amd.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libeonhip.so"

EON_OK = 0
EON_E_SHAPE = -1
EON_E_DEGREE_TOO_LARGE = -2
EON_E_DEVICE = -3
EON_E_OOM = -4
EON_E_ARG = -5
EON_ORDER_NATURAL = 0
EON_ORDER_BITREV = 1
EON_FOURSTEP_NATURAL = 0
EON_FOURSTEP_TRANSPOSED = 1
EON_MSM_PRECOMPUTE = 1
ABI_VERSION = 4  # include/eon.h eon_abi_version(): the layouts below (eon_collective, eon_g2_affine, ...)

_ERRNAMES = {
    EON_E_SHAPE: "EON_E_SHAPE",
    EON_E_DEGREE_TOO_LARGE: "EON_E_DEGREE_TOO_LARGE",
    EON_E_DEVICE: "EON_E_DEVICE",
    EON_E_OOM: "EON_E_OOM",
    EON_E_ARG: "EON_E_ARG",
}


class EonError(RuntimeError):
    """A nonzero return from the C ABI.  The reference panics in these cases."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class eon_fr(ctypes.Structure):
    _fields_ = [("l", ctypes.c_uint64 * 4)]


class eon_poseidon2_constants(ctypes.Structure):
    _fields_ = [("half_full_rounds", ctypes.c_uint32), ("partial_rounds", ctypes.c_uint32),
                ("beginning", ctypes.c_void_p), ("partial", ctypes.c_void_p), ("ending", ctypes.c_void_p)]


class eon_sym_node(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("a", ctypes.c_uint32), ("b", ctypes.c_uint32)]


class eon_air_program_stats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint32) for k in ("width", "num_public_values", "num_constraints",
                                               "max_constraint_degree", "num_instructions", "num_registers",
                                               "num_constants")]


class eon_clock_probe(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("clock_mhz_median", "clock_mhz_min", "clock_mhz_max", "products_per_s",
                                              "ms_per_launch")]


class eon_g1_affine(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint64 * 4), ("y", ctypes.c_uint64 * 4)]


_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_INT = ctypes.c_int

# name -> (restype, argtypes); the full exported surface of include/eon.h
SIGNATURES = {
    "eon_abi_version": (_U32, []),
    "eon_ctx_create": (_INT, [_INT, ctypes.POINTER(_P)]),
    "eon_ctx_destroy": (None, [_P]),
    "eon_last_error": (ctypes.c_char_p, [_P]),
    "eon_ctx_set_stream": (_INT, [_P, _P]),
    "eon_ctx_stream": (_P, [_P]),
    "eon_ctx_device": (_INT, [_P]),
    "eon_ctx_set_collective": (_INT, [_P, _P]),
    "eon_ctx_synchronize": (_INT, [_P]),
    "eon_ctx_trim": (_INT, [_P]),
    "eon_diag_clock_probe": (_INT, [_P, _U32, _U32, _P]),
    "eon_diag_prod_asm_check": (_INT, [_P, _U32, _U32, _P]),
    "eon_ctx_profile": (_INT, [_P, _INT]),
    "eon_ctx_profile_report": (_INT, [_P, ctypes.c_char_p, _U64]),
    "eon_ctx_set_serial": (_INT, [_P, _INT]),
    "eon_fourstep_dft_dev": (_INT, [_P, _P, _P, _U32, _INT, _P]),
    "eon_msm_sharded_dev": (_INT, [_P, _P, _P, _U64, _P, _P]),
    "eon_ctx_serial": (_INT, [_P]),
    "eon_dft_batch": (_INT, [_P, _P, _P, _U64, _U32, _INT]),
    "eon_idft_batch": (_INT, [_P, _P, _P, _U64, _U32]),
    "eon_coset_dft_batch": (_INT, [_P, _P, _P, _U64, _U32, _P, _INT]),
    "eon_coset_idft_batch": (_INT, [_P, _P, _P, _U64, _U32, _P]),
    "eon_coset_lde_batch": (_INT, [_P, _P, _P, _U64, _U32, _U32, _P, _INT]),
    "eon_dft_batch_dev": (_INT, [_P, _P, _P, _U64, _U32, _INT]),
    "eon_idft_batch_dev": (_INT, [_P, _P, _P, _U64, _U32]),
    "eon_coset_dft_batch_dev": (_INT, [_P, _P, _P, _U64, _U32, _P, _INT]),
    "eon_coset_idft_batch_dev": (_INT, [_P, _P, _P, _U64, _U32, _P]),
    "eon_coset_lde_batch_dev": (_INT, [_P, _P, _P, _U64, _U32, _U32, _P, _INT]),
    "eon_coset_dft_padded_batch": (_INT, [_P, _P, _P, _U64, _U32, _U32, _P, _INT]),
    "eon_coset_dft_padded_batch_dev": (_INT, [_P, _P, _P, _U64, _U32, _U32, _P, _INT]),
    "eon_msm_bases_create": (_INT, [_P, _P, _U64, _U32, ctypes.POINTER(_P)]),
    "eon_msm_bases_destroy": (None, [_P]),
    "eon_msm_bases_len": (_U64, [_P]),
    "eon_msm_g1": (_INT, [_P, _P, _P, _U64, _P]),
    "eon_msm_g1_dev": (_INT, [_P, _P, _P, _U64, _P]),
    "eon_g1_multi_exp": (_INT, [_P, _P, _P, _U64, _P]),
    "eon_msm_g1_columns": (_INT, [_P, _P, _P, _U64, _U32, _P]),
    "eon_msm_g1_columns_dev": (_INT, [_P, _P, _P, _U64, _U32, _P]),
    "eon_quotient_and_eval_columns_dev": (_INT, [_P, _P, _U64, _U32, _P, _P, _P]),
    "eon_eval_columns_dev": (_INT, [_P, _P, _U64, _U32, _P, _U32, _P]),
    "eon_msm_g1_columns_prepare_dev": (_INT, [_P, _P, _P, _U64, _U32, _P, ctypes.POINTER(_P)]),
    "eon_msm_g1_columns_prepared": (_INT, [_P, _P, _U32, _P, _P]),
    "eon_msm_scalars_destroy": (None, [_P]),
    "eon_kzg_opening_bases_create": (_INT, [_P, _P, _U64, _P, ctypes.POINTER(_P)]),
    "eon_kzg_opening_bases_create_many": (_INT, [_P, _P, _U64, _P, _U32, _P]),
    "eon_msm_bases_create_dev": (_INT, [_P, _P, _U64, _U32, ctypes.POINTER(_P)]),
    "eon_g1_srs_powers": (_INT, [_P, _P, _U64, _P]),
    "eon_g2_mul": (_INT, [_P, _P, _P, _P]),
    "eon_multi_pairing": (_INT, [_P, _P, _P, _U64, _P]),
    "eon_kzg_verify_batch": (_INT, [_P, _P, _P, _P, _P, _U64, _P, ctypes.POINTER(ctypes.c_int)]),
    "eon_g1_srs_powers_dev": (_INT, [_P, _P, _U64, _P]),
    "eon_selectors_on_coset_dev": (_INT, [_P, _U32, _U32, _P, _P]),
    "eon_p2air_create": (_INT, [_P, _P, _U32, ctypes.POINTER(_P)]),
    "eon_p2air_destroy": (None, [_P]),
    "eon_p2air_width": (_U32, [_P]),
    "eon_p2air_vector_len": (_U32, [_P]),
    "eon_p2air_constraints_per_perm": (_U32, [_P]),
    "eon_p2air_generate_trace_dev": (_INT, [_P, _P, _P, _U64, _P]),
    "eon_p2air_quotient_values_dev": (_INT, [_P, _P, _P, _U32, _U32, _P, _P]),
    "eon_air_program_create": (_INT, [_P, _P, _U32, _P, _U32, _P, _U32, _U32, _U32, ctypes.POINTER(_P)]),
    "eon_air_program_destroy": (None, [_P]),
    "eon_air_program_info": (_INT, [_P, _P]),
    "eon_air_program_log_quotient_degree": (_U32, [_P, _U32]),
    "eon_quotient_values_dev": (_INT, [_P, _P, _P, _U32, _U32, _P, _P, _U32, _P]),
    "eon_fr_lincomb_dev": (_INT, [_P, _P, _U32, _U64, _P, _P]),
    "eon_fourstep_twiddle_pack_dev": (_INT, [_P, _P, _U32, _U32, _U64, _U32, _U32, _P]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load libeonhip.so (once).  Raises if it is absent: the product path never falls back."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ["EON_LIB"]) if os.environ.get("EON_LIB") else LIB_PATH  # tuning variants
    if not path.exists():
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(os.fspath(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.eon_abi_version() != ABI_VERSION:
        raise ImportError(f"{path} has ABI version {lib.eon_abi_version()}, this binding expects {ABI_VERSION} "
                          f"(struct layouts differ): rebuild the library")
    _lib = lib
    return lib
