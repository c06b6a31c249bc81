"""plonky3_eon_amd -- MI355X-native prover hot path for the plonky3-eon BN254/KZG stack.

Kernels live in libeonhip.so (csrc/, C ABI include/eon.h); this package is the thin host-side
mirror of the reference's interfaces over that ABI:

* ``dft``   -- TwoAdicSubgroupDft<Fr> (Radix2Dit / Radix2DitParallel), dft/src/traits.rs
* ``field`` -- Fr value formatting for the ABI

There is no CPU fallback: importing an entry point loads libeonhip.so and raises if it is absent.
"""

from . import _lib  # noqa: F401
from .dft import Context, Radix2Dit, Radix2DitParallel, BitReversedMatrix, default_context  # noqa: F401
from ._lib import EonError  # noqa: F401

__all__ = ["Context", "Radix2Dit", "Radix2DitParallel", "BitReversedMatrix", "default_context", "EonError"]
