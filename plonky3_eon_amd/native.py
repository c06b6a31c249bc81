"""ctypes binding of the native prove driver libeonprove.so (include/eon_prove.h).

The driver is the C++ host side above eon.h (plonky3_eon_amd/host/): KzgPcs + prove for the
Poseidon2-AIR, the product host (tests/mirror_prover.py is a test-only Python mirror of the same
orchestration).  Its Proof has prover.Proof's shape, so the two are compared field by field in the tests.

Sharded prove: an eon_collective is either
* ``TorchCollective(group)`` -- a ctypes callback over torch.distributed (gloo stages through host
  memory; used by the CPU-hosted multi-rank tests), or
* ``RcclCollective(rank, world, group)`` -- the driver's own RCCL communicator (ncclAllGather on
  device buffers over xGMI); the 128-byte unique id is broadcast with torch.distributed.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

from . import _lib
from .collective import ALL_GATHER_FN, TorchCollective, eon_collective  # noqa: F401 (re-exported)
from .dft import Context, default_context
from .field import fr_to_abi, fr_unmont
from .proof import Opened, Proof, log_quotient_degree

PROVE_LIB_PATH = Path(__file__).resolve().parent / "libeonprove.so"

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_INT = ctypes.c_int

STAGES = ["commit to trace data", "trace LDE (get_evaluations_on_domain)", "quotient_values",
          "exchange partial quotients", "commit to quotient poly chunks", "open", "assemble columns"]
EON_STAGES = 8

class eon_proof(ctypes.Structure):
    _fields_ = [("trace_commit", _P), ("quotient_commit", _P), ("trace_opened", _P), ("trace_witnesses", _P),
                ("quotient_opened", _P), ("quotient_witnesses", _P), ("degree_bits", _U32),
                ("stage_ms", ctypes.c_double * EON_STAGES)]


# name -> (restype, argtypes): every entry point of include/eon_prove.h
SIGNATURES = {
    "eon_prove_abi_version": (_U32, []),
    "eon_kzg_pcs_create": (_INT, [_P, _U64, _P, ctypes.POINTER(_P)]),
    "eon_kzg_pcs_destroy": (None, [_P]),
    "eon_kzg_pcs_last_error": (ctypes.c_char_p, [_P]),
    "eon_rccl_unique_id": (_INT, [_P]),
    "eon_rccl_collective_init": (_INT, [_U32, _U32, _P, ctypes.POINTER(eon_collective)]),
    "eon_rccl_collective_info": (_INT, [ctypes.POINTER(eon_collective), ctypes.POINTER(ctypes.c_int32),
                                        ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                        ctypes.c_char_p, _U32]),
    "eon_rccl_collective_finalize": (None, [ctypes.POINTER(eon_collective)]),
    "eon_emulated_collective_init": (_INT, [_U32, _U32, ctypes.POINTER(eon_collective)]),
    "eon_prove_p2air": (_INT, [_P, _P, _P, _U64, _P, _P, _U32, ctypes.POINTER(eon_collective),
                               ctypes.POINTER(eon_proof)]),
    "eon_poseidon2_bn254_permute": (_INT, [_P, _P]),
    "eon_g1_to_bytes": (_INT, [_P, _P]),
    "eon_challenger_create": (_INT, [_P, ctypes.POINTER(_P)]),
    "eon_challenger_destroy": (None, [_P]),
    "eon_challenger_observe": (_INT, [_P, _P, _U64]),
    "eon_challenger_observe_g1": (_INT, [_P, _P, _U64]),
    "eon_challenger_sample": (_INT, [_P, _P]),
    "eon_challenger_state": (_INT, [_P, _P]),
    "eon_prove_p2air_fs": (_INT, [_P, _P, _P, _U64, _P, _U32, ctypes.POINTER(eon_collective),
                                  ctypes.POINTER(eon_proof), _P, _P]),
    "eon_prove_air": (_INT, [_P, _P, _P, _U64, _P, _U32, _P, _P, ctypes.POINTER(eon_proof)]),
    "eon_prove_air_fs": (_INT, [_P, _P, _P, _U64, _P, _U32, _P, ctypes.POINTER(eon_proof), _P, _P]),
}

_plib = None


def load() -> ctypes.CDLL:
    """Load libeonprove.so (after libeonhip.so, which it links).  Raises if it is absent."""
    global _plib
    if _plib is not None:
        return _plib
    _lib.load()
    path = Path(os.environ["EON_PROVE_LIB"]) if os.environ.get("EON_PROVE_LIB") else PROVE_LIB_PATH
    if not path.exists():
        raise ImportError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(os.fspath(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _plib = lib
    return lib


class NativeKzgPcs:
    """KzgPcs::new(max_degree, alpha) inside the native driver (SRS and bases on device)."""

    def __init__(self, max_degree: int, alpha: int, ctx: Context | None = None):
        self.ctx = ctx or default_context(0)
        self.lib = load()
        self.max_degree = max_degree
        h = ctypes.c_void_p()
        a = fr_to_abi(alpha)
        self.ctx.check(self.lib.eon_kzg_pcs_create(self.ctx.handle, max_degree, ctypes.byref(a), ctypes.byref(h)))
        self._h = h

    def check(self, rc: int):
        if rc != 0:
            raise _lib.EonError(rc, self.lib.eon_kzg_pcs_last_error(self._h).decode())

    def close(self):
        if getattr(self, "_h", None):
            self.lib.eon_kzg_pcs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RcclInitError(RuntimeError):
    """The RCCL communicator could not be made on every rank; raised on EVERY rank alike, so all of
    them can fall back together (a rank-local failure would leave the others in a collective)."""


class RcclCollective:
    """eon_collective backed by the driver's RCCL communicator.

    Construction is itself collective over the torch process group `group` and ends the same way
    on every rank: rank 0 broadcasts the unique id -- or a failure sentinel when
    eon_rccl_unique_id fails, so the other ranks never wait in a broadcast rank 0 skipped -- every
    rank initialises its communicator, and the ranks then agree on the outcome (an all-gather of
    the init codes).  If any rank failed, every rank finalises the communicator it may have made
    and raises RcclInitError."""

    def __init__(self, rank: int, world: int, group=None):
        import torch.distributed as dist

        self.lib = load()
        self.c = None
        idbuf = (ctypes.c_uint8 * 128)()
        id_rc = 0
        if rank == 0:
            id_rc = self.lib.eon_rccl_unique_id(idbuf)
        if world > 1:
            obj = [bytes(idbuf) if id_rc == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=group)
            if obj[0] is None:
                raise RcclInitError("eon_rccl_unique_id failed on rank 0")
            idbuf = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        elif id_rc != 0:
            raise RcclInitError(f"eon_rccl_unique_id failed ({id_rc})")
        c = eon_collective()
        try:
            rc = self.lib.eon_rccl_collective_init(rank, world, idbuf, ctypes.byref(c))
        except Exception:  # ctypes-level failure: report it to the other ranks like an error code
            rc = -1
        codes = [rc]
        if world > 1:
            codes = [None] * world
            dist.all_gather_object(codes, rc, group=group)
        if any(x != 0 for x in codes):
            if rc == 0:
                self.lib.eon_rccl_collective_finalize(ctypes.byref(c))
            bad = [g for g, x in enumerate(codes) if x != 0]
            raise RcclInitError(f"eon_rccl_collective_init failed on ranks {bad} (codes {[codes[g] for g in bad]})")
        self.c = c

    def info(self) -> dict:
        """ncclCommCount / ncclCommUserRank / ncclCommCuDevice and the device's PCI bus id, as the
        communicator reports them (bench.py's N > 1 line carries these per rank)."""
        n, r, d = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        pci = ctypes.create_string_buffer(64)
        rc = self.lib.eon_rccl_collective_info(ctypes.byref(self.c), ctypes.byref(n), ctypes.byref(r),
                                               ctypes.byref(d), pci, 64)
        if rc != 0:
            raise _lib.EonError(rc, "eon_rccl_collective_info")
        return {"nccl_comm_count": n.value, "nccl_user_rank": r.value, "nccl_cu_device": d.value,
                "nccl_pci_bus_id": pci.value.decode()}

    def close(self):
        if getattr(self, "c", None) is not None and self.c.user:
            self.lib.eon_rccl_collective_finalize(ctypes.byref(self.c))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EmulatedCollective:
    """eon_emulated_collective_init: the exchanges of rank `rank` in a `world`-rank prove emulated
    on one GPU (bench.py --emulate-world): same bytes and stream order, own data in every slot."""

    def __init__(self, rank: int, world: int):
        self.lib = load()
        self.c = eon_collective()
        rc = self.lib.eon_emulated_collective_init(rank, world, ctypes.byref(self.c))
        if rc != 0:
            raise _lib.EonError(rc, "eon_emulated_collective_init")


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc: int, what: str):
    if rc != 0:
        raise _lib.EonError(rc, what)


class Poseidon2Constants:
    """eon_poseidon2_constants over host arrays, the layout Poseidon2Air takes: begin/end
    (half_full_rounds, 3, 4) and partial (partial_rounds, 4) Montgomery u64 limbs."""

    def __init__(self, begin, partial, end):
        self.begin = np.ascontiguousarray(begin, dtype=np.uint64).reshape(-1, 3, 4)
        self.partial = np.ascontiguousarray(partial, dtype=np.uint64).reshape(-1, 4)
        self.end = np.ascontiguousarray(end, dtype=np.uint64).reshape(-1, 3, 4)
        self.c = _lib.eon_poseidon2_constants(self.begin.shape[0], self.partial.shape[0], _p(self.begin),
                                              _p(self.partial), _p(self.end))


def poseidon2_permute(consts: Poseidon2Constants, state) -> np.ndarray:
    """eon_poseidon2_bn254_permute: state = 3 Montgomery Fr (3, 4) u64."""
    s = np.ascontiguousarray(np.asarray(state, dtype=np.uint64).reshape(3, 4)).copy()
    _check(load().eon_poseidon2_bn254_permute(ctypes.byref(consts.c), _p(s)), "eon_poseidon2_bn254_permute")
    return s


def g1_to_bytes(point) -> bytes:
    """eon_g1_to_bytes of one eon_g1_affine (8 u64: x, y Fq Montgomery)."""
    p = np.ascontiguousarray(np.asarray(point, dtype=np.uint64).reshape(8))
    out = (ctypes.c_uint8 * 32)()
    _check(load().eon_g1_to_bytes(_p(p), out), "eon_g1_to_bytes")
    return bytes(out)


class Challenger:
    """DuplexChallenger<Fr, Poseidon2Bn254<3>, 3, 2> of libeonprove (eon_challenger_*)."""

    def __init__(self, consts: Poseidon2Constants):
        self.lib = load()
        self.consts = consts  # the C side copies them; kept for symmetry with the AIR
        h = _P()
        _check(self.lib.eon_challenger_create(ctypes.byref(consts.c), ctypes.byref(h)), "eon_challenger_create")
        self._h = h

    @property
    def handle(self):
        return self._h

    def observe(self, values):
        """Montgomery Fr limbs (..., 4)"""
        v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64).reshape(-1, 4))
        _check(self.lib.eon_challenger_observe(self._h, _p(v), v.shape[0]), "eon_challenger_observe")

    def observe_g1(self, points):
        """eon_g1_affine rows (..., 8)"""
        v = np.ascontiguousarray(np.asarray(points, dtype=np.uint64).reshape(-1, 8))
        _check(self.lib.eon_challenger_observe_g1(self._h, _p(v), v.shape[0]), "eon_challenger_observe_g1")

    def sample(self) -> np.ndarray:
        out = np.zeros(4, np.uint64)
        _check(self.lib.eon_challenger_sample(self._h, _p(out)), "eon_challenger_sample")
        return out

    def state(self) -> np.ndarray:
        out = np.zeros((3, 4), np.uint64)
        _check(self.lib.eon_challenger_state(self._h, _p(out)), "eon_challenger_state")
        return out

    def close(self):
        if getattr(self, "_h", None):
            self.lib.eon_challenger_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def prove_native(air, pcs: NativeKzgPcs, trace, alpha: int | None, zeta: int | None,
                 max_constraint_degree: int = 3, collective=None, challenger: Challenger | None = None,
                 public_values=()) -> Proof:
    """prover.prove through the C++ driver.  `air` is a Poseidon2Air (fused quotient kernel) or an
    air.AirProgram (any AIR, with `public_values`: canonical ints).  `trace`: (N, width, 4) device
    tensor; with a collective (world > 1, Poseidon2 only) `air`/`trace` are this rank's lanes and
    the proof is the full one.  With `challenger` (eon_prove_*_fs) alpha and zeta are sampled from
    the transcript and returned in proof.alpha / proof.zeta (canonical ints); the arguments are
    ignored."""
    from .air import AirProgram, _publics_limbs

    generic = isinstance(air, AirProgram)
    world = collective.c.world if collective is not None else 1
    w = air.width * world
    log_qd = air.log_quotient_degree() if generic else log_quotient_degree(max_constraint_degree)
    chunks = 1 << log_qd
    tc = np.zeros((w, 8), np.uint64)
    qc = np.zeros((chunks, 8), np.uint64)
    to = np.zeros((2, w, 4), np.uint64)
    tw = np.zeros((2, w, 8), np.uint64)
    qo = np.zeros((chunks, 4), np.uint64)
    qw = np.zeros((chunks, 8), np.uint64)
    out = eon_proof(_p(tc), _p(qc), _p(to), _p(tw), _p(qo), _p(qw), 0)
    t = trace.contiguous()
    import torch

    torch.cuda.synchronize(t.device)  # the trace was produced on torch's stream
    pcs.ctx.set_stream(None)
    coll = ctypes.byref(collective.c) if collective is not None else None
    pub = _publics_limbs(public_values)
    npub = len(public_values)
    if not generic and npub:
        raise ValueError("the Poseidon2-AIR has no public values")
    tp = ctypes.c_void_p(t.data_ptr())
    if challenger is None:
        a, z = fr_to_abi(alpha), fr_to_abi(zeta)
        if generic:
            pcs.check(pcs.lib.eon_prove_air(pcs._h, air.handle, tp, int(t.shape[0]), _p(pub), npub, ctypes.byref(a),
                                            ctypes.byref(z), ctypes.byref(out)))
        else:
            pcs.check(pcs.lib.eon_prove_p2air(pcs._h, air.handle, tp, int(t.shape[0]), ctypes.byref(a),
                                              ctypes.byref(z), max_constraint_degree, coll, ctypes.byref(out)))
    else:
        a_out, z_out = np.zeros(4, np.uint64), np.zeros(4, np.uint64)
        if generic:
            if collective is not None:
                raise ValueError("the generic AIR path is not lane-sharded")
            pcs.check(pcs.lib.eon_prove_air_fs(pcs._h, air.handle, tp, int(t.shape[0]), _p(pub), npub,
                                               challenger.handle, ctypes.byref(out), _p(a_out), _p(z_out)))
        else:
            pcs.check(pcs.lib.eon_prove_p2air_fs(pcs._h, air.handle, tp, int(t.shape[0]), challenger.handle,
                                                 max_constraint_degree, coll, ctypes.byref(out), _p(a_out),
                                                 _p(z_out)))
        alpha = fr_unmont(sum(int(v) << (64 * i) for i, v in enumerate(a_out)))
        zeta = fr_unmont(sum(int(v) << (64 * i) for i, v in enumerate(z_out)))
    opened_trace = Opened(values=[[to[0], to[1]]], witnesses=[[tw[0], tw[1]]])
    opened_quot = Opened(values=[[qo[c:c + 1]] for c in range(chunks)], witnesses=[[qw[c:c + 1]] for c in range(chunks)])
    timings = {name: out.stage_ms[i] for i, name in enumerate(STAGES)}
    if collective is None:
        timings.pop("exchange partial quotients")
        timings.pop("assemble columns")
    return Proof([tc], [qc[c:c + 1] for c in range(chunks)], [opened_trace, opened_quot], out.degree_bits, timings,
                 alpha, zeta)
