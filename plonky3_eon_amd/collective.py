"""eon_collective (include/eon.h) from Python: the ctypes struct and a torch.distributed-backed
implementation of its two callbacks.

``TorchCollective(rank, world, group, device)`` all-gathers / all-to-alls device buffers through
torch.distributed over `group`: RCCL on device tensors for the nccl backend, staged through host
memory for gloo (the CPU-hosted multi-rank tests, several ranks sharing one GPU).  The driver's own
RCCL communicator (no Python in the loop) is ``native.RcclCollective``.
"""

from __future__ import annotations

import ctypes

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_INT = ctypes.c_int

# int (*)(void* user, const void* send, void* recv, uint64_t bytes, void* hip_stream)
ALL_GATHER_FN = ctypes.CFUNCTYPE(_INT, _P, _P, _P, _U64, _P)
ALL_TO_ALL_FN = ctypes.CFUNCTYPE(_INT, _P, _P, _P, _U64, _P)


class eon_collective(ctypes.Structure):
    _fields_ = [("rank", _U32), ("world", _U32), ("all_gather", ALL_GATHER_FN), ("user", _P),
                ("all_to_all", ALL_TO_ALL_FN)]


class _DevBytes:
    """A raw device allocation seen as a uint8 torch tensor (zero-copy, __cuda_array_interface__)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2}


class TorchCollective:
    """eon_collective whose all-gather / all-to-all are torch.distributed over `group`."""

    def __init__(self, rank: int, world: int, group=None, device=0):
        self.rank, self.world = rank, world
        self.group = group
        self.device = device

        def wrap(body):
            def fn(user, send, recv, nbytes, stream):
                try:
                    import torch

                    torch.cuda.synchronize(self.device)  # the library's stream has produced `send`
                    body(send, recv, nbytes)
                    torch.cuda.synchronize(self.device)
                    return 0
                except Exception:  # a Python exception must not unwind through the C caller
                    import traceback

                    traceback.print_exc()
                    return 1
            return fn

        def all_gather(send, recv, nbytes):
            import torch

            from .distributed import all_gather_rows

            s = torch.as_tensor(_DevBytes(send, nbytes), device=f"cuda:{self.device}")
            r = torch.as_tensor(_DevBytes(recv, nbytes * world), device=f"cuda:{self.device}")
            r.copy_(all_gather_rows(s, self.group).reshape(-1))

        def all_to_all(send, recv, nbytes):
            import torch

            from .distributed import all_to_all_blocks

            s = torch.as_tensor(_DevBytes(send, nbytes * world), device=f"cuda:{self.device}")
            r = torch.as_tensor(_DevBytes(recv, nbytes * world), device=f"cuda:{self.device}")
            r.copy_(all_to_all_blocks(s.reshape(world, -1), self.group).reshape(-1))

        self._fns = (ALL_GATHER_FN(wrap(all_gather)), ALL_TO_ALL_FN(wrap(all_to_all)))  # keep the thunks alive
        self.c = eon_collective(rank, world, self._fns[0], None, self._fns[1])

    def ref(self):
        return ctypes.byref(self.c)
