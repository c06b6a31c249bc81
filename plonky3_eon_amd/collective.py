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
    """eon_collective whose all-gather / all-to-all are torch.distributed over `group`.

    Stream-ordered and copy-free: the callback makes the library's stream (`hip_stream`, the
    context's) torch's current stream for the call, so that the collective is ordered after the
    kernels that produced `send` and everything later on that stream is ordered after the
    collective -- no device-wide synchronize.  With the nccl (RCCL) backend the exchange writes
    straight into `recv` (all_gather_into_tensor / all_to_all_single on views of the caller's
    buffers); gloo stages through host memory (the CPU-hosted tests, several ranks per GPU)."""

    def __init__(self, rank: int, world: int, group=None, device=0):
        self.rank, self.world = rank, world
        self.group = group
        self.device = device
        self._streams = {}

        def wrap(body):
            def fn(user, send, recv, nbytes, stream):
                try:
                    import torch

                    dev = torch.device("cuda", self.device)
                    ext = self._streams.get(stream)
                    if ext is None:
                        ext = (torch.cuda.ExternalStream(stream, device=dev) if stream
                               else torch.cuda.default_stream(dev))  # NULL: the device's null stream
                        self._streams[stream] = ext
                    with torch.cuda.stream(ext):
                        body(send, recv, nbytes, dev)
                    return 0
                except Exception:  # a Python exception must not unwind through the C caller
                    import traceback

                    traceback.print_exc()
                    return 1
            return fn

        def nccl(group):
            import torch.distributed as dist

            return dist.get_backend(group) == "nccl"

        def all_gather(send, recv, nbytes, dev):
            import torch
            import torch.distributed as dist

            s = torch.as_tensor(_DevBytes(send, nbytes), device=dev)
            r = torch.as_tensor(_DevBytes(recv, nbytes * world), device=dev)
            if nccl(self.group):
                dist.all_gather_into_tensor(r, s, group=self.group)
            else:
                h = s.cpu()
                parts = [torch.empty_like(h) for _ in range(world)]
                dist.all_gather(parts, h, group=self.group)
                r.copy_(torch.cat(parts))

        def all_to_all(send, recv, nbytes, dev):
            import torch
            import torch.distributed as dist

            s = torch.as_tensor(_DevBytes(send, nbytes * world), device=dev)
            r = torch.as_tensor(_DevBytes(recv, nbytes * world), device=dev)
            if nccl(self.group):
                dist.all_to_all_single(r, s, group=self.group)
            else:
                h = s.cpu()
                hr = torch.empty_like(h)
                dist.all_to_all_single(hr, h, group=self.group)
                r.copy_(hr)

        self._fns = (ALL_GATHER_FN(wrap(all_gather)), ALL_TO_ALL_FN(wrap(all_to_all)))  # keep the thunks alive
        self.c = eon_collective(rank, world, self._fns[0], None, self._fns[1])

    def ref(self):
        return ctypes.byref(self.c)
