"""Multi-GPU hot path: one process per GPU, torch.distributed (backend "nccl" =
RCCL over xGMI on the MI355X node; "gloo" for the CPU tests and for several ranks sharing one
GPU).  Three shardings:

* the eon-uni-stark prove split by vector lane (below; the C++ driver's `eon_prove_p2air(_fs)` with
  an eon_collective, and the test-only Python mirror `tests/mirror_prover.prove(..., shard=)`);
* a single large forward DFT as a four-step N1 x N2 transform with one all_to_all
  (`fourstep_dft`, BASELINE configs[4] (i));
* an MSM split by point range with an all-gather of per-rank partial points
  (`msm_sharded`, configs[4] (ii)).

Lane-sharded prove:

The sharding is SURVEY.md 8(e)'s preferred scheme for the vectorized Poseidon2-AIR.  The AIR
evaluates its VECTOR_LEN lanes one after another (poseidon2-air/src/vectorized.rs:259-274), so
lane v owns trace columns [164 v, 164 v + 164) and constraints [160 v, 160 v + 160).  Rank g
owns a contiguous lane range [l0, l1):

* trace commit  -- coset_idft + column MSMs of its own columns (kzg/src/pcs.rs:223-265); no
                   exchange.
* quotient      -- its LDE columns (pcs.rs:267-287) and the partial folder accumulator over its
                   lanes (prover.rs:539-709).  The folder's running sum
                   sum_k alpha^(K-1-k) C_k (folder.rs:81-85) splits by lane: lane v's block is
                   weighted alpha^(K_lane (VL-1-v)).  A VectorizedPoseidon2Air over the rank's
                   l1 - l0 lanes weights its local lane v' by alpha^(K_lane (l1-l0-1-v')), so the
                   rank's partial times alpha^(K_lane (VL - l1)) is its exact share.  Every rank
                   all-gathers the partials (Q x 32 B each), the only data-path collective, and
                   combines them on device (eon_fr_lincomb_dev): mod-p sums are not an RCCL
                   reduction.  inv_vanishing is applied per partial and distributes over the sum.
* quotient commit and its opening -- 2 chunks x 1 column, replicated on every rank (identical
                   inputs, identical results).
* trace open    -- its columns at [zeta, zeta h] (pcs.rs:289-335); no exchange.
* assembly      -- one all-gather of the per-column results (commitment, 2 values,
                   2 witnesses): 32 u64 per column.

Every rank ends with the same Proof, equal to the single-GPU prove's.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .field import FR_MODULUS, fr_to_abi


@dataclass(frozen=True)
class Shard:
    """This rank's lanes of a VectorizedPoseidon2Air with `vector_len` lanes."""

    rank: int
    world: int
    vector_len: int
    group: object = None

    @property
    def lanes(self):
        return lane_range(self.rank, self.world, self.vector_len)

    def columns(self, cols_per_lane: int):
        l0, l1 = self.lanes
        return l0 * cols_per_lane, l1 * cols_per_lane


def lane_range(rank: int, world: int, vector_len: int):
    """Contiguous lane block of `rank`; every rank gets vector_len / world lanes."""
    if world < 1 or not 0 <= rank < world:
        raise _lib.EonError(_lib.EON_E_ARG, f"rank {rank} outside world {world}")
    if vector_len % world:
        raise _lib.EonError(_lib.EON_E_SHAPE, f"VECTOR_LEN {vector_len} does not split over {world} ranks")
    per = vector_len // world
    return rank * per, (rank + 1) * per


def lane_weights(alpha: int, vector_len: int, world: int, constraints_per_lane: int):
    """alpha^(K_lane (VL - l1_g)) for every rank g: the factor turning rank g's local folder
    accumulator into its share of the full one."""
    a = alpha % FR_MODULUS
    return [pow(a, constraints_per_lane * (vector_len - lane_range(g, world, vector_len)[1]), FR_MODULUS)
            for g in range(world)]


def all_gather_rows(t, group=None):
    """Stack `t` from every rank in rank order -> (world, *t.shape), on t's device.

    nccl (RCCL) gathers device buffers directly; other backends (gloo) stage through host
    memory, which is how the CPU tests and a several-ranks-per-GPU run exchange."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    t = t.contiguous()
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=group)
        return out
    h = t.cpu()
    parts = [torch.empty_like(h) for _ in range(world)]
    dist.all_gather(parts, h, group=group)
    return torch.stack(parts).to(t.device)


def combine_partials(ctx, parts, weights):
    """sum_g weights[g] * parts[g] over Fr on device: parts (G, Q, 4) int64 -> (Q, 4)."""
    import torch

    g, q = int(parts.shape[0]), int(parts.shape[1])
    if len(weights) != g:
        raise _lib.EonError(_lib.EON_E_SHAPE, "one weight per partial")
    out = torch.empty((q, 4), dtype=torch.int64, device=parts.device)
    coeffs = (_lib.eon_fr * g)(*[fr_to_abi(w) for w in weights])
    p = parts.contiguous()
    ctx.set_stream(torch.cuda.current_stream(p.device).cuda_stream)
    ctx.check(ctx.lib.eon_fr_lincomb_dev(ctx.handle, ctypes.c_void_p(p.data_ptr()), g, q, coeffs,
                                         ctypes.c_void_p(out.data_ptr())))
    return out


# per-column record exchanged at assembly: commitment (8) | value at zeta (4) | value at zeta h (4)
# | witness at zeta (8) | witness at zeta h (8)
COLUMN_RECORD = 32


def pack_columns(commit, values, witnesses) -> np.ndarray:
    return np.concatenate([commit, values[0], values[1], witnesses[0], witnesses[1]], axis=1).astype(np.uint64)


def unpack_columns(rec: np.ndarray):
    rec = rec.reshape(-1, COLUMN_RECORD)
    return rec[:, 0:8], [rec[:, 8:12], rec[:, 12:16]], [rec[:, 16:24], rec[:, 24:32]]


def gather_columns(local: np.ndarray, device, group=None) -> np.ndarray:
    """All-gather the (w_local, 32) per-column records -> (W, 32) in global column order."""
    import torch

    t = torch.from_numpy(np.ascontiguousarray(local).view(np.int64)).to(device)
    return all_gather_rows(t, group).cpu().numpy().view(np.uint64).reshape(-1, COLUMN_RECORD)


# ---- four-step NTT across ranks (BASELINE configs[4]) -----------------------------

def all_to_all_blocks(send, group=None):
    """send: (world, ...) -> recv with recv[g] = rank g's send[this rank] (RCCL all_to_all over
    xGMI for nccl; staged through host memory for gloo)."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send.contiguous(), group=group)
        return recv
    h = send.contiguous().cpu()
    recv = torch.empty_like(h)
    dist.all_to_all_single(recv, h, group=group)
    return recv.to(send.device)


def fourstep_split(log_n: int):
    """N = N1 N2 with N1 = 2^ceil(log_n / 2)."""
    log_n1 = (log_n + 1) // 2
    return log_n1, log_n - log_n1


def fourstep_dft(ctx, local, log_n: int, rank: int = 0, world: int = 1, group=None, natural: bool = False,
                 collective=None):
    """Forward DFT of length N = 2^log_n (Radix2Dit natural order, dft/src/traits.rs:27-61) split
    over `world` ranks as a four-step N1 x N2 transform: eon_fourstep_dft_dev (include/eon.h).

    local: this rank's (N1, N2/world, 4) int64 device block -- columns [rank C, (rank+1) C) of the
    N1 x N2 view M[i1][i2] = x[N2 i1 + i2].  Returns (natural=False) the (N2, N1/world, 4) block of
    the N2 x N1 view of X: out[k2][k1'] = X[N1 k2 + rank N1/world + k1'] -- one all_to_all -- or
    (natural=True) the rank's contiguous slice X[rank N/world, (rank+1) N/world) as (N/world, 4),
    after a second all_to_all.  `collective`: an eon_collective provider (TorchCollective over
    `group` by default, or native.RcclCollective)."""
    import torch

    log_n1, log_n2 = fourstep_split(log_n)
    n1, n2 = 1 << log_n1, 1 << log_n2
    cols = n2 // world
    if n2 % world or n1 % world:
        raise _lib.EonError(_lib.EON_E_SHAPE, f"2^{log_n} does not split over {world} ranks")
    if tuple(local.shape[:2]) != (n1, cols):
        raise _lib.EonError(_lib.EON_E_SHAPE, f"local block must be ({n1}, {cols}, 4)")
    local = local.contiguous()
    ctx.set_stream(torch.cuda.current_stream(local.device).cuda_stream)
    coll = None
    if world > 1:
        from .collective import TorchCollective

        coll = collective or TorchCollective(rank, world, group, local.device.index)
    shape = ((n1 * n2) // world, 4) if natural else (n2, n1 // world, 4)
    out = torch.empty(shape, dtype=torch.int64, device=local.device)
    layout = _lib.EON_FOURSTEP_NATURAL if natural else _lib.EON_FOURSTEP_TRANSPOSED
    ctx.check(ctx.lib.eon_fourstep_dft_dev(ctx.handle, ctypes.c_void_p(local.data_ptr()),
                                           ctypes.c_void_p(out.data_ptr()), log_n, layout,
                                           ctypes.byref(coll.c) if coll is not None else None))
    return out


def fourstep_scatter(x, log_n: int, rank: int, world: int):
    """The rank's input block of a natural-order vector x (N, 4): columns [rank C, (rank+1) C) of
    the N1 x N2 view."""
    log_n1, log_n2 = fourstep_split(log_n)
    c = (1 << log_n2) // world
    return x.reshape(1 << log_n1, 1 << log_n2, 4)[:, rank * c:(rank + 1) * c]


def fourstep_gather_index(log_n: int, rank: int, world: int):
    """Natural indices of X held by the rank's output block (N2, N1/world), row-major."""
    log_n1, log_n2 = fourstep_split(log_n)
    n1, n2 = 1 << log_n1, 1 << log_n2
    per = n1 // world
    k2 = np.arange(n2, dtype=np.int64)[:, None]
    k1 = rank * per + np.arange(per, dtype=np.int64)[None, :]
    return (n1 * k2 + k1).reshape(-1)


# ---- MSM sharded by point range (BASELINE configs[4] (ii)) -----------------------

def shard_range(n: int, rank: int, world: int):
    """Contiguous scalar / base range of `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def msm_sharded(bases, scalars_local, device, group=None, collective=None):
    """sum_i s_i P_i over every rank's range: eon_msm_sharded_dev (include/eon.h) -- a full
    Pippenger per rank on its contiguous range (`bases` = MsmBases over that range), an all-gather
    of the G affine partial points and their sum by EC additions (RCCL reductions cannot add curve
    points).  Returns the (8,) affine result (u64 limbs) on every rank."""
    import torch
    import torch.distributed as dist

    from .collective import TorchCollective

    ctx = bases.ctx
    dev = torch.device(device)
    s = torch.as_tensor(np.ascontiguousarray(scalars_local).view(np.int64)) if isinstance(scalars_local, np.ndarray) \
        else scalars_local
    s = s.reshape(-1, 4).contiguous().to(dev)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    coll = None
    if world > 1:
        coll = collective or TorchCollective(dist.get_rank(group), world, group, dev.index or 0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    out = (_lib.eon_g1_affine)()
    ctx.check(ctx.lib.eon_msm_sharded_dev(ctx.handle, bases._h, ctypes.c_void_p(s.data_ptr()), int(s.shape[0]),
                                          ctypes.byref(coll.c) if coll is not None else None, ctypes.byref(out)))
    return np.array(list(out.x) + list(out.y), dtype=np.uint64)
