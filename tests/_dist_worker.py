"""One rank of the lane-sharded prove tests (launched by test_distributed_*.py as a subprocess,
RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment, backend gloo).

  cpu  -- the sharding arithmetic and exchange with the C restatement oracle as the per-rank
          compute: per-lane trace slices, partial quotients, all_gather_rows, lane weights and
          gather_columns must reproduce the single-process oracle quotient.
  gpu  -- the product path (tests/mirror_prover.prove with a Shard) on cuda:0 for every rank;
          rank 0 also runs the unsharded prove and every proof field must match bit for bit.
  a2a  -- all_to_all_blocks layout, and the four-step decomposition with oracle DFTs standing in
          for the kernels (CPU).
  fourstep / msmshard -- the product four-step DFT and the point-range-sharded MSM on cuda:0,
          against the oracle's full-length DFT / MSM.
  native -- the C++ prove driver (libeonprove.so) sharded over the ranks with a torch.distributed
          eon_collective; rank 0 compares it with the driver's unsharded prove and the Python
          prover's.
  openshard -- KZG opening bases built by every rank alone and then sharded over the ranks
          (eon_ctx_set_collective) at the headline height 2^17: the witnesses must agree.

Writes {"ok": true} or {"ok": false, "why": ...} as JSON to argv[2].
"""

import json
import os
import sys
import traceback
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

from oracle import coracle as C  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

HF, PR, CPP = 4, 56, 164


def lim(x):
    return np.array(O.int_to_limbs(O.to_mont(x % O.P)), dtype=np.uint64)


def val(limbs):
    return O.from_mont(O.limbs_to_int([int(x) for x in limbs]))


def consts():
    py = O.p2_constants(2024, HF, PR)
    return C.P2Constants([[lim(x) for x in r] for r in py[0]], [lim(x) for x in py[1]],
                         [[lim(x) for x in r] for r in py[2]])


def lane_inputs(inputs, n, vl, l0, l1):
    """Permutation j sits at row j / VECTOR_LEN, lane j % VECTOR_LEN (generation.rs:14-72)."""
    return np.ascontiguousarray(inputs.reshape(n, vl, 3, 4)[:, l0:l1]).reshape(-1, 3, 4)


def run_cpu(rank, world, group):
    import torch

    from plonky3_eon_amd import distributed as D

    log_n, vl, log_qd = 3, 4, 1
    n = 1 << log_n
    k = consts()
    alpha = 0x1234567890ABCDEF1234
    inputs = C.random_fr(77, n * vl * 3).reshape(n * vl, 3, 4)
    full = C.p2_generate_trace(inputs, vl, k)
    l0, l1 = D.lane_range(rank, world, vl)
    c0, c1 = D.Shard(rank, world, vl).columns(CPP)
    local = C.p2_generate_trace(lane_inputs(inputs, n, vl, l0, l1), l1 - l0, k)
    if not np.array_equal(local, full[:, c0:c1]):
        return "lane trace != column slice of the full trace"

    def quotient(tr, lanes):
        lde = C.kzg_evaluations_on_domain(C.idft_batch(tr), log_n + log_qd, lim(O.GENERATOR))
        return C.p2_quotient_values(lde, log_n, log_qd, lanes, k, lim(alpha))

    part = quotient(local, l1 - l0)
    parts = D.all_gather_rows(torch.from_numpy(part.view(np.int64)), group).numpy().view(np.uint64)
    w = D.lane_weights(alpha, vl, world, 12 * HF + 2 * PR)
    got = [sum(w[g] * val(parts[g, i]) for g in range(world)) % O.P for i in range(parts.shape[1])]
    want = quotient(full, vl)
    if got != [val(x) for x in want]:
        return "combined partial quotients != full quotient"
    # assembly order: each rank's records land at its global columns
    rec = np.zeros((c1 - c0, D.COLUMN_RECORD), dtype=np.uint64)
    rec[:, 0] = np.arange(c0, c1)
    rec[:, 31] = rank
    allrec = D.gather_columns(rec, "cpu", group)
    if not (np.array_equal(allrec[:, 0], np.arange(vl * CPP))
            and np.array_equal(allrec[:, 31], np.repeat(np.arange(world), (vl // world) * CPP))):
        return "gather_columns order"
    return None


def run_gpu(rank, world, group):
    import torch

    from plonky3_eon_amd import Context
    from plonky3_eon_amd import distributed as D
    from plonky3_eon_amd.air import Poseidon2Air
    from mirror_kzg import GpuKzgPcs
    from mirror_prover import prove

    log_n, vl = int(os.environ.get("EON_T_LOG_N", "5")), int(os.environ.get("EON_T_VL", "4"))
    n = 1 << log_n
    k = consts()
    ctx = Context(0)
    dev = torch.device("cuda:0")
    inputs = C.random_fr(99, n * vl * 3).reshape(n * vl, 3, 4)
    alpha, zeta = 0x1234567890ABCDEF1234, 0xFEDCBA0987654321
    pcs = GpuKzgPcs(n, 12345, ctx)
    shard = D.Shard(rank, world, vl, group)
    l0, l1 = shard.lanes
    air = Poseidon2Air(k.begin, k.partial, k.end, l1 - l0, ctx)
    trace = air.generate_trace(torch.from_numpy(lane_inputs(inputs, n, vl, l0, l1).view(np.int64)).to(dev))
    p = prove(air, pcs, trace, alpha, zeta, shard=shard)
    if rank != 0:
        return None
    full_air = Poseidon2Air(k.begin, k.partial, k.end, vl, ctx)
    full = full_air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to(dev))
    q = prove(full_air, pcs, full, alpha, zeta)
    checks = [("trace_commit", p.trace_commit[0], q.trace_commit[0])]
    checks += [(f"quotient_commit[{c}]", p.quotient_commit[c], q.quotient_commit[c]) for c in range(2)]
    for r in range(2):
        for m in range(len(q.opened[r].values)):
            for pt in range(len(q.opened[r].values[m])):
                checks.append((f"opened[{r}].values[{m}][{pt}]", p.opened[r].values[m][pt], q.opened[r].values[m][pt]))
                checks.append((f"opened[{r}].witnesses[{m}][{pt}]", p.opened[r].witnesses[m][pt],
                               q.opened[r].witnesses[m][pt]))
    for name, a, b in checks:
        if not np.array_equal(np.asarray(a), np.asarray(b)):
            return f"{name} differs from the unsharded prove"
    return None


def _proof_fields(p):
    out = [("trace_commit", p.trace_commit[0])]
    out += [(f"quotient_commit[{c}]", p.quotient_commit[c]) for c in range(len(p.quotient_commit))]
    for r in range(2):
        for m in range(len(p.opened[r].values)):
            for pt in range(len(p.opened[r].values[m])):
                out.append((f"opened[{r}].values[{m}][{pt}]", p.opened[r].values[m][pt]))
                out.append((f"opened[{r}].witnesses[{m}][{pt}]", p.opened[r].witnesses[m][pt]))
    return out


def run_native(rank, world, group):
    import torch

    from plonky3_eon_amd import Context
    from plonky3_eon_amd import distributed as D
    from plonky3_eon_amd.air import Poseidon2Air
    from mirror_kzg import GpuKzgPcs
    from plonky3_eon_amd.native import Challenger, NativeKzgPcs, Poseidon2Constants, TorchCollective, prove_native
    from mirror_prover import prove

    log_n, vl = int(os.environ.get("EON_T_LOG_N", "5")), int(os.environ.get("EON_T_VL", "4"))
    n = 1 << log_n
    k = consts()
    ctx = Context(0)
    dev = torch.device("cuda:0")
    inputs = C.random_fr(98, n * vl * 3).reshape(n * vl, 3, 4)
    alpha, zeta = 0x1234567890ABCDEF1234, 0xFEDCBA0987654321
    npcs = NativeKzgPcs(n, 12345, ctx)
    l0, l1 = D.lane_range(rank, world, vl)
    air = Poseidon2Air(k.begin, k.partial, k.end, l1 - l0, ctx)
    trace = air.generate_trace(torch.from_numpy(lane_inputs(inputs, n, vl, l0, l1).view(np.int64)).to(dev))
    p = prove_native(air, npcs, trace, alpha, zeta, collective=TorchCollective(rank, world, group))
    # the Fiat-Shamir transcript: every rank observes the full (all-gathered) trace commitment
    pyc = O.p2_constants(99, 2, 22)
    ck = Poseidon2Constants([[lim(x) for x in r] for r in pyc[0]], [lim(x) for x in pyc[1]],
                            [[lim(x) for x in r] for r in pyc[2]])
    pf = prove_native(air, npcs, trace, None, None, collective=TorchCollective(rank, world, group),
                      challenger=Challenger(ck))
    if rank != 0:
        return None
    full_air = Poseidon2Air(k.begin, k.partial, k.end, vl, ctx)
    full = full_air.generate_trace(torch.from_numpy(inputs.view(np.int64)).to(dev))
    q = prove_native(full_air, npcs, full, alpha, zeta)
    r = prove(full_air, GpuKzgPcs(n, 12345, ctx), full, alpha, zeta)
    for (name, a), (_, b), (_, c) in zip(_proof_fields(p), _proof_fields(q), _proof_fields(r)):
        if not np.array_equal(np.asarray(a), np.asarray(b)):
            return f"{name}: sharded native prove differs from the unsharded one"
        if not np.array_equal(np.asarray(b), np.asarray(c)):
            return f"{name}: native prove differs from the Python prover"
    qf = prove_native(full_air, npcs, full, None, None, challenger=Challenger(ck))
    if (pf.alpha, pf.zeta) != (qf.alpha, qf.zeta):
        return "sharded Fiat-Shamir transcript differs from the unsharded one"
    for (name, a), (_, b) in zip(_proof_fields(pf), _proof_fields(qf)):
        if not np.array_equal(np.asarray(a), np.asarray(b)):
            return f"{name}: sharded Fiat-Shamir prove differs from the unsharded one"
    return None


def _tw_pack(y, log_n, log_n1, col0, parts):
    """The documented contract of eon_fourstep_twiddle_pack_dev, in Python ints (test only)."""
    n1, cols = y.shape[0], y.shape[1]
    w = O.two_adic_generator(log_n)
    per = n1 // parts
    send = np.zeros((parts, cols, per, 4), dtype=np.uint64)
    for k1 in range(n1):
        for i2 in range(cols):
            z = val(y[k1, i2]) * pow(w, (col0 + i2) * k1, O.P) % O.P
            send[k1 // per, i2, k1 % per] = lim(z)
    return send


def run_a2a(rank, world, group):
    import torch

    from plonky3_eon_amd import distributed as D

    send = torch.zeros((world, 3, 2), dtype=torch.int64)
    for h in range(world):
        send[h, :, 0] = rank
        send[h, :, 1] = h
    recv = D.all_to_all_blocks(send, group)
    for g in range(world):
        if not (bool((recv[g, :, 0] == g).all()) and bool((recv[g, :, 1] == rank).all())):
            return "all_to_all_blocks layout"
    for log_n in (6, 7):
        n = 1 << log_n
        log_n1, log_n2 = D.fourstep_split(log_n)
        x = C.random_fr(log_n, n).reshape(n, 4)
        local = np.ascontiguousarray(D.fourstep_scatter(x, log_n, rank, world))
        y = C.dft_batch(local)
        send = _tw_pack(y, log_n, log_n1, rank * local.shape[1], world)
        recv = D.all_to_all_blocks(torch.from_numpy(send.view(np.int64)), group).numpy().view(np.uint64)
        out = C.dft_batch(np.ascontiguousarray(recv.reshape(1 << log_n2, -1, 4)))
        want = C.dft_batch(x.reshape(n, 1, 4)).reshape(n, 4)
        if not np.array_equal(out.reshape(-1, 4), want[D.fourstep_gather_index(log_n, rank, world)]):
            return f"four-step decomposition at 2^{log_n}"
    return None


def run_fourstep(rank, world, group):
    import torch

    from plonky3_eon_amd import Context
    from plonky3_eon_amd import distributed as D

    ctx = Context(0)
    for log_n in (10, 11):
        n = 1 << log_n
        x = C.random_fr(log_n + 40, n).reshape(n, 4)
        local = torch.from_numpy(np.ascontiguousarray(D.fourstep_scatter(x, log_n, rank, world)).view(np.int64))
        full = C.dft_batch(x.reshape(n, 1, 4)).reshape(n, 4)
        # one all_to_all: the rank's block of the N2 x N1 view
        out = D.fourstep_dft(ctx, local.to("cuda:0"), log_n, rank, world, group)
        got = out.cpu().numpy().view(np.uint64).reshape(-1, 4)
        if not np.array_equal(got, full[D.fourstep_gather_index(log_n, rank, world)]):
            return f"four-step DFT 2^{log_n} rank {rank}/{world} (transposed layout)"
        # second all_to_all: the rank's contiguous natural slice
        out = D.fourstep_dft(ctx, local.to("cuda:0"), log_n, rank, world, group, natural=True)
        got = out.cpu().numpy().view(np.uint64).reshape(-1, 4)
        per = n // world
        if not np.array_equal(got, full[rank * per:(rank + 1) * per]):
            return f"four-step DFT 2^{log_n} rank {rank}/{world} (natural layout)"
    return None


def run_msmshard(rank, world, group):
    from plonky3_eon_amd import Context
    from plonky3_eon_amd import distributed as D
    from plonky3_eon_amd.msm import MsmBases

    ctx = Context(0)
    n = 3000
    srs = C.g1_srs(n, C.fr_from_u64(777))
    s = C.random_fr(5, n).reshape(n, 4)
    lo, hi = D.shard_range(n, rank, world)
    bases = MsmBases(np.ascontiguousarray(srs[lo:hi]), ctx, precompute=True)
    got = D.msm_sharded(bases, np.ascontiguousarray(s[lo:hi]), "cuda:0", group)
    if not np.array_equal(np.asarray(got).reshape(8), C.g1_msm(srs, s)):
        return "sharded MSM != full MSM"
    return None


def _device_fr(n, seed, dev):
    """n pseudo-random canonical Fr limbs (n, 4) generated on `dev` from a fixed seed, identical on
    every rank (top limb < 2^60 < p's, so every value is < p)."""
    import torch

    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    x = torch.randint(-(1 << 63), (1 << 63) - 1, (n, 4), generator=g, device=dev, dtype=torch.int64)
    x[:, 3] &= (1 << 60) - 1
    return x


def run_fourstep_full(rank, world, group):
    """BASELINE configs[4] (i) at full size: the 2^26 four-step DFT split over `world` ranks, both
    output layouts, against the world-1 eon_fourstep_dft_dev output and the single-network DFT."""
    import torch

    from plonky3_eon_amd import Context
    from plonky3_eon_amd import _lib as L
    from plonky3_eon_amd import distributed as D

    import ctypes

    ctx = Context(0)
    dev = torch.device("cuda:0")
    log_n = int(os.environ.get("EON_T_LOG_N", "26"))
    n = 1 << log_n
    log_n1, log_n2 = D.fourstep_split(log_n)
    n1, n2 = 1 << log_n1, 1 << log_n2
    x = _device_fr(n, 2026, dev)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    # world-1 references on this rank: the four-step with no collective and the one-network DFT
    ref4 = torch.empty_like(x)
    ctx.check(ctx.lib.eon_fourstep_dft_dev(ctx.handle, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(ref4.data_ptr()),
                                           log_n, L.EON_FOURSTEP_NATURAL, None))
    ref1 = torch.empty_like(x)
    ctx.check(ctx.lib.eon_dft_batch_dev(ctx.handle, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(ref1.data_ptr()),
                                        n, 1, L.EON_ORDER_NATURAL))
    torch.cuda.synchronize()
    if not torch.equal(ref4, ref1):
        return "world-1 four-step != single-network DFT"
    del ref1
    cols = n2 // world
    local = x.view(n1, n2, 4)[:, rank * cols:(rank + 1) * cols].contiguous()
    del x
    out = D.fourstep_dft(ctx, local, log_n, rank, world, group)  # one all_to_all
    per = n1 // world
    want = ref4.view(n2, n1, 4)[:, rank * per:(rank + 1) * per]
    if not torch.equal(out, want):
        return f"2^{log_n} four-step, transposed layout, rank {rank}/{world} != world-1 output"
    del out
    out = D.fourstep_dft(ctx, local, log_n, rank, world, group, natural=True)  # two all_to_alls
    if not torch.equal(out, ref4[rank * (n // world):(rank + 1) * (n // world)]):
        return f"2^{log_n} four-step, natural layout, rank {rank}/{world} != world-1 output"
    return None


def run_msmshard_full(rank, world, group):
    """BASELINE configs[4] (ii) at full size: the 2^24-term MSM over the alpha = 12345 SRS split by
    point range over `world` ranks (eon_msm_sharded_dev) == [f(alpha)] G."""
    import torch

    from plonky3_eon_amd import Context
    from plonky3_eon_amd import distributed as D
    from plonky3_eon_amd.msm import MsmBases, srs_powers

    ctx = Context(0)
    dev = torch.device("cuda:0")
    log_n = int(os.environ.get("EON_T_LOG_N", "24"))
    n = 1 << log_n
    lo, hi = D.shard_range(n, rank, world)
    srs = srs_powers(n, 12345, ctx)
    bases = MsmBases(np.ascontiguousarray(srs[lo:hi]), ctx, precompute=True)
    del srs
    s = _device_fr(n, 2424, dev)
    got = D.msm_sharded(bases, s[lo:hi].contiguous(), "cuda:0", group)
    bases.close()
    if rank != 0:
        return None
    sh = s.cpu().numpy().view(np.uint64).reshape(n, 1, 4)
    f_alpha = C.eval_poly_col(sh, 0, C.fr_from_u64(12345))
    if not np.array_equal(np.asarray(got).reshape(8), C.g1_mul(C.g1_generator(), f_alpha)):
        return f"2^{log_n} MSM sharded over {world} ranks != [f(alpha)]G"
    return None


def run_openshard(rank, world, group):
    import ctypes

    import torch

    from plonky3_eon_amd import Context
    from plonky3_eon_amd.msm import MsmBases, srs_powers
    from plonky3_eon_amd.native import TorchCollective

    ctx = Context(0)
    n, width = 1 << 17, 3
    srs = MsmBases(srs_powers(n + 1, 12345, ctx), ctx, precompute=True)
    coeffs = C.random_fr(11, n * width).reshape(n, width, 4)
    _, prep = srs.prepare_columns(torch.from_numpy(coeffs.view(np.int64)).to("cuda:0"), want_commitments=False)
    points = [C.random_fr(12, 1)[0], C.random_fr(13, 1)[0]]
    alone = prep.msm(srs.opening_bases_many(n, points))
    coll = TorchCollective(rank, world, group, 0)
    ctx.check(ctx.lib.eon_ctx_set_collective(ctx.handle, ctypes.byref(coll.c)))
    try:
        shared = prep.msm(srs.opening_bases_many(n, points))
    finally:
        ctx.check(ctx.lib.eon_ctx_set_collective(ctx.handle, None))
    if not np.array_equal(alone, shared):
        return f"rank {rank}: sharded opening bases give different witnesses"
    # spot-check one witness against the reference's route (quotient, then commit_column)
    if rank == 0:
        q, _ = C.quotient_and_eval(coeffs[:, 1], points[0])
        g = srs_powers(n - 1, 12345, ctx)
        if not np.array_equal(shared[0, 1], C.g1_msm(g, q)):
            return "witness != commit_column(quotient)"
    return None


def run_rcclagree(rank, world, group):
    """native.RcclCollective's collective agreement on a fake libeonprove (no GPU): EON_T_FAIL=id
    fails rank 0's eon_rccl_unique_id, init1 fails rank 1's eon_rccl_collective_init, none fails
    nothing.  Every rank must end the same way (all raise RcclInitError, or all succeed), and a
    rank whose own init succeeded must finalise it when another rank failed."""
    from plonky3_eon_amd import native

    fail = os.environ["EON_T_FAIL"]
    calls = []

    class FakeLib:
        def eon_rccl_unique_id(self, buf):
            calls.append("id")
            if fail == "id":
                return -3
            buf[0] = 42
            return 0

        def eon_rccl_collective_init(self, r, w, idbuf, out):
            calls.append("init")
            if idbuf[0] != 42:
                return -9  # the id did not arrive
            return -3 if (fail == "init1" and r == 1) else 0

        def eon_rccl_collective_finalize(self, c):
            calls.append("finalize")

    saved = native.load
    native.load = lambda: FakeLib()
    try:
        try:
            native.RcclCollective(rank, world, group)
            outcome = "ok"
        except native.RcclInitError:
            outcome = "raised"
    finally:
        native.load = saved
    want = "ok" if fail == "none" else "raised"
    if outcome != want:
        return f"rank {rank}: {outcome}, expected {want} ({calls})"
    if fail == "id" and "init" in calls:
        return f"rank {rank} initialised after a failed unique id ({calls})"
    if fail == "init1" and rank != 1 and "finalize" not in calls:
        return f"rank {rank} kept its communicator after rank 1 failed ({calls})"
    return None


def main():
    import torch.distributed as dist

    mode, out = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # EON_T_BACKEND=nccl: RCCL on device buffers (one rank per GPU, so a one-GPU box runs world 1
    # only) -- the backend bench.py uses at N > 1; gloo ranks may share one GPU
    if os.environ.get("EON_T_BACKEND", "gloo") == "nccl":
        import torch

        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn = {"cpu": run_cpu, "gpu": run_gpu, "a2a": run_a2a, "fourstep": run_fourstep,
              "msmshard": run_msmshard, "native": run_native, "openshard": run_openshard,
              "fourstep_full": run_fourstep_full, "msmshard_full": run_msmshard_full,
              "rcclagree": run_rcclagree}[mode]
        why = fn(rank, world, None)
    except Exception:
        why = traceback.format_exc()
    finally:
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()
    Path(out).write_text(json.dumps({"ok": why is None, "why": why}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
