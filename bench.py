#!/usr/bin/env python3
"""bench.py -- MI355X benchmark of the plonky3-eon BN254/KZG prover hot path.

Contract (see DESIGN.md "Measurement"): `python bench.py --gpus N --steps K --warmup W` runs W
untimed steps, then times exactly K steps bracketed by a barrier + device synchronize, takes the
max over ranks, and rank 0 prints ONE JSON line.  For N > 1 it is launched by
torch.distributed.run (one process per GPU, RCCL backend); the workload is column-sharded, so
each rank owns its own columns and there is no collective on the data path (weak scaling).

Workload (default, BASELINE.json configs[1]): Radix2DitParallel-semantics coset_lde_batch of a
2^20 x 64 BN254 Fr matrix, added_bits = 1, shift = GENERATOR = 5, natural output order -- the LDE
that KzgPcs::get_evaluations_on_domain needs (kzg/src/pcs.rs:267-287) and dft/benches/fft.rs
times.  Inputs are synthetic uniform Fr, resident in HBM before the timed region.

Also reported:
  roofline     -- for the dominant kernel: algorithmic bytes per launch / average launch
                  duration (HIP events on the launch stream, eon_ctx_profile) vs 8 TB/s HBM;
                  `valu` adds the integer roofline (algorithmic mulmods / measured peak).
  cpu_baseline -- the C restatement of Radix2DitParallel::coset_lde_batch (oracle/eon_oracle.c,
                  OpenMP) timed on this host on a bounded column sample, rank 0 at N = 1 only.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "eon-uni-stark prove ms, Poseidon2-AIR 2^20 rows KZG/BN254, at 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# measured 256-bit Montgomery multiply peak (tools/ubench_mulmod.hip, MI355X, FIPS variant)
MULMOD_PEAK_PER_S = 1.27e11
FR_P = [0x43E1F593F0000001, 0x2833E84879B97091, 0xB85045B68181585D, 0x30644E72E131A029]


def synthetic_fr(rows: int, cols: int, seed: int) -> np.ndarray:
    """Uniform-ish canonical Fr Montgomery limbs: the top limb is drawn below P's top limb, so
    every value is < P (synthetic data; the distribution is irrelevant to the kernels' cost)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.integers(0, 2**64, size=(rows, cols, 4), dtype=np.uint64)
    x[..., 3] %= np.uint64(FR_P[3])
    return x


def lde_mulmods(log_n: int, width: int, b: int) -> float:
    """Algorithmic mulmods of one coset LDE: W*((1+2^b)*(N/2)*log2 N + N)."""
    n = 1 << log_n
    return width * ((1 + (1 << b)) * (n / 2) * log_n + n)


def cpu_baseline_lde(log_n: int, width: int, b: int, sample_cols: int) -> dict:
    from oracle import coracle

    coracle.build()
    x = synthetic_fr(1 << log_n, sample_cols, 7)
    shift = coracle.fr_from_u64(5)
    coracle.r2dp_coset_lde_batch(x[:1024], b, shift)  # warm-up (page in, thread pool)
    t0 = time.perf_counter()
    coracle.r2dp_coset_lde_batch(x, b, shift)
    dt = time.perf_counter() - t0
    scale = width / sample_cols
    return {
        "value": round(dt * scale * 1e3, 1),
        "unit": "ms",
        "cores": coracle.num_threads(),
        "kind": "port",
        "sample": f"2^{log_n} rows x {sample_cols} of {width} columns (C restatement of "
        f"Radix2DitParallel::coset_lde_batch, OpenMP), {dt:.2f} s measured, x{scale:g} "
        f"extrapolated linearly in columns",
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--added-bits", type=int, default=1)
    ap.add_argument("--order", choices=["natural", "bitrev"], default="natural")
    ap.add_argument("--cpu-sample-cols", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from plonky3_eon_amd import Context
    from plonky3_eon_amd import _lib as L
    from plonky3_eon_amd.field import fr_to_abi
    import ctypes

    ctx = Context(local_rank)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)

    n, w, b = 1 << args.log_n, args.width, args.added_bits
    order = L.EON_ORDER_NATURAL if args.order == "natural" else L.EON_ORDER_BITREV
    x_host = synthetic_fr(n, w, 1234 + rank)
    x = torch.from_numpy(x_host.view(np.int64)).to(dev)
    out = torch.empty((n << b, w, 4), dtype=torch.int64, device=dev)
    shift = fr_to_abi(5)

    def step():
        ctx.check(ctx.lib.eon_coset_lde_batch_dev(ctx.handle, ctypes.c_void_p(x.data_ptr()),
                                                  ctypes.c_void_p(out.data_ptr()), n, w, b,
                                                  ctypes.byref(shift), order))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    prof = ctx.profile_report()
    ctx.profile(False)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = elapsed * 1e3 / args.steps
    # dominant kernel: largest total time
    kname, kst = max(prof.items(), key=lambda kv: kv[1]["total_ms"])
    avg_ms = kst["total_ms"] / kst["launches"]
    bytes_per_launch = kst["alg_bytes"] / kst["launches"]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    lde_bytes = n * w * 32 + (n << b) * w * 32
    mulmods = lde_mulmods(args.log_n, w, b)
    gpu_total_ms = sum(v["total_ms"] for v in prof.values()) / args.steps

    result = {
        "metric": METRIC,
        "value": round(ms_per_step, 3),
        "unit": "ms",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bn254-fr (u32x8 Montgomery)",
        "data": "synthetic uniform Fr, resident in HBM",
        "config": {
            "workload": f"configs[1]: batched LDE NTT, coset_lde_batch 2^{args.log_n} rows x {w} cols over "
            f"BN254 Fr, added_bits={b}, shift=5, {args.order} output (per GPU; column-sharded)",
            "global_batch": w * world,
            "seq_len": n,
            "parallelism": f"column-shard x{world}",
        },
        "throughput": {
            "lde_elements_per_s": round(world * n * w / (ms_per_step * 1e-3), 1),
            "alg_GBps_whole_lde": round(world * lde_bytes / (ms_per_step * 1e-3) / 1e9, 2),
            "mulmod_per_s": round(world * mulmods / (ms_per_step * 1e-3), 1),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": None,
            "avg_launch_ms": round(avg_ms, 4),
            "alg_bytes_per_launch": int(bytes_per_launch),
            "valu": {
                "binding": True,
                "achieved_mulmod_per_s": round(mulmods / (gpu_total_ms * 1e-3), 1),
                "peak_mulmod_per_s": MULMOD_PEAK_PER_S,
                "frac": round(mulmods / (gpu_total_ms * 1e-3) / MULMOD_PEAK_PER_S, 4),
            },
            "kernels": prof,
        },
        "cpu_baseline": None,
    }
    traffic_file = ROOT / "profiles" / "traffic_lde.json"
    if traffic_file.exists():
        try:
            tf = json.loads(traffic_file.read_text())
            if tf.get("kernel") == kname and tf.get("workload") == result["config"]["workload"]:
                result["roofline"]["traffic"] = tf.get("bytes_per_launch")
        except Exception:
            pass

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_lde(args.log_n, w, b, min(args.cpu_sample_cols, w))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result))
    return 0


if __name__ == "__main__":
    sys.exit(main())
