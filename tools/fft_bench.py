#!/usr/bin/env python3
"""The reference's DFT benchmark matrix on one MI355X (dft/benches/fft.rs:11-27): 256 columns of
BN254 Fr at log sizes 14, 16, 18, 20, 22; dft_batch for Radix2Dit (natural) and Radix2DitParallel
(bit-reversed storage), idft_batch (Radix2Dit), coset_lde_batch(1, GENERATOR) for both.

Inputs are drawn on the device (canonical Fr limbs), outputs preallocated: each entry is the
median of --reps launches timed with HIP events on the launch stream, after one warm-up.  Also
printed per entry: algorithmic mulmods (W (N/2) log N per transform, as BASELINE.md section 3) over
the measured 1.80e11/s product peak, and HBM bytes (read N W 32 + write out) over 8 TB/s.
--cpu adds the C restatement (oracle/eon_oracle.c, OpenMP) at 2^14 x 256 for the same ops.

usage: python tools/fft_bench.py [--logs 14,16,18,20,22] [--reps 5] [--cpu] > fft_bench.json
"""

from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

MULMOD_PEAK = 1.80e11
HBM_PEAK = 8.0e12
COLS = 256


def dev_random_fr(n, w, seed):
    import torch

    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    x = torch.randint(-(2**63), 2**63 - 1, (n, w, 4), dtype=torch.int64, device="cuda:0", generator=g)
    x[..., 3] &= 0x2FFFFFFFFFFFFFFF
    return x


def mulmods(op, log_n, w):
    n = 1 << log_n
    if op == "coset_lde":  # idft + scaling, padded coset dft of 2N
        return w * ((n / 2) * log_n + n + n * (log_n + 1) + n)
    if op == "idft":
        return w * ((n / 2) * log_n + n)
    return w * (n / 2) * log_n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--logs", default="14,16,18,20,22")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args()
    import torch

    from plonky3_eon_amd import Context
    from plonky3_eon_amd import _lib as L
    from plonky3_eon_amd.field import fr_to_abi

    torch.cuda.set_device(0)
    ctx = Context(0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    gen = fr_to_abi(5)
    P = ctypes.c_void_p
    nat, rev = L.EON_ORDER_NATURAL, L.EON_ORDER_BITREV
    ops = [("dft", "Radix2Dit", nat), ("dft", "Radix2DitParallel", rev), ("idft", "Radix2Dit", nat),
           ("coset_lde", "Radix2Dit", nat), ("coset_lde", "Radix2DitParallel", rev)]
    rows = []
    for log_n in [int(v) for v in args.logs.split(",")]:
        n = 1 << log_n
        x = dev_random_fr(n, COLS, 1000 + log_n)
        out = torch.empty((2 * n, COLS, 4), dtype=torch.int64, device="cuda:0")
        for op, dft, order in ops:
            def launch():
                if op == "dft":
                    ctx.check(ctx.lib.eon_dft_batch_dev(ctx.handle, P(x.data_ptr()), P(out.data_ptr()), n, COLS, order))
                elif op == "idft":
                    ctx.check(ctx.lib.eon_idft_batch_dev(ctx.handle, P(x.data_ptr()), P(out.data_ptr()), n, COLS))
                else:
                    ctx.check(ctx.lib.eon_coset_lde_batch_dev(ctx.handle, P(x.data_ptr()), P(out.data_ptr()), n, COLS,
                                                              1, ctypes.byref(gen), order))

            launch()
            times = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                launch()
                b.record(stream)
                b.synchronize()
                times.append(a.elapsed_time(b))
            ms = sorted(times)[len(times) // 2]
            out_rows = 2 * n if op == "coset_lde" else n
            mm = mulmods(op, log_n, COLS)
            byts = (n + out_rows) * COLS * 32
            rows.append({"log_n": log_n, "op": op, "dft": dft, "ms": round(ms, 3),
                         "valu_frac": round(mm / (ms * 1e-3) / MULMOD_PEAK, 3),
                         "hbm_GBps": round(byts / (ms * 1e-3) / 1e9, 1),
                         "hbm_frac": round(byts / (ms * 1e-3) / HBM_PEAK, 4)})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
        del x, out
        torch.cuda.empty_cache()
    res = {"bench": "dft/benches/fft.rs shape: 256 columns, BN254 Fr, coset_lde(1, GENERATOR)",
           "device": torch.cuda.get_device_name(0), "reps": args.reps, "timing": "median HIP-event time per launch",
           "rows": rows}
    if args.cpu:
        import numpy as np

        from oracle import coracle as C

        C.build()
        x = C.random_fr(14, (1 << 14) * COLS).reshape(1 << 14, COLS, 4)
        g = C.fr_from_u64(5)
        cpu = {}
        for name, f in [("dft Radix2Dit", lambda: C.dft_batch(x)), ("dft Radix2DitParallel", lambda: C.r2dp_dft_batch(x)),
                        ("idft Radix2Dit", lambda: C.idft_batch(x)),
                        ("coset_lde Radix2Dit", lambda: C.coset_lde_batch(x, 1, g)),
                        ("coset_lde Radix2DitParallel", lambda: C.r2dp_coset_lde_batch(x, 1, g))]:
            t0 = time.perf_counter()
            f()
            cpu[name] = round((time.perf_counter() - t0) * 1e3, 1)
        res["cpu_baseline_2e14"] = {"ms": cpu, "cores": C.num_threads(), "kind": "port",
                                    "sample": "2^14 x 256, C restatement (OpenMP over columns)"}
        del np
    print(json.dumps(res))


if __name__ == "__main__":
    main()
