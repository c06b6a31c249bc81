#!/usr/bin/env python3
"""bench.py -- MI355X benchmark of the plonky3-eon BN254/KZG prover hot path.

Contract (see DESIGN.md "Measurement"): `python bench.py --gpus N --steps K --warmup W` runs W
untimed steps, then times exactly K steps bracketed by a barrier + device synchronize, takes the
max over ranks, and rank 0 prints ONE JSON line.  For N > 1 it runs one process per GPU (RCCL
backend): under torch.distributed.run as launched by the driver, or, started without a launcher
(no WORLD_SIZE), it starts torch.distributed.run itself as a child process before touching the
GPU and relays rank 0's line.  WORLD_SIZE != --gpus is an error.

Workloads (--workload):
  prove (default)  BASELINE.json configs[3] and the headline metric: eon-uni-stark prove of the
                   vectorized Poseidon2-AIR (VECTOR_LEN 8, log-trace-length 17 = 2^20
                   permutations) with KzgPcs over BN254.  At N > 1 the ONE proof is split by vector
                   lane (plonky3_eon_amd/distributed.py): strong scaling.
  lde              configs[1]: coset_lde_batch 2^20 x 64, added_bits 1, shift 5 (column-sharded,
                   weak scaling).
  msm              configs[2]: 2^20-point MSM over the alpha = 12345 SRS (weak scaling).
  ntt4, msm-shard  configs[4]: 2^26 four-step DFT (one all_to_all) and 2^24-point MSM split by
                   point range (strong scaling).
Inputs are synthetic, resident in HBM before the timed region.

Also reported:
  roofline     -- for the dominant kernel (largest total time): algorithmic bytes per launch
                   / average launch duration (HIP events on the launch
                  stream, eon_ctx_profile, over serialized profiled steps after the timed region)
                  vs 8 TB/s HBM, `traffic` from this round's committed PMC pass
                  (profiles/<round>/traffic_*.json, raw FETCH + WRITE, stamped with the commit it measured);
                  `valu` is the binding integer roofline of the same kernel: its algorithmic
                  256-bit Montgomery products per launch / launch duration vs the measured
                  mulmod peak (tools/ubench_r29.hip), and vs the product rate measured live on
                  this box by the clock probe (`frac_live`).
  gpu_clock_inkernel_mhz -- the shader clock held under a product chain right after the timed
                  region (eon_diag_clock_probe: s_memtime / s_memrealtime), beside `gpu_sclk`
                  (sysfs, which is not the in-kernel clock).
  cpu_baseline -- the C restatement (oracle/eon_oracle.c, OpenMP) of the same work timed on this
                  host on a bounded sample, rank 0 at N = 1 only.
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
# measured 256-bit Montgomery multiply peak on MI355X: the radix-2^29 carry-free product with its
# columns chained through one accumulator (tools/ubench_r29.hip, profiles/r01_ubench_r29.txt:
# 1.80e11/s; the radix-2^32 FIPS product of the quotient kernel peaks at 1.29e11/s,
# tools/ubench_mulmod.hip)
MULMOD_PEAK_PER_S = 1.80e11
# k_piece_sum29's instruction-issue cost per wave-addition: its gfx950 ISA (the addition block, the
# per-pair loads / unpack / key logic, the flush and run-start paths weighted by how often a wave
# takes them) priced with the measured SIMD cycles per wave-instruction at 4 waves per SIMD
SIMDS = 1024  # 256 CUs x 4 SIMDs
PIECE_ISSUE_CYCLES = 9550
PIECE_ISSUE_SOURCE = ("tools/isa_count.py --costs profiles/r06/s4/ubench_isa2.txt over the round-6 build: "
                      "addition block 9067 + per pair ~250 + (flush ~206 + run start ~93) x 0.77 (profiles/r06/s5/INDEX.md)")
# PMC traffic files are read from this round's profile directory only (see main())
TRAFFIC_ROUND = "r06"
FR_P = [0x43E1F593F0000001, 0x2833E84879B97091, 0xB85045B68181585D, 0x30644E72E131A029]


def _sig(x: float, n: int = 4) -> float:
    """x to n significant figures (a latency-bound workload's GB/s is far below 0.01)."""
    return float(f"{x:.{n}g}")


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


class SclkSampler:
    """The GPU's current shader clock (sysfs pp_dpm_sclk, the '*' level) sampled every 0.2 s in a
    background thread while the timed steps run, so box-to-box clock differences under this VALU
    load show in the bench line.  Only the card whose PCI address matches the device is read
    when torch reports it; readings that are unavailable (no sysfs access) leave the field null."""

    def __init__(self, dev):
        import glob
        import threading

        self.samples = []
        self.paths = sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk"))
        try:
            import torch

            pr = torch.cuda.get_device_properties(dev)
            bus = getattr(pr, "pci_bus_id", None)
            dom = getattr(pr, "pci_domain_id", 0) or 0
            pdev = getattr(pr, "pci_device_id", 0) or 0
            if bus is not None:
                tag = f"{dom:04x}:{bus:02x}:{pdev:02x}."
                mine = [q for q in self.paths if tag in os.path.realpath(os.path.dirname(q))]
                if mine:
                    self.paths = mine
        except Exception:
            pass
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _read(self):
        out = []
        for q in self.paths:
            try:
                for line in open(q):
                    if line.rstrip().endswith("*"):
                        out.append(int(line.split(":")[1].strip().split("Mhz")[0].split("MHz")[0]))
            except (OSError, ValueError, IndexError):
                pass
        return out

    def _run(self):
        while not self._stop.wait(0.2):
            v = self._read()
            if v:
                self.samples.append(max(v) if len(v) > 1 and len(self.paths) > 1 else v[0])

    def start(self):
        if self.paths:
            self._t.start()
        return self

    def stop(self):
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=1)
        if not self.samples:
            return None
        xs = sorted(self.samples)
        return {"median_mhz": xs[len(xs) // 2], "min_mhz": xs[0], "max_mhz": xs[-1], "samples": len(xs),
                "source": "sysfs pp_dpm_sclk" + (" (%d cards, max)" % len(self.paths) if len(self.paths) > 1 else "")}


def host_cpu() -> str:
    """The host CPU model (/proc/cpuinfo), recorded beside every CPU baseline."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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
    # T = 1 beside T = nproc: one thread on 2 sample columns
    with coracle.threads(1):
        t0 = time.perf_counter()
        coracle.r2dp_coset_lde_batch(x[:, :2].copy(), b, shift)
        dt1 = time.perf_counter() - t0
    return {
        "value": round(dt * scale * 1e3, 1),
        "unit": "ms",
        "cores": coracle.num_threads(),
        "kind": "port",
        "host_cpu": host_cpu(),
        "sample": f"2^{log_n} rows x {sample_cols} of {width} columns (C restatement of "
        f"Radix2DitParallel::coset_lde_batch, OpenMP), {dt:.2f} s measured, x{scale:g} "
        f"extrapolated linearly in columns",
        "t1": {"value": round(dt1 * width / 2 * 1e3, 1), "unit": "ms", "cores": 1,
               "sample": f"2^{log_n} rows x 2 columns on one thread, {dt1:.2f} s measured, x{width / 2:g} "
                         f"extrapolated linearly in columns"},
    }


def cpu_baseline_msm(bases_host: np.ndarray, scalars_host: np.ndarray) -> dict:
    from oracle import coracle

    coracle.build()
    n = bases_host.shape[0]
    t0 = time.perf_counter()
    coracle.g1_msm(bases_host, scalars_host)
    dt = time.perf_counter() - t0
    # T = 1 beside T = nproc: one thread on the first n / 4 points
    m = max(n // 4, 1)
    with coracle.threads(1):
        t0 = time.perf_counter()
        coracle.g1_msm(bases_host[:m], scalars_host[:m])
        dt1 = time.perf_counter() - t0
    return {
        "value": round(dt * 1e3, 1),
        "unit": "ms",
        "cores": coracle.num_threads(),
        "kind": "port",
        "host_cpu": host_cpu(),
        "sample": f"full input: {n} points (C Pippenger restatement: signed windows, XYZZ mixed additions, OpenMP over "
        f"window x point-chunk tasks; halo2curves msm_best is not in the reference tree)",
        "t1": {"value": round(dt1 * n / m * 1e3, 1), "unit": "ms", "cores": 1,
               "sample": f"{m} of {n} points on one thread, {dt1:.2f} s measured, x{n / m:g} extrapolated "
                         f"linearly (Pippenger's cost per point falls slowly with n: an upper bound)"},
    }


class LdeWorkload:
    """configs[1]: coset_lde_batch 2^log_n x width, added_bits, shift 5."""

    def __init__(self, args, ctx, dev, rank):
        import torch

        from plonky3_eon_amd import _lib as L
        from plonky3_eon_amd.field import fr_to_abi

        self.args, self.ctx = args, ctx
        self.n, self.w, self.b = 1 << args.log_n, args.width, args.added_bits
        self.order = L.EON_ORDER_NATURAL if args.order == "natural" else L.EON_ORDER_BITREV
        self.x = torch.from_numpy(synthetic_fr(self.n, self.w, 1234 + rank).view(np.int64)).to(dev)
        self.out = torch.empty((self.n << self.b, self.w, 4), dtype=torch.int64, device=dev)
        self.shift = fr_to_abi(5)
        # read N W 32 B + write 2^b N W 32 B
        self.alg_bytes_per_step = self.n * self.w * 32 + (self.n << self.b) * self.w * 32

    def step(self):
        import ctypes

        c = self.ctx
        c.check(c.lib.eon_coset_lde_batch_dev(c.handle, ctypes.c_void_p(self.x.data_ptr()),
                                              ctypes.c_void_p(self.out.data_ptr()), self.n, self.w,
                                              self.b, ctypes.byref(self.shift), self.order))

    def describe(self, world):
        a = self.args
        return (f"configs[1]: batched LDE NTT, coset_lde_batch 2^{a.log_n} rows x {self.w} cols over "
                f"BN254 Fr, added_bits={self.b}, shift=5, {a.order} output (per GPU; column-sharded)",
                self.w * world, self.n, f"column-shard x{world}")

    def throughput(self, world, ms):
        n, w, b = self.n, self.w, self.b
        lde_bytes = n * w * 32 + (n << b) * w * 32
        mulmods = lde_mulmods(self.args.log_n, w, b)
        return {
            "lde_elements_per_s": round(world * n * w / (ms * 1e-3), 1),
            "alg_GBps_whole_lde": round(world * lde_bytes / (ms * 1e-3) / 1e9, 2),
            "mulmod_per_s": round(world * mulmods / (ms * 1e-3), 1),
        }, mulmods

    def cpu_baseline(self):
        a = self.args
        return cpu_baseline_lde(a.log_n, self.w, self.b, min(a.cpu_sample_cols, self.w))


class MsmWorkload:
    """configs[2]: KZG commit MSM, 2^log_msm SRS points (alpha = 12345) x uniform Fr scalars."""

    def __init__(self, args, ctx, dev, rank):
        import ctypes

        import torch

        from plonky3_eon_amd import _lib as L
        from plonky3_eon_amd.field import fr_to_abi

        self.args, self.ctx = args, ctx
        self.n = 1 << args.log_msm
        self.bases_dev = torch.empty((self.n, 8), dtype=torch.int64, device=dev)
        alpha = fr_to_abi(12345)
        ctx.check(ctx.lib.eon_g1_srs_powers_dev(ctx.handle, ctypes.byref(alpha), self.n,
                                                ctypes.c_void_p(self.bases_dev.data_ptr())))
        h = ctypes.c_void_p()
        ctx.check(ctx.lib.eon_msm_bases_create_dev(ctx.handle, ctypes.c_void_p(self.bases_dev.data_ptr()),
                                                   self.n, L.EON_MSM_PRECOMPUTE, ctypes.byref(h)))
        self.bases = h
        if args.msm_scalars == "small":
            # all scalars < 2^64, as kzg/benches/kzg_benches.rs:16-22
            from plonky3_eon_amd.field import ints_to_limbs

            # the full u64 range, as Fr::new(rng.random::<u64>()) (kzg_benches.rs:19)
            vals = np.random.Generator(np.random.PCG64(3 + rank)).integers(0, 2**64, self.n, dtype=np.uint64)
            self.scalars_host = np.ascontiguousarray(ints_to_limbs([int(v) for v in vals]), dtype=np.uint64)
        else:
            self.scalars_host = synthetic_fr(self.n, 1, 3 + rank).reshape(self.n, 4)
        self.scalars = torch.from_numpy(self.scalars_host.view(np.int64)).to(dev)
        self.out = np.zeros(8, dtype=np.uint64)

    def step(self):
        import ctypes

        c = self.ctx
        c.check(c.lib.eon_msm_g1_dev(c.handle, self.bases, ctypes.c_void_p(self.scalars.data_ptr()),
                                     self.n, self.out.ctypes.data_as(ctypes.c_void_p)))

    def describe(self, world):
        return (f"configs[2]: KZG commit MSM, 2^{self.args.log_msm} BN254 G1 SRS points (alpha=12345, "
                f"fixed-base window table built untimed) x "
                f"{'scalars < 2^64 (kzg_benches)' if self.args.msm_scalars == 'small' else 'uniform Fr scalars'} (per GPU)",
                world, self.n, f"msm-shard x{world}")

    def throughput(self, world, ms):
        # Pippenger mixed additions: n * ceil(255 / c) nonzero-digit pairs (c chosen by the library)
        return {
            "points_per_s": round(world * self.n / (ms * 1e-3), 1),
            "alg_GBps": round(world * self.n * 96 / (ms * 1e-3) / 1e9, 3),
        }, None

    def cpu_baseline(self):
        return cpu_baseline_msm(self.bases_dev.cpu().numpy().view(np.uint64), self.scalars_host)


def p2_constants_limbs(seed: int, hf: int = 4, pr: int = 56):
    """Deterministic Poseidon2 round constants as Montgomery limbs (synthetic; the reference draws
    them from SmallRng, poseidon2-air/src/constants.rs:37-46)."""
    x = synthetic_fr(6 * hf + pr, 1, seed).reshape(-1, 4)
    return x[:3 * hf].reshape(hf, 3, 4), x[3 * hf:3 * hf + pr], x[3 * hf + pr:].reshape(hf, 3, 4)


def _cpu_prove_e2e(log_n: int, vl: int, consts, horner: bool) -> dict:
    """One end-to-end prove of the C restatement (oracle/prove_oracle.py: commit, LDE, quotient,
    quotient commit, open with the reference's per-column quotient_and_eval + commit_column) at
    log-trace log_n; horner=False substitutes the coset-DFT LDE for the reference's Horner
    get_evaluations_on_domain (kzg/src/pcs.rs:267-287)."""
    from oracle import coracle as C
    from oracle import prove_oracle

    n = 1 << log_n
    k = C.P2Constants(*consts)
    tr = C.p2_generate_trace(synthetic_fr(n * vl, 3, 5).reshape(-1, 3, 4), vl, k)
    srs = C.g1_srs(n + 1, C.fr_from_u64(12345))

    def lde_sub(coeffs, log_q, shift):
        pad = np.zeros(((1 << log_q) - coeffs.shape[0],) + coeffs.shape[1:], dtype=np.uint64)
        return C.coset_dft_batch(np.concatenate([coeffs, pad]), shift)

    st = {}
    t0 = time.perf_counter()
    prove_oracle.prove(tr, srs, k, vl, 7, 11, lde_fn=None if horner else lde_sub, timings=st)
    dt = time.perf_counter() - t0
    return {"log_trace": log_n, "lde": "horner (reference)" if horner else "coset DFT (substituted)",
            "ms": round(dt * 1e3, 1), "stage_ms": {a: round(b * 1e3, 1) for a, b in st.items()}}


def cpu_baseline_prove(log_n: int, vl: int, consts, full: bool = False) -> dict:
    """CPU restatement of the prove on this host: MEASURED end-to-end proves at small log-trace
    sizes, and the full-size figure PROJECTED from measured full-size
    components (C4 (ii); a full CPU run is infeasible: get_evaluations_on_domain's Horner is
    ~4.5e13 mulmods)."""
    from oracle import coracle as C

    C.build()
    # measured end-to-end proves at n = 8 (reference Horner LDE), 10 and 12
    # (coset-DFT LDE substituted: the Horner loop alone is quadratic)
    measured = [_cpu_prove_e2e(8, vl, consts, True), _cpu_prove_e2e(10, vl, consts, False),
                _cpu_prove_e2e(12, vl, consts, False)]
    if full:  # --cpu-full: 2^10 with the reference's Horner LDE as well (minutes)
        measured += [_cpu_prove_e2e(10, vl, consts, True)]
    n = 1 << log_n
    w = 164 * vl
    q = 2 * n
    alpha = C.fr_from_u64(12345)
    comp = {}
    # trace coset_idft (Radix2Dit in KzgPcs): 16 sample columns, linear in width
    x = synthetic_fr(n, 16, 11)
    t0 = time.perf_counter(); C.idft_batch(x); dt = time.perf_counter() - t0
    comp["trace idft"] = dt * w / 16
    # one full-size MSM of n points (signed-window Pippenger, OpenMP inside, as the reference runs
    # each commit_column); prove runs w (trace) + 2 (quotient) + 2w + 2 (open) of them
    pts = C.g1_srs(1 << 12, alpha)
    pts = np.concatenate([pts] * (n >> 12))
    s = synthetic_fr(n, 1, 12).reshape(n, 4)
    t0 = time.perf_counter(); C.g1_msm(pts, s); dt = time.perf_counter() - t0
    n_msm = 3 * w + 4
    comp["msm x%d" % n_msm] = dt * n_msm
    msm_ms = dt * 1e3  # noqa
    # get_evaluations_on_domain by Horner (kzg/src/pcs.rs:267-287): Q * w evaluations of degree n
    coeffs = synthetic_fr(n, 1, 13)
    t0 = time.perf_counter()
    for k in range(16):
        C.eval_poly_col(coeffs, 0, C.fr_from_u64(k + 7))
    dt = (time.perf_counter() - t0) / 16
    comp["lde horner (reference)"] = dt * q * w / C.num_threads()
    # the same values by coset LDE (C restatement), 16 sample columns
    t0 = time.perf_counter(); C.coset_lde_batch(x, 1, C.fr_from_u64(5)); dt = time.perf_counter() - t0
    lde_fft = dt * w / 16
    # quotient_values on 4096 sample rows
    k = C.P2Constants(*consts)
    lde_s = synthetic_fr(1 << 12, w, 14)
    t0 = time.perf_counter(); C.p2_quotient_values(lde_s, 11, 1, vl, k, alpha); dt = time.perf_counter() - t0
    comp["quotient_values"] = dt * q / 4096
    total = sum(comp.values())
    alt = total - comp["lde horner (reference)"] + lde_fft
    # T = 1 beside T = nproc: the same components on one thread, smaller samples
    comp1 = {}
    with C.threads(1):
        t0 = time.perf_counter(); C.idft_batch(x[:, :2].copy()); dt = time.perf_counter() - t0
        comp1["trace idft"] = dt * w / 2
        t0 = time.perf_counter(); C.g1_msm(pts, s); dt = time.perf_counter() - t0
        comp1["msm x%d" % n_msm] = dt * n_msm
        t0 = time.perf_counter(); C.eval_poly_col(coeffs, 0, C.fr_from_u64(7)); dt = time.perf_counter() - t0
        comp1["lde horner (reference)"] = dt * q * w
        t0 = time.perf_counter(); C.p2_quotient_values(lde_s[:512].copy(), 8, 1, vl, k, alpha); dt = time.perf_counter() - t0
        comp1["quotient_values"] = dt * q / 512
    total1 = sum(comp1.values())
    return {
        "value": round(total * 1e3, 1),
        "unit": "ms",
        "cores": C.num_threads(),
        "kind": "port",
        "host_cpu": host_cpu(),
        "projected": True,
        "t1": {"value": round(total1 * 1e3, 1), "unit": "ms", "cores": 1, "projected": True,
               "components_ms": {k2: round(v * 1e3, 1) for k2, v in comp1.items()},
               "sample": "the same full-size components on one thread (trace idft 2 columns, one 2^%d MSM, "
                         "one Horner point, quotient 512 rows), scaled as the T = nproc leg" % log_n},
        "sample": "value = full-size prove PROJECTED as the sum of full-size component samples of the C "
                  "restatement (trace idft 16/%d cols, one measured 2^%d MSM x %d, Horner LDE 16 points, "
                  "quotient 4096 rows), reference algorithms incl. the Horner get_evaluations_on_domain; "
                  "`measured` holds end-to-end proves of the same AIR run here" % (w, log_n, n_msm),
        "components_ms": {k2: round(v * 1e3, 1) for k2, v in comp.items()},
        "msm_2_%d_measured_ms" % log_n: round(msm_ms, 1),
        "with_coset_lde_ms": round(alt * 1e3, 1),
        "measured": measured,
    }


class ProveWorkload:
    """configs[3]: eon-uni-stark prove of the vectorized Poseidon2-AIR (VECTOR_LEN 8, 2^(log_n+3)
    permutations, log-trace-length log_n) with KzgPcs over BN254 (SRS max_degree 2^log_n,
    alpha 12345); alpha / zeta sampled from the Fiat-Shamir transcript (DuplexChallenger over
    Poseidon2Bn254<3>, 8 full + 56 partial rounds, synthetic constants; --transcript fixed keeps
    them constant).  At N > 1 the ONE proof is split
    by vector lane over the ranks (plonky3_eon_amd/distributed.py): strong scaling.

    The prove runs in the C++ driver (libeonprove.so, include/eon_prove.h; at N > 1 its
    all-gathers go through its own RCCL communicator, or torch.distributed's process group when the
    ranks share a GPU / with --collective torch)."""

    scaling = "strong"

    def __init__(self, args, ctx, dev, rank):
        import torch

        from plonky3_eon_amd.air import Poseidon2Air
        from plonky3_eon_amd.distributed import Shard

        self.args, self.ctx = args, ctx
        self.log_n, self.vl = args.log_trace, args.vector_len
        n = 1 << self.log_n
        world = int(os.environ.get("WORLD_SIZE", "1"))
        self.emulate = args.emulate_world
        if self.emulate > 1 and world > 1:
            raise SystemExit("--emulate-world is a one-process proxy (run it without --gpus)")
        if self.emulate > 1:
            # rank 0 of an `emulate`-rank lane-sharded prove on this one GPU: its lanes, its
            # commit / LDE / quotient / open work, the replicated transcript over all
            # 164 * VECTOR_LEN commitments, and device copies standing in for the exchanges
            self.shard = Shard(0, self.emulate, self.vl)
        else:
            self.shard = Shard(rank, world, self.vl) if world > 1 else None
        l0, l1 = self.shard.lanes if self.shard else (0, self.vl)
        self.consts = p2_constants_limbs(99)
        self.air = Poseidon2Air(*self.consts, l1 - l0, ctx)
        self.p2air = self.air  # trace generation always runs the Poseidon2 tracegen kernel
        if args.air == "generic":
            # the same AIR through the generic quotient path: its symbolic constraints compiled by
            # eon_air_program_create and run by k_air_quotient (prover.rs:539-709 for any EonAir)
            if world > 1:
                raise SystemExit("--air generic is single-GPU (the lane-sharded prove uses the fused AIR)")
            from plonky3_eon_amd.air import AirProgram

            self.air = AirProgram(self.p2air, ctx)
        from plonky3_eon_amd.native import (EmulatedCollective, NativeKzgPcs, RcclCollective, RcclInitError,
                                            TorchCollective)

        self.pcs = NativeKzgPcs(n, 12345, ctx)
        self.coll = None
        if self.emulate > 1:
            self.coll = EmulatedCollective(0, self.emulate)
        elif world > 1:
            # the driver's own RCCL communicator (ncclAllGather on the eon stream, called from the
            # C++ driver thread: no Python on the exchange path) when every rank has its own GPU;
            # torch.distributed's process group (a ctypes callback into Python per exchange) when
            # the ranks share a device (EON_BENCH_ONE_DEVICE rehearsals: RCCL refuses two ranks on
            # one GPU) or with --collective torch
            kind = choose_collective(args.collective, os.environ)
            self.collective_kind = kind
            self.coll = None
            if kind == "rccl":
                try:
                    self.coll = RcclCollective(rank, world)
                except RcclInitError as e:
                    # raised on every rank alike (the ranks agree on the outcome inside
                    # RcclCollective), so all of them fall back together; anything else fails fast
                    print(f"bench.py: RCCL communicator failed ({e}); using torch.distributed", file=sys.stderr)
                    self.collective_kind = "torch (rccl init failed)"
            if self.coll is None:
                self.coll = TorchCollective(rank, world, None, device=dev.index)
        # the same 2^(log_n) x VECTOR_LEN permutation inputs on every rank; rank g takes its lanes
        # (permutation j sits at row j / VECTOR_LEN, lane j % VECTOR_LEN)
        inputs = synthetic_fr(n * self.vl, 3, 5).reshape(n, self.vl, 3, 4)[:, l0:l1]
        inputs = torch.from_numpy(np.ascontiguousarray(inputs).reshape(-1, 3, 4).view(np.int64)).to(dev)
        self.trace = self.p2air.generate_trace(inputs)
        del inputs
        self.alpha, self.zeta = 0x1234567890ABCDEF1234567, 0xFEDCBA09876543210FEDCBA
        self.fs = args.transcript == "fs"
        self.ch_consts = p2_constants_limbs(77)  # the challenger's own permutation
        self.timings = []

    def step(self):
        from plonky3_eon_amd.native import Challenger, Poseidon2Constants, prove_native

        # config.initialise_challenger() per proof (prover.rs:164)
        ch = Challenger(Poseidon2Constants(*self.ch_consts)) if self.fs else None
        p = prove_native(self.air, self.pcs, self.trace, self.alpha, self.zeta, collective=self.coll,
                         challenger=ch)
        self.timings.append(p.timings_ms)

    def describe(self, world):
        w = 164 * self.vl
        par = f"lane-shard x{world} ({getattr(self, 'collective_kind', 'torch')} collective)" if world > 1 else "single"
        if self.emulate > 1:
            par = (f"EMULATED rank 0 of lane-shard x{self.emulate} on one GPU (its lanes and the full "
                   f"transcript; exchanges replaced by local device copies; not a valid proof)")
        return (f"configs[3]: eon-uni-stark prove, Poseidon2-AIR (VECTOR_LEN {self.vl}, width {w}) "
                f"log-trace-length {self.log_n} (2^{self.log_n + (self.vl.bit_length() - 1)} permutations), "
                f"KzgPcs over BN254" + (", Fiat-Shamir transcript" if self.fs else ", fixed alpha/zeta")
                + (", generic AIR program quotient (k_air_quotient)" if self.args.air == "generic" else ""),
                world, 1 << self.log_n, par)

    def throughput(self, world, ms):
        n = 1 << self.log_n
        st = {}
        for k in self.timings[self.args.warmup:self.args.warmup + self.args.steps]:  # the timed steps
            for a, b in k.items():
                st[a] = st.get(a, 0.0) + b / self.args.steps
        return {
            "permutations_per_s": round(n * self.vl / (ms * 1e-3), 1),
            "stage_ms": {a: round(b, 2) for a, b in st.items()},
        }, None

    def cpu_baseline(self):
        return cpu_baseline_prove(self.log_n, self.vl, self.consts, full=self.args.cpu_full)



class QuotientWorkload:
    """quotient_values alone at the headline size (configs[3]'s quotient stage): the Poseidon2-AIR
    (VECTOR_LEN 8, 1280 constraints) over a 2^(log_trace+1) x 1312 LDE, through the fused kernel
    (--air fused, k_p2_quotient) or the generic compiled program (--air generic, k_air_quotient;
    prover.rs:539-709 for any EonAir).  Synthetic canonical LDE values resident in HBM."""

    def __init__(self, args, ctx, dev, rank):
        import torch

        from plonky3_eon_amd.air import AirProgram, Poseidon2Air

        self.args, self.ctx = args, ctx
        self.log_n, self.vl, self.log_qd = args.log_trace, args.vector_len, 1
        p2 = Poseidon2Air(*p2_constants_limbs(99), self.vl, ctx)
        self.air = AirProgram(p2, ctx) if args.air == "generic" else p2
        self.p2 = p2
        q = 1 << (self.log_n + self.log_qd)
        g = torch.Generator(device=dev)
        g.manual_seed(5 + rank)
        self.lde = torch.randint(-(1 << 63), (1 << 63) - 1, (q, p2.width, 4), generator=g, device=dev,
                                 dtype=torch.int64)
        self.lde[..., 3] &= (1 << 60) - 1  # canonical (< p)
        self.alpha = 0x1234567890ABCDEF1234567
        self.alg_bytes_per_step = q * p2.width * 32 + q * 32

    def step(self):
        self.out = self.air.quotient_values(self.lde, self.log_n, self.log_qd, self.alpha)

    def describe(self, world):
        kind = "generic AIR program (k_air_quotient)" if self.args.air == "generic" else "fused kernel (k_p2_quotient)"
        prog = ""
        if self.args.air == "generic":
            st = self.air.stats
            prog = f", {st['num_instructions']} instructions, {st['num_registers']} registers"
        return (f"configs[3] quotient stage: quotient_values of the Poseidon2-AIR (VECTOR_LEN {self.vl}, "
                f"{160 * self.vl} constraints) over 2^{self.log_n + self.log_qd} x {self.p2.width} LDE rows, {kind}{prog}",
                world, 1 << (self.log_n + self.log_qd), "single")

    def throughput(self, world, ms):
        return {"rows_per_s": round(world * (1 << (self.log_n + self.log_qd)) / (ms * 1e-3), 1)}, None

    def cpu_baseline(self):
        from oracle import coracle as C

        C.build()
        k = C.P2Constants(*p2_constants_limbs(99))
        rows = 4096
        lde_s = synthetic_fr(rows, 164 * self.vl, 14)
        t0 = time.perf_counter()
        C.p2_quotient_values(lde_s, 11, 1, self.vl, k, C.fr_from_u64(12345))
        dt = time.perf_counter() - t0
        q = 1 << (self.log_n + self.log_qd)
        return {"value": round(dt * q / rows * 1e3, 1), "unit": "ms", "cores": C.num_threads(), "kind": "port",
                "sample": f"C restatement of quotient_values on {rows} of {q} rows ({dt:.2f} s), scaled linearly"}


class VerifyWorkload:
    """KzgPcs::verify's verify_batch (kzg/src/util.rs:245-292) of every opening
    of the configs[3] proof -- 1312 trace columns at zeta and zeta h plus the quotient chunks at
    zeta, 2626 (commitment, witness, value, point) quadruples -- on the GPU
    (eon_kzg_verify_batch: the product of the 2 x 2626 pairings, merged per opening point by
    bilinearity into 3 pairs, Miller loops and one final exponentiation).  The proof is made once
    by the configs[3] prove (untimed); the openings are host arrays, as a verifier receives them."""

    latency_bound = True

    def __init__(self, args, ctx, dev, rank):
        from oracle import pyoracle as O
        from plonky3_eon_amd import verify as GV

        args.transcript = "fs"
        pw = ProveWorkload(args, ctx, dev, rank)
        from plonky3_eon_amd.native import Challenger, Poseidon2Constants, prove_native

        proof = prove_native(pw.air, pw.pcs, pw.trace, None, None,
                             challenger=Challenger(Poseidon2Constants(*pw.ch_consts)))
        self.GV, self.ctx = GV, ctx
        log_n = args.log_trace

        def fr_l(x):
            return np.array(O.int_to_limbs(O.to_mont(x % O.P)), dtype=np.uint64)

        tc = np.asarray(proof.trace_commit[0]).reshape(-1, 8)
        tr, qo = proof.opened
        zn = proof.zeta * O.two_adic_generator(log_n) % O.P
        com, wit, val, pts = [], [], [], []
        for p, z in enumerate((proof.zeta, zn)):
            com.append(tc)
            wit.append(np.asarray(tr.witnesses[0][p]).reshape(-1, 8))
            val.append(np.asarray(tr.values[0][p]).reshape(-1, 4))
            pts.append(np.tile(fr_l(z), (tc.shape[0], 1)))
        for c, qc in enumerate(proof.quotient_commit):
            com.append(np.asarray(qc).reshape(1, 8))
            wit.append(np.asarray(qo.witnesses[c][0]).reshape(1, 8))
            val.append(np.asarray(qo.values[c][0]).reshape(1, 4))
            pts.append(fr_l(proof.zeta)[None])
        self.com, self.wit, self.val, self.pts = (np.ascontiguousarray(np.concatenate(a), dtype=np.uint64)
                                                  for a in (com, wit, val, pts))
        self.n = self.com.shape[0]
        self.g2a = GV.g2_mul(12345, ctx=ctx)
        self.alg_bytes_per_step = self.n * (64 + 64 + 32 + 32)
        del pw

    def step(self):
        if self.GV.verify_batch(self.com, self.wit, self.val, self.pts, self.g2a, ctx=self.ctx) is not True:
            raise SystemExit("verify_batch rejected the configs[3] proof")

    def describe(self, world):
        return (f"N4: KzgPcs::verify_batch of the configs[3] proof's {self.n} openings (1312 trace columns at "
                f"zeta and zeta h, quotient chunks at zeta) on the GPU: pairings merged per opening point",
                world, self.n, "single")

    def throughput(self, world, ms):
        return {"openings_per_s": round(self.n / (ms * 1e-3), 1)}, None

    def cpu_baseline(self):
        # the restated verify_batch (oracle/pairing.py: 2 Miller loops per opening, one final
        # exponentiation, pure Python) on 2 and 4 openings, extended linearly to all of them
        from oracle import pairing as E
        from oracle import pyoracle as O
        from oracle import verify_oracle as V

        def pt(row):
            return O.g1_from_bytes(np.ascontiguousarray(row, dtype=np.uint64).reshape(8).tobytes())

        ops = [(pt(self.com[i]), pt(self.wit[i]), V.fr_int(self.val[i]), V.fr_int(self.pts[i])) for i in range(4)]
        g2a = E.g2_alpha(12345)
        ts = {}
        for k in (2, 4):
            t0 = time.perf_counter()
            assert E.verify_batch(ops[:k], g2a)
            ts[k] = time.perf_counter() - t0
        per = (ts[4] - ts[2]) / 2
        fixed = max(ts[2] - 2 * per, 0.0)
        return {"value": round((fixed + per * self.n) * 1e3, 1), "unit": "ms", "cores": 1, "kind": "port",
                "sample": f"oracle/pairing.py verify_batch on 2 and 4 openings ({ts[2]:.2f} / {ts[4]:.2f} s), "
                          f"linear in the openings to {self.n}"}


class FourStepWorkload:
    """configs[4] (i): one forward DFT of 2^log_n Fr (natural in / natural out semantics) as a
    four-step N1 x N2 transform split over the ranks, one RCCL all_to_all for the transpose
    (plonky3_eon_amd.distributed.fourstep_dft).  Total size fixed: strong scaling."""

    scaling = "strong"

    def __init__(self, args, ctx, dev, rank):
        import torch

        from plonky3_eon_amd import distributed as D

        self.args, self.ctx, self.dev, self.rank = args, ctx, dev, rank
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.log_n = args.log_ntt
        log_n1, log_n2 = D.fourstep_split(self.log_n)
        cols = (1 << log_n2) // self.world
        self.local = torch.from_numpy(synthetic_fr(1 << log_n1, cols, 4321 + rank).view(np.int64)).to(dev)
        # 2 N 32 B (read + write once), this rank's 1/world share
        self.alg_bytes_per_step = 2 * (1 << self.log_n) * 32 // self.world

    def step(self):
        from plonky3_eon_amd import distributed as D

        self.out = D.fourstep_dft(self.ctx, self.local, self.log_n, self.rank, self.world)

    def describe(self, world):
        return (f"configs[4] (i): forward DFT 2^{self.log_n} over BN254 Fr, four-step "
                f"2^{(self.log_n + 1) // 2} x 2^{self.log_n // 2}, all_to_all transpose over {world} GPU(s)",
                1, 1 << self.log_n, f"fourstep x{world}")

    def throughput(self, world, ms):
        n = 1 << self.log_n
        return {"elements_per_s": round(n / (ms * 1e-3), 1)}, (n / 2) * self.log_n / world + n / world

    def cpu_baseline(self):
        from oracle import coracle

        coracle.build()
        log_s = 22
        x = synthetic_fr(1 << log_s, 1, 99)
        coracle.dft_batch(x[:1024])
        t0 = time.perf_counter()
        coracle.dft_batch(x)
        dt = time.perf_counter() - t0
        scale = ((1 << self.log_n) * self.log_n) / ((1 << log_s) * log_s)
        return {
            "value": round(dt * scale * 1e3, 1),
            "unit": "ms",
            "cores": coracle.num_threads(),
            "kind": "port",
            "sample": f"C restatement of Radix2Dit::dft_batch on one 2^{log_s} column ({dt:.2f} s), "
                      f"scaled by N log N to 2^{self.log_n}",
        }


class MsmShardWorkload:
    """configs[4] (ii): one MSM of 2^log_msm points split by contiguous point range over the ranks
    (2^24 / G per GPU), per-rank Pippenger + all-gather of the partial points + their sum
    (plonky3_eon_amd.distributed.msm_sharded).  Total size fixed: strong scaling.  Bases are a
    synthetic SRS (alpha^i G1, per-rank alpha), fixed-base tables built untimed."""

    scaling = "strong"

    def __init__(self, args, ctx, dev, rank):
        from plonky3_eon_amd import distributed as D
        from plonky3_eon_amd.msm import MsmBases, srs_powers

        self.args, self.ctx, self.dev = args, ctx, dev
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        n = 1 << args.log_shard_msm
        lo, hi = D.shard_range(n, rank, self.world)
        self.n_total, self.n_local = n, hi - lo
        self.bases = MsmBases(srs_powers(self.n_local, 777 + rank, ctx), ctx, precompute=True)
        import torch

        self.scalars = torch.from_numpy(synthetic_fr(self.n_local, 1, 55 + rank).view(np.int64)).to(dev)
        self.group = None

    def step(self):
        from plonky3_eon_amd import distributed as D

        if self.world > 1:
            self.out = D.msm_sharded(self.bases, self.scalars.reshape(-1, 4), self.dev, self.group)
        else:
            self.out = self.bases.msm(self.scalars.reshape(-1, 4))

    def describe(self, world):
        return (f"configs[4] (ii): MSM 2^{self.args.log_shard_msm} BN254 G1 points split by point range over "
                f"{world} GPU(s) (2^{self.args.log_shard_msm} / {world} per GPU)", 1, self.n_total,
                f"msm-shard x{world}")

    def throughput(self, world, ms):
        return {"points_per_s": round(self.n_total / (ms * 1e-3), 1)}, None

    def cpu_baseline(self):
        from oracle import coracle

        coracle.build()
        n = 1 << 18
        pts = coracle.g1_srs(1 << 12, coracle.fr_from_u64(777))
        pts = np.concatenate([pts] * (n >> 12))
        s = synthetic_fr(n, 1, 12).reshape(n, 4)
        t0 = time.perf_counter()
        coracle.g1_msm(pts, s)
        dt = time.perf_counter() - t0
        scale = self.n_total / n
        return {
            "value": round(dt * scale * 1e3, 1),
            "unit": "ms",
            "cores": coracle.num_threads(),
            "kind": "port",
            "projected": True,
            "sample": f"C Pippenger restatement on 2^18 points ({dt:.2f} s), scaled linearly to "
                      f"2^{self.args.log_shard_msm}",
        }

def choose_collective(flag: str, env) -> str:
    """The N > 1 prove's exchange path: the driver's own RCCL communicator unless the ranks share
    one device (EON_BENCH_ONE_DEVICE=1: RCCL refuses two ranks on one GPU) or the process group is
    not nccl (EON_BENCH_BACKEND=gloo rehearsals), or as --collective says."""
    if flag != "auto":
        return flag
    shared = env.get("EON_BENCH_ONE_DEVICE") == "1"
    return "torch" if shared or env.get("EON_BENCH_BACKEND", "nccl") != "nccl" else "rccl"


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default: 3 (prove), 10 (lde, msm)")
    ap.add_argument("--warmup", type=int, default=None, help="default: 1 (prove), 3 (lde, msm)")
    ap.add_argument("--workload", choices=["prove", "lde", "msm", "ntt4", "msm-shard", "quotient", "verify"],
                    default="prove")
    ap.add_argument("--air", choices=["fused", "generic"], default="fused",
                    help="prove / quotient: the Poseidon2-AIR's quotient through the fused kernel or the "
                         "generic compiled constraint program")
    ap.add_argument("--log-ntt", type=int, default=26, help="ntt4: transform size (configs[4] (i))")
    ap.add_argument("--log-shard-msm", type=int, default=24, help="msm-shard: total points (configs[4] (ii))")
    ap.add_argument("--log-trace", type=int, default=17)
    ap.add_argument("--vector-len", type=int, default=8)
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--added-bits", type=int, default=1)
    ap.add_argument("--order", choices=["natural", "bitrev"], default="natural")
    ap.add_argument("--log-msm", type=int, default=20)
    ap.add_argument("--msm-scalars", choices=["uniform", "small"], default="uniform",
                    help="msm: uniform Fr scalars, or all < 2^64 (kzg/benches/kzg_benches.rs:16-22)")
    ap.add_argument("--cpu-sample-cols", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-clock-probe", action="store_true",
                    help="skip the in-kernel clock probe after the timed region (~2 s)")
    ap.add_argument("--cpu-full", action="store_true",
                    help="prove: also the larger end-to-end CPU restatement runs (2^10 Horner, 2^12; minutes)")
    ap.add_argument("--serial", action="store_true",
                    help="every step in serial mode (eon_ctx_set_serial): for rocprofv3 kernel traces "
                         "whose per-kernel durations are isolated")
    ap.add_argument("--transcript", choices=["fs", "fixed"], default="fs",
                    help="prove: alpha/zeta from the Fiat-Shamir transcript (default) or fixed")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="prove: time rank 0 of an N-rank lane-sharded prove on this one GPU (its lanes, "
                         "the full replicated transcript, local copies for the exchanges) -- a per-rank "
                         "proxy, not a multi-GPU measurement")
    ap.add_argument("--collective", choices=["auto", "torch", "rccl"], default="auto",
                    help="prove at N > 1: all-gathers through the driver's own RCCL communicator "
                         "(rccl: no Python on the exchange path; the default with one GPU per rank) or "
                         "torch.distributed's process group (torch: a ctypes callback per exchange; the "
                         "default when the ranks share one device, which RCCL refuses)")
    return ap


def rank_evidence(wl, rank: int, local_rank: int, dev, elapsed_s: float, steps: int, world: int) -> dict:
    """One rank's record for the N > 1 line (bench.py main): where it ran, what the RCCL
    communicator reports (when the workload uses the driver's own, native.RcclCollective.info),
    and its own timings before the max over ranks."""
    import socket

    import torch

    p = torch.cuda.get_device_properties(dev)
    rec = {
        "rank": rank,
        "local_rank": local_rank,
        "hostname": socket.gethostname(),
        "device": torch.cuda.current_device(),
        "pci_bus_id": "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id),
        "gpu": p.name,
        "collective": getattr(wl, "collective_kind", "torch"),
        "ms_per_step": round(elapsed_s * 1e3 / steps, 3),
    }
    coll = getattr(wl, "coll", None)
    if coll is not None and hasattr(coll, "info"):
        try:
            rec.update(coll.info())
        except Exception as e:  # the record is evidence, not the measurement: say what failed
            rec["nccl_info_error"] = str(e)
    try:
        thr, _ = wl.throughput(world, elapsed_s * 1e3 / steps)
        if isinstance(thr, dict) and "stage_ms" in thr:
            rec["stage_ms"] = thr["stage_ms"]
    except Exception:
        pass
    return rec


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n: int) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: start N ranks through
    torch.distributed.run as a CHILD process (this process never touches the GPU and never execs),
    let rank 0's JSON line through on the inherited stdout, and exit with the launcher's status
    (non-zero if any rank failed)."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py")]
    cmd += sys.argv[1:]
    print(f"bench.py: --gpus {n} without WORLD_SIZE: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr,
          flush=True)
    return subprocess.call(cmd)


def main() -> int:
    args = make_parser().parse_args()
    if args.steps is None:
        args.steps = 3 if args.workload == "prove" else 10
    if args.warmup is None:
        args.warmup = 1 if args.workload == "prove" else 3
    if args.gpus < 1:
        print(f"bench.py: --gpus must be >= 1 (got {args.gpus})", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return self_launch(args.gpus)  # before any GPU call: the parent only waits

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        # a run whose rank count differs from --gpus would time the wrong configuration
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # EON_BENCH_BACKEND=gloo and EON_BENCH_ONE_DEVICE=1 rehearse the N > 1 code path with every
    # rank on cuda:0 (a one-GPU box); the timings of such a run mean nothing
    backend = os.environ.get("EON_BENCH_BACKEND", "nccl")
    local_dev = 0 if os.environ.get("EON_BENCH_ONE_DEVICE") == "1" else local_rank
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from plonky3_eon_amd import Context

    ctx = Context(local_dev)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    wl = {"lde": LdeWorkload, "msm": MsmWorkload, "prove": ProveWorkload, "ntt4": FourStepWorkload,
          "msm-shard": MsmShardWorkload, "quotient": QuotientWorkload,
          "verify": VerifyWorkload}[args.workload](args, ctx, dev, rank)

    if args.serial:
        ctx.set_serial(True)
    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    sclk = SclkSampler(dev).start()
    t0 = time.perf_counter()
    for i in range(args.steps):
        wl.step()
        print(f"step {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms since start", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    sclk_stats = sclk.stop()
    if world > 1:
        dist.barrier()
    # per-launch HIP-event timings come from extra steps after the timed region, run in serial
    # mode (eon_ctx_set_serial: every kernel on the context stream, none on the MSM / opening side
    # streams), so that each launch's duration is its own and not shared with the kernels of the
    # other streams -- the same durations `rocprofv3 --kernel-trace` reports for `--serial`
    # (profiles/r02_*_kernel_stats.csv)
    prof_steps = max(1, min(args.steps, 2))
    ctx.set_serial(True)
    wl.step()  # warm the serial path's workspaces
    torch.cuda.synchronize()
    ctx.profile(True)
    t_p0 = time.perf_counter()
    for _ in range(prof_steps):
        wl.step()
    torch.cuda.synchronize()
    serial_ms = (time.perf_counter() - t_p0) * 1e3 / prof_steps
    prof = ctx.profile_report()
    ctx.profile(False)
    ctx.set_serial(args.serial)
    # the clock the chip holds under this VALU load, and the product peak at that clock, measured
    # now on this box (eon_diag_clock_probe; MI355X_MICROARCH.md DVFS item 6): ~2 s of the
    # roofline denominator's own product chain, stamped with s_memtime / s_memrealtime
    clock = None
    if not args.no_clock_probe:
        clock = ctx.clock_probe(160, 1024)
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    ranks = None
    if world > 1:
        # what each rank ran on and saw, gathered to rank 0: the device ordinal and PCI address
        # torch reports, the RCCL communicator's own view (ncclCommCount / ncclCommUserRank /
        # ncclCommCuDevice, and that device's PCI bus id), and the rank's own timings -- so that
        # the N-GPU line shows N ranks on N distinct GPUs under one N-rank communicator
        ranks = [None] * world
        dist.all_gather_object(ranks, rank_evidence(wl, rank, local_rank, dev, elapsed, args.steps, world))
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = elapsed * 1e3 / args.steps
    kname, kst = max(prof.items(), key=lambda kv: kv[1]["total_ms"])
    avg_ms = kst["total_ms"] / kst["launches"]
    bytes_per_launch = kst["alg_bytes"] / kst["launches"]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    gpu_total_ms = sum(v["total_ms"] for v in prof.values()) / prof_steps
    workload, gbatch, seq, par = wl.describe(world)
    thr, mulmods = wl.throughput(world, ms_per_step)

    roof = {
        "bound": "hbm",
        "kernel": kname,
        "achieved": _sig(achieved),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": _sig(achieved / HBM_PEAK_GBPS),
        "traffic": None,
        "avg_launch_ms": round(avg_ms, 4),
        "alg_bytes_per_launch": int(bytes_per_launch),
        "timing": "HIP events on the launch stream over %d serialized profiled steps after the timed "
                  "region (eon_ctx_set_serial: no kernel overlap), %.1f ms per serialized step" % (prof_steps, serial_ms),
        "kernel_ms_per_step": round(kst["total_ms"] / prof_steps, 3),
        "kernels": prof,
    }
    step_bytes = getattr(wl, "alg_bytes_per_step", None)
    if step_bytes:
        # a DFT/LDE is a chain of NTT passes (k_ntt_pass29 variants, the twiddle pack of the
        # four-step): section 8(d) prices the whole transform, so the roofline is its algorithmic
        # bytes over the step's total (serialized) kernel time
        roof["kernel"] = "all %d launches of the step (%s)" % (
            sum(v["launches"] for v in prof.values()) // prof_steps, ", ".join(sorted(prof)))
        roof["avg_launch_ms"] = round(gpu_total_ms, 4)
        roof["alg_bytes_per_launch"] = int(step_bytes)
        roof["achieved"] = _sig(step_bytes / (gpu_total_ms * 1e-3) / 1e9)
        roof["frac"] = _sig(step_bytes / (gpu_total_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS)
        roof["kernel_ms_per_step"] = round(gpu_total_ms, 3)
    if kst.get("design_bytes"):
        # what the kernel's access pattern moves (fixed-base table gathers) vs section 8(d)'s bytes
        dpl = kst["design_bytes"] / kst["launches"]
        roof["design_bytes_per_launch"] = int(dpl)
        roof["design_GBps"] = round(dpl / (avg_ms * 1e-3) / 1e9, 2)
    kmm = kst.get("alg_mulmods", 0)
    if kmm:
        rate = kmm / kst["launches"] / (avg_ms * 1e-3)
        roof["valu"] = {
            "binding": True,
            "alg_mulmods_per_launch": int(kmm / kst["launches"]),
            "achieved_mulmod_per_s": round(rate, 1),
            "peak_mulmod_per_s": MULMOD_PEAK_PER_S,
            "frac": round(rate / MULMOD_PEAK_PER_S, 4),
        }
        if clock:
            # the same kernel against the product rate this box sustained at the clock it held
            roof["valu"]["peak_live_mulmod_per_s"] = round(clock["products_per_s"], 1)
            roof["valu"]["frac_live"] = round(rate / clock["products_per_s"], 4)
            if kname == "k_piece_sum":
                # the piece sums against their own instruction-issue floor at this clock: the gfx950
                # ISA of the loop weighted by the measured issue cost of each instruction
                # (tools/isa_count.py --costs, tools/ubench_isa2.hip)
                adds = rate / 10  # 10 algorithmic products per XYZZ mixed addition
                floor = SIMDS * 64 * clock["clock_mhz_median"] * 1e6 / PIECE_ISSUE_CYCLES
                roof["valu"]["issue_floor"] = {
                    "cycles_per_wave_addition": PIECE_ISSUE_CYCLES,
                    "additions_per_s": round(adds, 1),
                    "floor_additions_per_s": round(floor, 1),
                    "frac": round(adds / floor, 4),
                    "source": PIECE_ISSUE_SOURCE,
                }
    if mulmods is not None:
        roof["valu_whole_step"] = {
            "achieved_mulmod_per_s": round(mulmods / (gpu_total_ms * 1e-3), 1),
            "frac": round(mulmods / (gpu_total_ms * 1e-3) / MULMOD_PEAK_PER_S, 4),
        }
        if "valu" not in roof:
            roof["valu"] = dict(roof["valu_whole_step"], binding=True,
                                peak_mulmod_per_s=MULMOD_PEAK_PER_S)
    if getattr(wl, "latency_bound", False):
        # a handful of pairs: single-thread Miller loops and final exponentiation chains, bound by
        # their dependent-instruction latency, not by HBM or the VALU throughput
        roof["bound"] = "latency"
        roof["hbm_frac"] = roof["frac"]
    if "valu" in roof:
        # the binding resource is the VALU issue of the 256-bit Montgomery products (SURVEY.md
        # 8(d)); achieved / peak / frac stay the HBM figures of section 8(d)'s algorithmic bytes
        roof["bound"] = "valu"
        roof["valu"]["unit"] = "mulmod/s"
        roof["hbm_frac"] = roof["frac"]
    result = {
        "metric": METRIC,
        "value": round(ms_per_step, 3),
        "unit": "ms",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": False,
        "scaling": getattr(wl, "scaling", "weak"),
        "vs_baseline": None,
        "dtype": "bn254 Fr/Fq (256-bit Montgomery: u32x8 in HBM, u29x9 MSM accumulators)",
        "data": "synthetic uniform Fr, resident in HBM",
        "config": {"workload": workload, "global_batch": gbatch, "seq_len": seq, "parallelism": par},
        "throughput": thr,
        "gpu_sclk": sclk_stats,
        "gpu_clock_inkernel_mhz": round(clock["clock_mhz_median"], 1) if clock else None,
        "gpu_clock_probe": ({k: round(v, 4 if k == "ms_per_launch" else 1) for k, v in clock.items()} | {
            "source": "eon_diag_clock_probe after the timed region: 161 launches of a radix-2^29 product chain "
                      "(4096 x 256 threads, 2 chains, 1024 products each), median over blocks of "
                      "delta s_memtime / delta s_memrealtime x 100 MHz"}) if clock else None,
        "roofline": roof,
        "cpu_baseline": None,
    }
    # PMC traffic of THIS round's build only (tools/gpu_pmc.sh -> profiles/<round>/traffic_*.json,
    # stamped with the commit it measured); an older round's file describes another build
    traffic_file = ROOT / "profiles" / TRAFFIC_ROUND / f"traffic_{args.workload}.json"
    if traffic_file.exists():
        try:
            tf = json.loads(traffic_file.read_text())
            if tf.get("kernel") == kname and tf.get("workload") == workload:
                roof["traffic"] = tf.get("bytes_per_launch")
                roof["traffic_source"] = ("%s (commit %s; raw FETCH_SIZE %.3g GB + WRITE_SIZE %.3g GB per launch; "
                                          "the x2 streaming-read correction is not applied to these gathers)") % (
                    traffic_file.relative_to(ROOT), tf.get("commit", "?"), tf["fetch_size_kb_per_launch"] * 1024 / 1e9,
                    tf["write_size_kb_per_launch"] * 1024 / 1e9)
                if tf.get("bytes_per_launch_x2_streaming"):
                    roof["traffic_x2_streaming_upper"] = tf["bytes_per_launch_x2_streaming"]
        except Exception:
            pass

    if ranks is not None:
        result["ranks"] = ranks
        result["distinct_gpus"] = len({r["pci_bus_id"] for r in ranks})
        counts = {r.get("nccl_comm_count") for r in ranks}
        result["rccl_comm_count"] = counts.pop() if len(counts) == 1 else sorted(counts, key=str)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = wl.cpu_baseline()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result))
    return 0


if __name__ == "__main__":
    sys.exit(main())
