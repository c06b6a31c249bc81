"""Batched column MSM probe: n x cols scalars against the SRS table, as KzgPcs::commit runs it."""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np
import torch

from bench import synthetic_fr
from plonky3_eon_amd import Context
from plonky3_eon_amd.msm import MsmBases, srs_powers

ap = argparse.ArgumentParser()
ap.add_argument("--log-n", type=int, default=17)
ap.add_argument("--cols", type=int, default=128)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
ctx = Context(0)
n = 1 << a.log_n
bases = MsmBases(srs_powers(n, 12345, ctx), ctx, precompute=True)
m = torch.from_numpy(synthetic_fr(n, a.cols, 3).view(np.int64)).to("cuda:0")
bases.msm_columns(m)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    bases.msm_columns(m)
torch.cuda.synchronize()
print(f"msm_columns 2^{a.log_n} x {a.cols}: {(time.perf_counter() - t0) / a.reps * 1e3:.2f} ms", flush=True)
