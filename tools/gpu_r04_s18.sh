#!/bin/bash
# Round-4 session 18: occupancy bounds of the bucket reduction (k_bucket_reduce29 at 4 waves per
# SIMD, br4: 128 VGPRs with spills, vs 3 at 157) and the group finish (gf3: 3 waves with spills, vs
# 2 at 228 VGPRs) -- MSM tests on each variant, then the same-call A/B on the MSM and the prove,
# with the per-kernel times of the prove's profiled steps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for v in br4 gf3; do
  EON_LIB=$PWD/variants/libeonhip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py -x -q -m gpu \
    --timeout 300 --timeout-method thread > $O/pytest_s18_$v.txt 2>&1 || { tail -30 $O/pytest_s18_$v.txt; exit 1; }
  tail -1 $O/pytest_s18_$v.txt
done
timeout -k 10 1000 bash tools/gpu_probe.sh br4 gf3 || exit 1
for f in default br4 gf3 default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 2) for n, v in k.items() if 'reduce' in n or 'finish' in n})"
done
