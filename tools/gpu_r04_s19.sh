#!/bin/bash
# Round-4 session 19: MSM digits with four rows per thread and 16-byte stores (k_msm_digits4,
# default) vs one row per thread (variants/libeonhip_row1.so) -- MSM, KZG-open and prove tests,
# then the same-call A/B on the MSM and the prove with the digit kernel's profiled time.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s19.txt 2>&1 || { tail -30 $O/pytest_s19.txt; exit 1; }
tail -1 $O/pytest_s19.txt
timeout -k 10 1000 bash tools/gpu_probe.sh row1 || exit 1
for f in default row1 default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 2) for n, v in k.items() if 'digits' in n or 'sort' in n})"
done
