#!/bin/bash
# Round-4 session 23: bucket starts with sixteen keys per thread (four 16-byte loads in flight) vs
# one 16-byte load per thread (variants/libeonhip_mbase.so: the previous msm.hip) -- sort_check, MSM /
# KZG-open / prove tests, then the same-call A/B on the MSM and the prove with the profiled times.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 tools/sort_check > $O/sort_check.txt 2>&1 && grep -c '"ok":1' $O/sort_check.txt && ! grep -q '"ok":0' $O/sort_check.txt || { tail -5 $O/sort_check.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s22.txt 2>&1 || { tail -30 $O/pytest_s22.txt; exit 1; }
tail -1 $O/pytest_s22.txt
timeout -k 10 1000 bash tools/gpu_probe.sh mbase || exit 1
for f in default mbase default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 2) for n, v in k.items() if 'start' in n or 'sort' in n})"
done
