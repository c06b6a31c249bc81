#!/bin/bash
# Round 5, session 3: digit-sort ranking with v_bitop3 masks (4 VALU per digit bit instead of the
# 64-bit select form) -- tools/sort_check against the host stable sort, MSM / KZG-open / prove
# tests, then the same-call A/B against the round-4 ranking (variants/libeonhip_soldrank.so).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 tools/sort_check > $O/sort_check.txt 2>&1 && grep -c '"ok":1' $O/sort_check.txt && ! grep -q '"ok":0' $O/sort_check.txt || { tail -5 $O/sort_check.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s3.txt 2>&1 || { tail -30 $O/pytest_s3.txt; exit 1; }
tail -1 $O/pytest_s3.txt
timeout -k 10 1000 bash tools/gpu_probe.sh soldrank || exit 1
for f in default soldrank default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
m=json.load(open('$O/probe_msm_$f.json'))
print('$f', d['value'], m['value'], {n: round(v['total_ms'], 2) for n, v in k.items() if 'digits' in n or 'sort' in n})"
done
