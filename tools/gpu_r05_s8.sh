#!/bin/bash
# Round 5, session 8: the few-group MSM reduction with interleaved independent products
# (add29_ilp / dbl29_ilp) and radix-2^29 block trees -- MSM / golden / prove tests, then the
# same-call A/B against the previous build (variants/libeonhip_segold.so) on the single MSM, the
# 2^24 MSM and the prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_golden.py tests/test_gpu_msm_batches.py tests/test_gpu_prove.py tests/test_gpu_kzg_open.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s8.txt 2>&1 || { tail -30 $O/pytest_s8.txt; exit 1; }
tail -1 $O/pytest_s8.txt
PROBE_WORKLOADS="msm msm-shard prove" timeout -k 10 1000 bash tools/gpu_probe.sh segold || exit 1
for f in default segold default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_msm_$f.json')); k=d['roofline']['kernels']
print('msm $f', d['value'], {n: round(v['total_ms'] / v['launches'], 3) for n, v in k.items()})"
done
