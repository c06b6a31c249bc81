#!/bin/bash
# Round 5, session 27: buckets per reduction segment 4 / 16 (EON_SEG; 8 by default) -- MSM / prove
# tests on seg4, then the same-call A/B on prove and msm with the bucket-reduction and group-finish
# times.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
cp plonky3_eon_amd/libeonhip.so $O/.keep_default.so
cp variants/libeonhip_seg4.so plonky3_eon_amd/libeonhip.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s27.txt 2>&1 || { tail -30 $O/pytest_s27.txt; exit 1; }
tail -1 $O/pytest_s27.txt
cp $O/.keep_default.so plonky3_eon_amd/libeonhip.so && rm -f $O/.keep_default.so
PROBE_WORKLOADS="prove msm" timeout -k 10 1100 bash tools/gpu_probe.sh seg4 seg16 || exit 1
for f in default seg4 seg16 default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 1) for n, v in k.items() if 'reduce' in n or 'finish' in n})"
done
