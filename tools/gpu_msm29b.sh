#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench_r29 > gpurun_out/ubench_r29.txt 2>&1 && head -1 gpurun_out/ubench_r29.txt \
 && timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_msm.txt 2>&1 \
 && tail -1 gpurun_out/pytest_msm.txt \
 && timeout -k 10 300 python bench.py --workload msm --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_msm29.json 2>gpurun_out/b_msm29.err \
 && timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_prove29.json 2>gpurun_out/b_prove29.err
rc=$?
tail -3 gpurun_out/pytest_msm.txt
for f in b_msm29 b_prove29; do python3 -c "
import json; d=json.load(open('gpurun_out/$f.json')); r=d['roofline']
print('$f', d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r.get('valu',{}).get('frac'), d.get('throughput',{}).get('stage_ms'))" 2>/dev/null; done
exit $rc
