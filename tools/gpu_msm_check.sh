#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_msm.py -x -q -m gpu > gpurun_out/pytest_msm.txt 2>&1 \
  && tail -2 gpurun_out/pytest_msm.txt \
  && timeout -k 10 400 python bench.py --workload msm --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_msm.json 2> gpurun_out/bench_msm.err \
  && python3 -c "
import json; d=json.load(open('gpurun_out/bench_msm.json'))
print('ms', d['ms_per_step'], d['throughput'])
for k,v in d['roofline']['kernels'].items(): print(' ', k, v['launches'], round(v['total_ms']/v['launches'],3))"
rc=$?; tail -5 gpurun_out/pytest_msm.txt; exit $rc
