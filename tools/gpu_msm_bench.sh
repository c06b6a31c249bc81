#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload msm --steps 5 --warmup 2 > gpurun_out/bench_msm.json 2> gpurun_out/bench_msm.err \
  && cat gpurun_out/bench_msm.json \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_msm -o msm --output-format csv -- python3 bench.py --workload msm --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_msm.err \
  && cat gpurun_out/prof_msm/msm_kernel_stats.csv
