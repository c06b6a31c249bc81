#!/bin/bash
# Per-step prove timings, then a kernel trace of 3 proves (for tools/timeline.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/prove_steps.py 8 > gpurun_out/steps.txt 2>&1 \
 && cut -c1-300 gpurun_out/steps.txt \
 && rm -rf gpurun_out/trace4 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace4 -o p -- python3 tools/prove_steps.py 3 > gpurun_out/trace4.txt 2>&1 \
 && find gpurun_out/trace4 -name '*kernel_trace.csv'
