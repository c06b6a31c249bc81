#!/bin/bash
# Per-rank proxy of the 8-GPU lane-sharded prove: VECTOR_LEN 1 (164 columns) on one GPU, with a
# kernel trace of the last steps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/prove_steps.py 5 --vector-len 1 > gpurun_out/steps_vl1.txt 2>&1 \
 && cut -c1-300 gpurun_out/steps_vl1.txt \
 && rm -rf gpurun_out/trace_vl1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_vl1 -o p -- python3 tools/prove_steps.py 4 --vector-len 1 > gpurun_out/trace_vl1.txt 2>&1 \
 && find gpurun_out/trace_vl1 -name '*kernel_trace.csv'
