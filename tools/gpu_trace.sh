#!/bin/bash
# Kernel trace (start/end timestamps) of one prove, for tools/timeline.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o prove -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${EXTRA} > gpurun_out/trace_bench.json 2> gpurun_out/trace.err
rc=$?
find gpurun_out/trace -name '*kernel_trace.csv' | head -3
exit $rc
