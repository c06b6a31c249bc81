#!/bin/bash
# Round 5, session 10: kernel trace of the overlapped prove (3 proves) -> tools/exposure.py
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o prove -- python3 bench.py --steps 1 --warmup 2 --no-cpu-baseline --no-clock-probe > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
python3 tools/exposure.py $(find $O/trace -name '*kernel_trace.csv' | head -1) > $O/prove_exposure.txt && cat $O/prove_exposure.txt
