#!/bin/bash
# Round-4 exposure trace of the final build: kernel trace of an overlapped headline prove and
# tools/exposure.py over one steady-state period (what runs while no piece sum does).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
rm -rf $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o prove -- python3 bench.py --steps 1 \
  --warmup 1 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 tools/exposure.py $f > $O/prove_exposure.txt && cat $O/prove_exposure.txt
