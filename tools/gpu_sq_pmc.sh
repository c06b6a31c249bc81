#!/bin/bash
# SQ counters (issue/stall breakdown) of the prove's kernels: one pass, counters only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/sq_pmc
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --kernel-trace -d gpurun_out/sq_pmc -o sq --output-format csv -- python3 tools/prove_steps.py 1 > gpurun_out/sq_pmc.txt 2>&1
rc=$?
find gpurun_out/sq_pmc -name '*.csv' | head
exit $rc
