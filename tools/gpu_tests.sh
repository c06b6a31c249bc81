#!/bin/bash
# GPU parity tests (optionally a subset: pass pytest args), then smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export EON_TEST_HEARTBEAT=$PWD/gpurun_out/heartbeat.txt
ARGS=${@:-tests}
timeout -k 10 900 python -u -m pytest $ARGS -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.txt | tail -40
exit $rc
