#!/bin/bash
# MSM / opening / prove parity tests, then per-step prove timings (diagnostic).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_msm_prove.txt 2>&1 \
 && tail -2 gpurun_out/pytest_msm_prove.txt \
 && timeout -k 10 200 python -u tools/prove_steps.py 4 > gpurun_out/steps.txt 2>&1 \
 && cut -c1-300 gpurun_out/steps.txt \
 && EON_MSM_PREP_SERIAL=1 timeout -k 10 200 python -u tools/prove_steps.py 3 > gpurun_out/steps_serial.txt 2>&1 \
 && cut -c1-300 gpurun_out/steps_serial.txt
rc=$?
grep -E 'PASS|FAIL|Error|error' gpurun_out/pytest_msm_prove.txt | tail -40
exit $rc
