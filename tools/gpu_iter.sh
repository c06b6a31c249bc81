#!/bin/bash
# One iteration: MSM / opening / prove parity, per-step prove timings, kernel trace of 3 proves.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_msm_prove.txt 2>&1 \
 && tail -2 gpurun_out/pytest_msm_prove.txt \
 && timeout -k 10 200 python -u tools/prove_steps.py 6 > gpurun_out/steps.txt 2>&1 \
 && cut -c1-300 gpurun_out/steps.txt \
 && ${AB:-true} \
 && rm -rf gpurun_out/trace4 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace4 -o p -- python3 tools/prove_steps.py 3 > gpurun_out/trace4.txt 2>&1 \
 && find gpurun_out/trace4 -name '*kernel_trace.csv'
rc=$?
tail -30 gpurun_out/pytest_msm_prove.txt | grep -v '^$' | tail -15
exit $rc
