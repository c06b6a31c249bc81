#!/bin/bash
# Transcript round: prove GPU tests (incl. Fiat-Shamir), the sharded native prove, prove timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_prove.py tests/test_gpu_kzg_open.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fs.txt 2>&1 \
 && tail -2 gpurun_out/pytest_fs.txt \
 && timeout -k 10 900 python -u -m pytest tests/test_distributed_gpu.py -x -q -k native --timeout 800 --timeout-method thread > gpurun_out/pytest_fs_dist.txt 2>&1 \
 && tail -2 gpurun_out/pytest_fs_dist.txt \
 && timeout -k 10 200 python -u tools/prove_steps.py 4 ${STEPS_ARGS:-} > gpurun_out/steps.txt 2>&1 \
 && cut -c1-300 gpurun_out/steps.txt
rc=$?
tail -25 gpurun_out/pytest_fs.txt | grep -v '^$' | tail -12
tail -12 gpurun_out/pytest_fs_dist.txt 2>/dev/null
exit $rc
