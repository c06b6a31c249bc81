#!/bin/bash
# Round 5, session 24: repeat of session 23's A/B with 2^30-pair batches added (bp29, bp30 against
# the default 2^28) on the 1-GPU and the emulated 8-rank prove; prove tests on bp30.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
cp plonky3_eon_amd/libeonhip.so $O/.keep_default.so
cp variants/libeonhip_bp30.so plonky3_eon_amd/libeonhip.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm_batches.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s24.txt 2>&1 || { tail -30 $O/pytest_s24.txt; exit 1; }
tail -1 $O/pytest_s24.txt
cp $O/.keep_default.so plonky3_eon_amd/libeonhip.so && rm -f $O/.keep_default.so
PROBE_WORKLOADS="prove" timeout -k 10 1000 bash tools/gpu_probe.sh bp29 bp30 || exit 1
cp $O/probe_summary.txt $O/probe_summary_1gpu.txt
PROBE_WORKLOADS="prove" PROBE_ARGS="--emulate-world 8" timeout -k 10 900 bash tools/gpu_probe.sh bp29 bp30 || exit 1
