#!/bin/bash
# Round 5, session 23: column MSM batches of up to 2^29 digit pairs (EON_MSM_BATCH_LOG_PAIRS=29:
# the prove's 1312 columns in 6 batches of <= 256, a rank's 164 in one) against 2^28 -- prove /
# MSM-batch tests on the variant, then the same-call A/B on the 1-GPU and the emulated 8-rank prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
cp plonky3_eon_amd/libeonhip.so $O/.keep_default.so
cp variants/libeonhip_bp29.so plonky3_eon_amd/libeonhip.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm_batches.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s23.txt 2>&1 || { tail -30 $O/pytest_s23.txt; exit 1; }
tail -1 $O/pytest_s23.txt
cp $O/.keep_default.so plonky3_eon_amd/libeonhip.so && rm -f $O/.keep_default.so
PROBE_WORKLOADS="prove" timeout -k 10 900 bash tools/gpu_probe.sh bp29 || exit 1
cp $O/probe_summary.txt $O/probe_summary_1gpu.txt
PROBE_WORKLOADS="prove" PROBE_ARGS="--emulate-world 8" timeout -k 10 900 bash tools/gpu_probe.sh bp29 || exit 1
