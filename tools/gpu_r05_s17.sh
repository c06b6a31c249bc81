#!/bin/bash
# Round 5, session 17b: k_segment_sum29 with the segment length from seg29_for (4 at 2^18 buckets,
# 8 at 2^19) and k_scalar_or in radix 2^29 -- MSM tests, then the same-call A/B against the
# previous commit (head) on msm, msm-shard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_configs4.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s17.txt 2>&1 || { tail -30 $O/pytest_s17.txt; exit 1; }
tail -1 $O/pytest_s17.txt
PROBE_WORKLOADS="msm msm-shard" timeout -k 10 900 bash tools/gpu_probe.sh head || exit 1
