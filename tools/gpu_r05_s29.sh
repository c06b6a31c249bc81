#!/bin/bash
# Round 5, session 29: the single MSM's group tree writes the fixed-base results in place (no
# device copy) -- MSM tests, the same-call A/B against the previous commit (variants/libeonhip_head.so)
# on msm, then tools/gpu_r05_s28.sh (the two-rank one-GPU rehearsal of the N > 1 bench path).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s29.txt 2>&1 || { tail -30 $O/pytest_s29.txt; exit 1; }
tail -1 $O/pytest_s29.txt
PROBE_WORKLOADS="msm" timeout -k 10 600 bash tools/gpu_probe.sh head || exit 1
bash tools/gpu_r05_s28.sh
