#!/bin/bash
# Round-4 session 15: digit sort with 1024-thread tiles of 16384 pairs (variants/libeonhip_t1024.so:
# digit runs of ~64 pairs per tile instead of ~32, half the tiles to look back over) -- MSM tests on
# the variant, then the same-call A/B on the MSM and the headline prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
EON_LIB=$PWD/variants/libeonhip_t1024.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s15.txt 2>&1 || { tail -30 $O/pytest_s15.txt; exit 1; }
tail -1 $O/pytest_s15.txt
PROBE_WORKLOADS="msm prove" timeout -k 10 900 bash tools/gpu_probe.sh t1024 && cat $O/probe_summary.txt
