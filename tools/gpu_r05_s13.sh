#!/bin/bash
# Round 5, session 13: the single MSM's weighted bucket reduction as two block scans
# (k_segment_scan29 + k_block_scan29, EON_SEG_SCAN=1) -- the whole GPU suite, then the same-call
# A/B against the per-segment double-and-add (variants/libeonhip_seg0.so) on msm and msm-shard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_s13.txt 2>&1 \
  || { tail -30 $O/pytest_s13.txt; exit 1; }
tail -1 $O/pytest_s13.txt
PROBE_WORKLOADS="msm msm-shard" timeout -k 10 900 bash tools/gpu_probe.sh seg0 || exit 1
