#!/bin/bash
# Round 5, session 19: the single MSM's fixed-base window width capped at 16 / 17 / 18
# (EON_MSM_CMAX_PRE; the library picks 19 at 2^20, 20 at 2^24) -- same-call A/B on msm, msm-shard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PROBE_WORKLOADS="msm msm-shard" timeout -k 10 1100 bash tools/gpu_probe.sh c16 c17 c18 || exit 1
