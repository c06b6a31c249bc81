#!/bin/bash
# A/B of a tuning build (variants/libeonhip_<name>.so, built by `python -m plonky3_eon_amd._build
# variant <name> DEFINES` and copied to variants/) against the default library on the msm and prove
# workloads.  The box's tree is a scratch copy: the variant replaces plonky3_eon_amd/libeonhip.so
# there for the second half, so that libeonprove.so (linked to libeonhip.so) uses it too.
# usage: tools/gpu_probe.sh <name>
set -o pipefail
mkdir -p gpurun_out
V=${1:?variant name}
run() {
  timeout -k 10 200 python3 bench.py --workload msm --no-cpu-baseline > gpurun_out/probe_msm_$1.json 2>/dev/null &&
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 > gpurun_out/probe_prove_$1.json 2>/dev/null
}
run default && cp variants/libeonhip_$V.so plonky3_eon_amd/libeonhip.so && run $V
