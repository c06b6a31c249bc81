#!/bin/bash
# A/B of tuning builds (variants/libeonhip_<name>.so, built by `python -m plonky3_eon_amd._build
# variant <name> DEFINES` and copied to variants/) against the default library on the msm and prove
# workloads.  The box's tree is a scratch copy: each variant in turn replaces
# plonky3_eon_amd/libeonhip.so there, so that libeonprove.so (linked to libeonhip.so) uses it too.
# usage: tools/gpu_probe.sh <name>...
set -o pipefail
mkdir -p gpurun_out
[ $# -ge 1 ] || { echo "usage: $0 <variant>..."; exit 2; }
# PROBE_WORKLOADS (default "msm prove"): the bench.py workloads timed per library; PROBE_ARGS: extra
# bench.py arguments for every run (e.g. "--air generic")
run() {
  local line="$1"
  for w in ${PROBE_WORKLOADS:-msm prove}; do
    local st=10
    [ $w = prove ] && st=3
    timeout -k 10 300 python3 bench.py --workload $w $PROBE_ARGS --no-cpu-baseline --steps $st > gpurun_out/probe_${w}_$1.json \
      2>/dev/null || return 1
    line="$line $w $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" \
      gpurun_out/probe_${w}_$1.json)"
  done
  echo "$line" | tee -a gpurun_out/probe_summary.txt
}
: > gpurun_out/probe_summary.txt
cp plonky3_eon_amd/libeonhip.so gpurun_out/.libeonhip_default.so
run default || exit 1
for V in "$@"; do
  cp variants/libeonhip_$V.so plonky3_eon_amd/libeonhip.so && run $V || exit 1
done
cp gpurun_out/.libeonhip_default.so plonky3_eon_amd/libeonhip.so && rm -f gpurun_out/.libeonhip_default.so
run default2
