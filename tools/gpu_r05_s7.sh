#!/bin/bash
# Round 5, session 7: piece-sum chunk length for the single 2^20 MSM (16 pairs per thread by
# default; pt18: 32, pt17: 64), same-call A/B on configs[2].
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
PROBE_WORKLOADS=msm timeout -k 10 600 bash tools/gpu_probe.sh pt18 pt17 || exit 1
for f in default pt18 pt17 default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_msm_$f.json')); k=d['roofline']['kernels']
print('msm $f', d['value'], {n: round(v['total_ms'] / v['launches'], 3) for n, v in k.items()})"
done
