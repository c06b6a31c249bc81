#!/bin/bash
# Prove bench under settings of one environment knob: knob_bench.sh VAR v1 v2 ...
set -o pipefail
mkdir -p gpurun_out/knob
var=$1; shift
for v in "$@"; do
  env $var=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/knob/${var}_$v.json 2>/dev/null || exit 1
  python3 -c "
import json; t=open('gpurun_out/knob/${var}_$v.json').read(); d=json.loads(t[t.index('{'):]); print('$var=$v:', d['value'], 'ms', d['throughput']['stage_ms'])"
done
