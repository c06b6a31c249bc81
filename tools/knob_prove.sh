#!/bin/bash
# prove_steps under several MSM scheduling knobs (env assignments as arguments)
mkdir -p gpurun_out
: > gpurun_out/knobs.txt
for kv in "$@"; do
  echo "== $kv" >> gpurun_out/knobs.txt
  env $kv timeout -k 10 120 python tools/prove_steps.py 3 2>&1 | grep step | cut -c1-200 >> gpurun_out/knobs.txt || break
done
cat gpurun_out/knobs.txt
