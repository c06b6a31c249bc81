#!/bin/bash
# prove steps with rocm-smi clock/power samples alongside (diagnoses intermittent slow steps)
mkdir -p gpurun_out
( for i in $(seq 1 120); do date +%s.%N; rocm-smi -c -P -t 2>/dev/null | grep -E "sclk|Power|Temperature \(Sensor junction\)|mclk"; sleep 0.25; done ) > gpurun_out/smi.txt 2>&1 &
SMI=$!
timeout -k 10 200 python tools/prove_steps.py 8 > gpurun_out/steps_r29.txt 2>&1
EON_MSM_R32=1 timeout -k 10 200 python tools/prove_steps.py 5 > gpurun_out/steps_r32.txt 2>&1
kill $SMI
grep step gpurun_out/steps_r29.txt gpurun_out/steps_r32.txt | cut -c1-80
