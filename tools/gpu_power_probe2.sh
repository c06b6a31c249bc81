#!/bin/bash
# bench.py runs with rocm-smi clock/power samples alongside
mkdir -p gpurun_out
( for i in $(seq 1 400); do date +%s.%N; rocm-smi -c -P -t 2>/dev/null | grep -E "sclk|Power|Temperature \(Sensor junction\)"; sleep 0.1; done ) > gpurun_out/smi2.txt 2>&1 &
SMI=$!
for r in 1 2 3; do
  date +%s.%N >> gpurun_out/bench_marks.txt
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b$r.json 2> gpurun_out/b$r.err
  grep step gpurun_out/b$r.err
done
kill $SMI
