#!/bin/bash
# Round-4 check on one MI355X: the GPU suite, the headline bench, the emulated per-rank proves
# (bench.py --emulate-world), the host transcript microbench and the >2^30-pair sort check.
# Usage: tools/gpu_r04_check.sh [tests|notests]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
lscpu | grep -E "Model name|^CPU\(s\)|MHz" > $O/host_cpu.txt || true
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
  tail -2 $O/pytest_gpu.txt
fi
timeout -k 10 120 tools/ubench_transcript > $O/ubench_transcript.json && cat $O/ubench_transcript.json &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_prove.json 2> $O/bench_prove.err &&
  cut -c1-300 $O/bench_prove.json &&
for W in 8 4 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --emulate-world $W --steps 5 \
    > $O/bench_emul$W.json 2> $O/bench_emul$W.err || { tail -20 $O/bench_emul$W.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_emul$W.json')); print($W, d['value'], d['throughput']['stage_ms'])"
done &&
timeout -k 10 300 tools/sort_check huge > $O/sort_check_huge.txt 2>&1 && cat $O/sort_check_huge.txt
