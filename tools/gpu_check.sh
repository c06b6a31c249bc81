#!/bin/bash
# One GPU session: parity tests, a bench line, and a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; steps are chained so the first failure ends the run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.txt 2>&1 \
  && tail -3 gpurun_out/pytest_gpu.txt \
  && timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err \
  && cat gpurun_out/bench.json \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o lde --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/prof.err \
  && ls -R gpurun_out/prof | head -20
rc=$?
tail -5 gpurun_out/pytest_gpu.txt
exit $rc
