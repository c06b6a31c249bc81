#!/bin/bash
# Round measurement on one MI355X: GPU parity tests, the default bench line (configs[3] prove), and
# a rocprofv3 kernel-trace summary of the same workload in serial mode (bench.py --serial: every
# kernel alone on the device, so per-kernel averages are isolated and agree with the bench line's
# roofline timings).  Usage: [TESTS="tests/test_x.py ..."] tools/gpu_measure.sh [tests|notests] [workload]
# [noprof]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W=${2:-prove}
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
  tail -3 gpurun_out/pytest_gpu.txt
fi
timeout -k 10 600 python3 bench.py --workload $W > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err \
  || { tail -20 gpurun_out/bench_$W.err; exit 1; }
cat gpurun_out/bench_$W.json | cut -c1-400
[ "${3:-prof}" = noprof ] && exit 0
rm -rf gpurun_out/stats_$W
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_$W -o s -- \
  python3 bench.py --workload $W --serial --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/stats_$W.json 2> gpurun_out/stats_$W.err || { tail -20 gpurun_out/stats_$W.err; exit 1; }
find gpurun_out/stats_$W -name '*kernel_stats.csv'
