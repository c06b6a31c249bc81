#!/bin/bash
# Round 5, session 16: k_scalar_or's atomics spread over 64 copies of its 8 words (4096 blocks) --
# MSM tests, the single-MSM timeline and the A/B against the previous commit (variants/libeonhip_head.so).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s16.txt 2>&1 || { tail -30 $O/pytest_s16.txt; exit 1; }
tail -1 $O/pytest_s16.txt
rm -rf $O/tl_msm
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_msm -o t -- \
  python3 bench.py --workload msm --steps 5 --warmup 2 --no-cpu-baseline --no-clock-probe > $O/tl_msm.json 2> $O/tl_msm.err \
  || { tail -5 $O/tl_msm.err; exit 1; }
python3 tools/step_timeline.py $(find $O/tl_msm -name '*kernel_trace.csv' | head -1) msm_digits 2 > $O/tl_msm16.txt || exit 1
grep -E "scalar_or|span" $O/tl_msm16.txt
PROBE_WORKLOADS="msm" timeout -k 10 900 bash tools/gpu_probe.sh head || exit 1
