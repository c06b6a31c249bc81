#!/bin/bash
# Round 5, session 15: the first MSM batch's piece sums launched before the count read-back (the
# kernel reads the pair count on the device), and k_scalar_or at 256 blocks -- MSM / KZG-open /
# prove tests, the single-MSM timeline, and the same-call A/B against the previous commit
# (variants/libeonhip_head.so) on msm and prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s15.txt 2>&1 || { tail -30 $O/pytest_s15.txt; exit 1; }
tail -1 $O/pytest_s15.txt
rm -rf $O/tl_msm
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_msm -o t -- \
  python3 bench.py --workload msm --steps 5 --warmup 2 --no-cpu-baseline --no-clock-probe > $O/tl_msm.json 2> $O/tl_msm.err \
  || { tail -5 $O/tl_msm.err; exit 1; }
python3 tools/step_timeline.py $(find $O/tl_msm -name '*kernel_trace.csv' | head -1) msm_digits 2 > $O/tl_msm15.txt || exit 1
tail -25 $O/tl_msm15.txt
PROBE_WORKLOADS="msm prove" timeout -k 10 900 bash tools/gpu_probe.sh head || exit 1
