#!/bin/bash
# Round 5, session 14: kernel timeline of the single 2^20 MSM (configs[2]) and of the 2^20 x 64 LDE
# (configs[1]): where the step's wall time goes besides kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for w in msm lde; do
  rm -rf $O/tl_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$w -o t -- \
    python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-clock-probe > $O/tl_$w.json 2> $O/tl_$w.err \
    || { tail -5 $O/tl_$w.err; exit 1; }
done
python3 tools/step_timeline.py $(find $O/tl_msm -name '*kernel_trace.csv' | head -1) msm_digits 2 > $O/tl_msm.txt || exit 1
python3 tools/step_timeline.py $(find $O/tl_lde -name '*kernel_trace.csv' | head -1) ntt_pass 1 > $O/tl_lde.txt || exit 1
tail -40 $O/tl_msm.txt
