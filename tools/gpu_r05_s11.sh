#!/bin/bash
# Round 5, session 11: DIT NTT passes normalising every third stage (EON_NTT_NORM_EVERY=3) --
# DFT / LDE / prove tests, then the same-call A/B against every other stage
# (variants/libeonhip_norm2.so) on the lde and prove workloads.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 tools/ubench_mad_nop > $O/ubench_mad_nop.txt 2>&1 && cat $O/ubench_mad_nop.txt || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_dft_small.py tests/test_gpu_dft_large.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s11.txt 2>&1 || { tail -30 $O/pytest_s11.txt; exit 1; }
tail -1 $O/pytest_s11.txt
PROBE_WORKLOADS="lde prove" timeout -k 10 900 bash tools/gpu_probe.sh norm2 || exit 1
