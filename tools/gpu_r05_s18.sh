#!/bin/bash
# Round 5, session 18: the natural-order coset LDE as two DIT networks (bit-reversed gathers;
# EON_LDE_DIT=1) -- DFT tests, then the same-call A/B against the DIF inverse network
# (variants/libeonhip_ldedif.so) on lde, plus the MSM tests of session 17b's build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dft_small.py tests/test_gpu_dft_large.py tests/test_golden.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s18.txt 2>&1 || { tail -30 $O/pytest_s18.txt; exit 1; }
tail -1 $O/pytest_s18.txt
PROBE_WORKLOADS="lde" timeout -k 10 900 bash tools/gpu_probe.sh ldedif || exit 1
