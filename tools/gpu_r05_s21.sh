#!/bin/bash
# Round 5, session 21: the digit kernels convert scalars out of Montgomery form with the radix-2^29
# product, the host result conversion inverts by binary extended Euclid -- sort_check (the new
# 17-20-bit shapes on the narrow passes), MSM / KZG-open / prove tests, then the same-call A/B
# against the previous commit (variants/libeonhip_head.so) on msm and prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 tools/sort_check > $O/sort_check21.txt 2>&1 && ! grep -q '"ok":0' $O/sort_check21.txt || { tail -8 $O/sort_check21.txt; exit 1; }
grep -c '"ok":1' $O/sort_check21.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s21.txt 2>&1 || { tail -30 $O/pytest_s21.txt; exit 1; }
tail -1 $O/pytest_s21.txt
PROBE_WORKLOADS="msm prove" timeout -k 10 900 bash tools/gpu_probe.sh head || exit 1
