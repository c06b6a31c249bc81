#!/bin/bash
# Round 5, session 20: 17..20-bit digit sorts in two passes of <= 10 bits (1024-bin k_sort_pass,
# EON_SORT_WIDE=1) -- sort_check (shapes incl. 17-20 bits; timing at 2^28 x 16 / 19 / 20 bits), MSM /
# KZG-open / prove / configs[4] tests, then the same-call A/B against three narrow passes
# (variants/libeonhip_narrow.so) on msm and msm-shard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 240 tools/sort_check big > $O/sort_check20.txt 2>&1 && ! grep -q '"ok":0' $O/sort_check20.txt || { tail -8 $O/sort_check20.txt; exit 1; }
grep -E '"time"|"huge"' $O/sort_check20.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py tests/test_gpu_configs4.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s20.txt 2>&1 || { tail -30 $O/pytest_s20.txt; exit 1; }
tail -1 $O/pytest_s20.txt
PROBE_WORKLOADS="msm msm-shard" timeout -k 10 900 bash tools/gpu_probe.sh narrow || exit 1
