#!/bin/bash
# Round 5, session 26: digit-sort tiles of 1024 threads x 16 pairs (EON_SORT_THREADS=1024: half the
# tiles, so half the look-back steps; one block of 16 waves per CU instead of two of 8) --
# sort_check of both builds (shapes + 2^28 timing), MSM / prove tests on the variant, then the
# same-call A/B on msm and prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 240 tools/sort_check big > $O/sort_check26_512.txt 2>&1 && ! grep -q '"ok":0' $O/sort_check26_512.txt || { tail -8 $O/sort_check26_512.txt; exit 1; }
timeout -k 10 240 variants/sort_check_st1024 big > $O/sort_check26_1024.txt 2>&1 && ! grep -q '"ok":0' $O/sort_check26_1024.txt || { tail -8 $O/sort_check26_1024.txt; exit 1; }
grep -h '"time"' $O/sort_check26_512.txt $O/sort_check26_1024.txt
cp plonky3_eon_amd/libeonhip.so $O/.keep_default.so
cp variants/libeonhip_st1024.so plonky3_eon_amd/libeonhip.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s26.txt 2>&1 || { tail -30 $O/pytest_s26.txt; exit 1; }
tail -1 $O/pytest_s26.txt
cp $O/.keep_default.so plonky3_eon_amd/libeonhip.so && rm -f $O/.keep_default.so
PROBE_WORKLOADS="msm prove" timeout -k 10 1000 bash tools/gpu_probe.sh st1024 || exit 1
for f in default st1024 default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 1) for n, v in k.items() if 'sort' in n})"
done
