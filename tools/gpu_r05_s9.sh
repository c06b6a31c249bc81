#!/bin/bash
# Round 5, session 9: one memset for every sort pass's tile counter and status words --
# sort_check (incl. the 2^28 timing), MSM / prove tests, the single-MSM bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 180 tools/sort_check big > $O/sort_check9.txt 2>&1 && ! grep -q '"ok":0' $O/sort_check9.txt || { tail -5 $O/sort_check9.txt; exit 1; }
grep '"time"' $O/sort_check9.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s9.txt 2>&1 || { tail -30 $O/pytest_s9.txt; exit 1; }
tail -1 $O/pytest_s9.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload msm --no-cpu-baseline --no-clock-probe > $O/bench_msm9_$i.json 2> $O/bench_msm9.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_msm9_$i.json')); print('msm', d['value'])"
done
