#!/bin/bash
# Round 5, session 6: (1) digit-sort variants: base, early (tile counts published before the
# ranking), early4 (+ 4-wide look-back), nolb (timing probe); (2) the whole GPU suite on the
# committed build; (3) kernel trace of the single 2^20 MSM (what remains between its kernels).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
: > $O/sort_variants6.txt
for v in base early early4 rts nolb; do
  timeout -k 10 180 variants/sort_check_$v big > $O/sort_check6_$v.txt 2>&1 || { tail -3 $O/sort_check6_$v.txt; exit 1; }
  echo "$v ok=$(grep -c '"ok":1' $O/sort_check6_$v.txt) bad=$(grep -c '"ok":0' $O/sort_check6_$v.txt) $(grep '"time"' $O/sort_check6_$v.txt | tr '\n' ' ')" | tee -a $O/sort_variants6.txt
done
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_s6.txt 2>&1 \
  || { tail -30 $O/pytest_s6.txt; exit 1; }
tail -1 $O/pytest_s6.txt
rm -rf $O/trace_msm
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_msm -o t -- \
  python3 bench.py --workload msm --steps 5 --warmup 2 --no-cpu-baseline --no-clock-probe > $O/trace_msm.json 2> $O/trace_msm.err \
  || { tail -20 $O/trace_msm.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/trace_msm.json')); print('msm', d['value'])"
