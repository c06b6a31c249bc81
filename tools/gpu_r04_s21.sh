#!/bin/bash
# Round-4 session 21: fused quotient with carry-free Horner steps and S-box inputs (add29_lazy where
# the sum only feeds a product) -- quotient and prove tests, then the same-call A/B against the
# previous fold (variants/libeonhip_qbase.so).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_quotient.py tests/test_gpu_air_program.py tests/test_gpu_prove.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_s21.txt 2>&1 || { tail -30 $O/pytest_s21.txt; exit 1; }
tail -1 $O/pytest_s21.txt
q() {  # name [lib]
  EON_LIB=$2 timeout -k 10 300 python3 bench.py --workload quotient --no-cpu-baseline > $O/bench_qf_$1.json 2> $O/bench_qf_$1.err &&
  python3 -c "import json; d=json.load(open('$O/bench_qf_$1.json')); print('$1', d['value'])"
}
V=$PWD/variants
q lazy && q base $V/libeonhip_qbase.so && q lazy2 && q base2 $V/libeonhip_qbase.so
