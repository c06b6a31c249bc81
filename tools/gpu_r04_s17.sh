#!/bin/bash
# Round-4 session 17: generic interpreter with raw (unreduced) leaf operands chosen per use by the
# compiler's bound tracking -- AIR-program and prove tests, then the same-call A/B against the
# previous interpreter (variants/libeonhip_airbase.so).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_air_program.py tests/test_gpu_prove.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_s17.txt 2>&1 || { tail -30 $O/pytest_s17.txt; exit 1; }
tail -1 $O/pytest_s17.txt
q() {  # name [lib]
  EON_LIB=$2 timeout -k 10 300 python3 bench.py --workload quotient --air generic --no-cpu-baseline > $O/bench_qr_$1.json 2> $O/bench_qr_$1.err &&
  python3 -c "import json; d=json.load(open('$O/bench_qr_$1.json')); print('$1', d['value'])"
}
V=$PWD/variants
q raw && q base $V/libeonhip_airbase.so && q raw2 && q base2 $V/libeonhip_airbase.so
