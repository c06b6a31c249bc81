#!/bin/bash
# Round-4 session 10: the radix-2^29 generic interpreter with its four slots written out (no
# scratch): AIR-program tests, then the generic quotient bench twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_air_program.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_air29.txt 2>&1 || { tail -30 $O/pytest_air29.txt; exit 1; }
tail -1 $O/pytest_air29.txt
q() {  # name air
  timeout -k 10 300 python3 bench.py --workload quotient --air $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err &&
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['value'], d['roofline'].get('valu', {}).get('frac'))"
}
q qgen29u_1 generic && q qgen29u_2 generic
