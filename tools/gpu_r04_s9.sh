#!/bin/bash
# Round-4 session 9: the quotient kernels in radix-2^29 arithmetic -- the fused Poseidon2 fold and
# the generic interpreter (29-form register file, compiler-tracked value bounds) -- their tests
# (quotient vs oracle, generic == fused, register-file modes, prove parity), then the quotient
# benches and the headline prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_quotient.py tests/test_gpu_air_program.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_q29.txt 2>&1 || { tail -30 $O/pytest_q29.txt; exit 1; }
tail -1 $O/pytest_q29.txt
q() {  # name air
  timeout -k 10 300 python3 bench.py --workload quotient --air $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err &&
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['value'], d['roofline'].get('valu', {}).get('frac'))"
}
q qgen29_1 generic && q qfused29_1 fused && q qgen29_2 generic && q qfused29_2 fused &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_prove.json 2> $O/bench_prove.err &&
  python3 -c "
import json; d=json.load(open('$O/bench_prove.json')); print('prove', d['value'], d['throughput']['stage_ms'], d.get('gpu_sclk'))"
