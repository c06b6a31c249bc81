#!/bin/bash
# Round-4 session 11: scratch-free hot loops -- k_piece_sum29's pair quads picked from registers
# (they sat in scratch behind a pointer select: eight scratch stores per quad and a flat load per
# pair), k_eval_block's accumulators in registers, the fused quotient's unrolled state loops and
# pre-converted round constants, the interpreter's four written-out slots.  Tests first, then the
# same-call A/B against variants/libeonhip_base.so (the msm.hip / kzg.hip of the previous commit)
# on the MSM and the headline prove, then both quotient benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_quotient.py \
  tests/test_gpu_air_program.py tests/test_gpu_prove.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_s11.txt 2>&1 \
  || { tail -30 $O/pytest_s11.txt; exit 1; }
tail -1 $O/pytest_s11.txt
timeout -k 10 900 bash tools/gpu_probe.sh base || exit 1
q() {  # name air
  timeout -k 10 300 python3 bench.py --workload quotient --air $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err &&
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['value'], d['roofline'].get('valu', {}).get('frac'))"
}
q qgen29u generic && q qfused29u fused
