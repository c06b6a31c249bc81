#!/bin/bash
# Round-4 session 14: tail-aware piece-sum chunk size (piece_log_chunk; EON_MSM_TAIL=0 is the old
# rule) -- MSM tests, then the same-call A/B on the headline prove and the emulated 8-rank prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s14.txt 2>&1 || { tail -30 $O/pytest_s14.txt; exit 1; }
tail -1 $O/pytest_s14.txt
b() {  # name tail args...
  local n=$1 t=$2; shift 2
  EON_MSM_TAIL=$t timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err &&
  python3 -c "import json; d=json.load(open('$O/bench_$n.json')); print('$n', d['value'], d['throughput']['stage_ms'])"
}
b e8_tail 1 --emulate-world 8 --steps 5 && b e8_old 0 --emulate-world 8 --steps 5 &&
b p_tail 1 --steps 5 && b p_old 0 --steps 5 &&
b e8_tail2 1 --emulate-world 8 --steps 5 && b e8_old2 0 --emulate-world 8 --steps 5 &&
b p_tail2 1 --steps 5 && b p_old2 0 --steps 5
