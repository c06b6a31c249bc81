#!/bin/bash
# Round-4 session 8: generic quotient with register 0 in VGPRs (5 waves per SIMD) vs LDS only
# (EON_AIR_VREGS=0), its tests, then issue/stall PMC of the interpreter and of the fused Poseidon2
# quotient kernel (tools/gpu_pmc_kernel.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_air_program.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_air.txt 2>&1 || { tail -30 $O/pytest_air.txt; exit 1; }
tail -1 $O/pytest_air.txt
qgen() {  # name [EON_AIR_VREGS]
  EON_AIR_VREGS=$2 timeout -k 10 300 python3 bench.py --workload quotient --air generic --no-cpu-baseline \
    > $O/bench_qgen_$1.json 2> $O/bench_qgen_$1.err || { tail -20 $O/bench_qgen_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/bench_qgen_$1.json')); print('qgen $1', d['value'], d['roofline']['valu']['frac'])"
}
qgen v1 1 && qgen v0 0 && qgen v1b 1 && qgen v0b 0 &&
BENCH_EXTRA="--air generic" timeout -k 10 400 bash tools/gpu_pmc_kernel.sh quotient k_air_quotient qgen &&
timeout -k 10 400 bash tools/gpu_pmc_kernel.sh quotient k_p2_quotient qfused
