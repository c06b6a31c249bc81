#!/bin/bash
# Round-4 session 16: (1) generic interpreter -- multi-reader leaves loaded once into registers
# (OP_LOAD, default) vs every leaf an operand mode (EON_AIR_LOADS=0), plus timing probes (wrong
# results, the previous build's leaf code): leaf loads replaced by a register value (noload) or left
# unreduced (nored); (2) opening-bases finish with 2 / 4 lanes per row for short slices vs one lane
# (variants/libeonhip_splitoff.so) on the emulated 8-rank prove.  Tests first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_air_program.py tests/test_gpu_prove.py tests/test_gpu_kzg_open.py tests/test_distributed_gpu.py \
  -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_s16.txt 2>&1 || { tail -30 $O/pytest_s16.txt; exit 1; }
tail -1 $O/pytest_s16.txt
EON_AIR_LOADS=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_air_program.py -x -q -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_s16_noloads.txt 2>&1 || { tail -30 $O/pytest_s16_noloads.txt; exit 1; }
tail -1 $O/pytest_s16_noloads.txt
q() {  # name loads [lib]
  EON_AIR_LOADS=$2 EON_LIB=$3 timeout -k 10 300 python3 bench.py --workload quotient --air generic --no-cpu-baseline > $O/bench_qp_$1.json 2> $O/bench_qp_$1.err &&
  python3 -c "import json; d=json.load(open('$O/bench_qp_$1.json')); print('$1', d['value'])"
}
e() {  # name [lib]
  EON_LIB=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --emulate-world 8 --steps 5 > $O/bench_e8_$1.json 2> $O/bench_e8_$1.err &&
  python3 -c "import json; d=json.load(open('$O/bench_e8_$1.json')); print('e8_$1', d['value'], d['throughput']['stage_ms']['open'])"
}
V=$PWD/variants
q loads 1 && q noloads 0 && q probe_noload 0 $V/libeonhip_noload.so && q probe_nored 0 $V/libeonhip_nored.so && q loads2 1 && q noloads2 0 &&
e split && e splitoff $V/libeonhip_splitoff.so && e split2 && e splitoff2 $V/libeonhip_splitoff.so
