#!/bin/bash
# Round-4 session 13: generic interpreter variants, same call -- registers 0 (v1) or 0 and 1 (v2)
# in VGPRs, v2 with 128-thread blocks, against the radix-2^29 default (all registers in LDS).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
q() {  # name [lib]
  EON_LIB=$2 timeout -k 10 300 python3 bench.py --workload quotient --air generic --no-cpu-baseline > $O/bench_qg_$1.json 2> $O/bench_qg_$1.err &&
  python3 -c "import json; d=json.load(open('$O/bench_qg_$1.json')); print('$1', d['value'])"
}
V=$PWD/variants
q v2 $V/libeonhip_v2.so && q v2w5 $V/libeonhip_v2w5.so && q v2b $V/libeonhip_v2.so && q v2w5b $V/libeonhip_v2w5.so
