#!/bin/bash
# NTT tile sweep: parity (small DFT tests) and timing (LDE bench + prove) per (EON_NTT_TILE, EON_NTT_LOG_CB).
set -o pipefail
mkdir -p gpurun_out/nsw
for cfg in "10 -1" "10 0" "11 1" "11 2" "12 2"; do
  set -- $cfg
  export EON_NTT_TILE=$1 EON_NTT_LOG_CB=$2
  timeout -k 10 300 python -m pytest tests/test_gpu_dft_small.py -x -q -k "not ctx_passes1 and not ctx_passes3" > gpurun_out/nsw/t_$1_$2.log 2>&1 || { echo "tile=$1 cb=$2 parity FAIL"; tail -5 gpurun_out/nsw/t_$1_$2.log; exit 1; }
  timeout -k 10 300 python3 bench.py --workload lde --no-cpu-baseline > gpurun_out/nsw/l_$1_$2.json 2>/dev/null || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/nsw/p_$1_$2.json 2>/dev/null || exit 1
  python3 -c "
import json
def ld(f):
    t=open(f).read(); return json.loads(t[t.index('{'):])
l=ld('gpurun_out/nsw/l_$1_$2.json'); p=ld('gpurun_out/nsw/p_$1_$2.json')
print('tile=$1 cb=$2 parity ok | lde', l['value'], 'ms | prove', p['value'], 'ms', p['throughput']['stage_ms']['trace LDE (get_evaluations_on_domain)'])"
done
