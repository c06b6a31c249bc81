#!/bin/bash
# Bench the default library and tuning variants (build/variants/libeonhip_<name>.so) on the MSM and
# prove workloads; prints one line per (variant, workload).
set -o pipefail
mkdir -p gpurun_out/var
for v in default "$@"; do
  if [ "$v" = default ]; then unset EON_LIB; else export EON_LIB=$PWD/build/variants/libeonhip_$v.so; fi
  for w in msm prove; do
    timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/var/${v}_$w.json 2>/dev/null || exit 1
    python3 -c "
import json; t=open('gpurun_out/var/${v}_$w.json').read(); d=json.loads(t[t.index('{'):]); r=d['roofline']
ks=r['kernels']; ps=ks.get('k_piece_sum',{})
print('$v', '$w', d['value'], 'ms | piece_sum avg', round(ps.get('total_ms',0)/max(ps.get('launches',1),1),3), '| valu', r.get('valu',{}).get('frac'))"
  done
done
