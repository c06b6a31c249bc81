#!/bin/bash
# Prove bench with the MSM sort stream on 0 (unmasked) / k dedicated CUs.
set -o pipefail
mkdir -p gpurun_out/scu
for k in 0 "$@"; do
  EON_MSM_SORT_CUS=$k timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/scu/p$k.json 2>/dev/null || exit 1
  python3 -c "
import json; t=open('gpurun_out/scu/p$k.json').read(); d=json.loads(t[t.index('{'):]); print('sort CUs $k:', d['value'], 'ms', d['throughput']['stage_ms'])"
done
