#!/bin/bash
# Round 5, session 31: the piece sums' next table entry prefetched into LDS by global_load_lds_dwordx4
# (EON_PIECE_PREFETCH=1) -- MSM / KZG-open / prove tests on the variant, then the same-call A/B on
# msm, msm-shard and prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
cp plonky3_eon_amd/libeonhip.so $O/.keep_default.so
cp variants/libeonhip_pf.so plonky3_eon_amd/libeonhip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s31.txt 2>&1 || { tail -30 $O/pytest_s31.txt; exit 1; }
tail -1 $O/pytest_s31.txt
cp $O/.keep_default.so plonky3_eon_amd/libeonhip.so && rm -f $O/.keep_default.so
PROBE_WORKLOADS="msm msm-shard prove" timeout -k 10 1000 bash tools/gpu_probe.sh pf || exit 1
for f in default pf default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 1) for n, v in k.items() if 'piece' in n})"
done
