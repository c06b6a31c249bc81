#!/bin/bash
# Round 5, session 25: piece-sum chunks of up to 2^8 sorted pairs (EON_LOG_CHUNK_MAX=8; the prove's
# 2^29-pair batches then run 2^8-pair chunks) -- MSM / prove tests on the variant, then the
# same-call A/B on the 1-GPU and the emulated 8-rank prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
cp plonky3_eon_amd/libeonhip.so $O/.keep_default.so
cp variants/libeonhip_lcm8.so plonky3_eon_amd/libeonhip.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s25.txt 2>&1 || { tail -30 $O/pytest_s25.txt; exit 1; }
tail -1 $O/pytest_s25.txt
cp $O/.keep_default.so plonky3_eon_amd/libeonhip.so && rm -f $O/.keep_default.so
PROBE_WORKLOADS="prove" timeout -k 10 1000 bash tools/gpu_probe.sh lcm8 || exit 1
cp $O/probe_summary.txt $O/probe_summary_1gpu.txt
for f in default lcm8 default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 1) for n, v in k.items() if v['total_ms'] > 5})"
done
PROBE_WORKLOADS="prove" PROBE_ARGS="--emulate-world 8" timeout -k 10 900 bash tools/gpu_probe.sh lcm8 || exit 1
