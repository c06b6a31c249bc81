#!/bin/bash
# Round 5, session 22: column MSMs split into at least 4 batches of >= 32 columns
# (EON_MSM_MIN_BATCHES=4) -- MSM-batch / prove / sharded tests, then the same-call A/B against the
# old batching (variants/libeonhip_mb1.so) on the emulated 8-rank prove and the 1-GPU prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py tests/test_distributed_gpu.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s22.txt 2>&1 || { tail -30 $O/pytest_s22.txt; exit 1; }
tail -1 $O/pytest_s22.txt
PROBE_WORKLOADS="prove" PROBE_ARGS="--emulate-world 8" timeout -k 10 900 bash tools/gpu_probe.sh mb1 || exit 1
cp $O/probe_summary.txt $O/probe_summary_e8.txt
for f in default mb1 default2; do
  python3 -c "import json; d=json.load(open('$O/probe_prove_$f.json')); print('$f', d['value'], d['throughput']['stage_ms'])"
done
PROBE_WORKLOADS="prove" timeout -k 10 900 bash tools/gpu_probe.sh mb1 || exit 1
