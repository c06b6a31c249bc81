#!/bin/bash
# Radix-4 rounds in the r29 NTT pass (EON_NTT_R4=1): DFT parity, LDE bench A/B, prove A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--workload lde --steps 5 --warmup 2 --no-cpu-baseline"
EON_NTT_R4=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_dft_small.py tests/test_gpu_dft_large.py tests/test_golden.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r4.txt 2>&1 \
 && tail -2 gpurun_out/pytest_r4.txt \
 && for kv in X=1 EON_NTT_R4=1 "EON_NTT_R4=1 EON_NTT_TPB=256" X=1; do echo "== $kv"; env $kv timeout -k 10 200 python bench.py $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['avg_launch_ms'])" || exit 1; done \
 && bash tools/knob_prove.sh X=1 EON_NTT_R4=1 "EON_NTT_R4=1 EON_NTT_TPB=256" | grep -E "==|step 2" | cut -c1-200
rc=$?
tail -15 gpurun_out/pytest_r4.txt | grep -v '^$' | tail -8
exit $rc
