#!/bin/bash
# Per-rank proxies of the lane-sharded prove (VECTOR_LEN 1 / 2 / 4 = one rank's share at 8 / 4 / 2
# GPUs), then a kernel trace of the VECTOR_LEN 1 prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/proxies.txt
for vl in 1 2 4; do
  echo "== vector-len $vl" >> gpurun_out/proxies.txt
  timeout -k 10 120 python -u tools/prove_steps.py 4 --vector-len $vl 2>&1 | grep step | cut -c1-260 >> gpurun_out/proxies.txt || exit 1
done
cat gpurun_out/proxies.txt
rm -rf gpurun_out/trace_vl1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_vl1 -o p -- python3 tools/prove_steps.py 3 --vector-len 1 > gpurun_out/trace_vl1.txt 2>&1
