#!/bin/bash
# NTT tile/threads sweep on the configs[1] LDE (timing only; parity is covered by pytest -m gpu).
mkdir -p gpurun_out
for cfg in "128 -1" "256 -1" "512 -1" "512 2" "256 2" "512 1"; do
  set -- $cfg
  EON_NTT_TPB=$1 EON_NTT_LOG_CB=$2 timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sweep.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sweep.json'));print('tpb=$1 log_cb=$2', d['ms_per_step'], {k:round(v['total_ms']/v['launches'],3) for k,v in d['roofline']['kernels'].items()})"
done
