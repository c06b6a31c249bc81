#!/bin/bash
# Round 5, session 32: DIT networks exchange unreduced 29-limb planes between passes (EON_NTT_MID=1:
# no reduce / pack / unpack at the pass boundaries) -- DFT / golden / prove tests, then the
# same-call A/B against the packed exchange (variants/libeonhip_mid0.so) on lde and prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dft_small.py tests/test_gpu_dft_large.py tests/test_golden.py tests/test_gpu_fft_bench_shape.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s32.txt 2>&1 || { tail -30 $O/pytest_s32.txt; exit 1; }
tail -1 $O/pytest_s32.txt
PROBE_WORKLOADS="lde prove" timeout -k 10 1000 bash tools/gpu_probe.sh mid0 || exit 1
for f in default mid0 default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 1) for n, v in k.items() if 'ntt' in n})"
done
