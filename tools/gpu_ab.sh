#!/bin/bash
# One GPU session: parity tests on the in-tree library, then a same-call A/B of the in-tree library
# against tuning builds (variants/libeonhip_<name>.so, `python -m plonky3_eon_amd._build variant
# <name> DEFINES...` + copy to variants/), through tools/gpu_probe.sh.
#   TESTS      test files for the in-tree library (default: the MSM / KZG-open / prove / golden files)
#   VTESTS     test files run against each variant before its timing (default: none)
#   PROBE_WORKLOADS, PROBE_ARGS   as in tools/gpu_probe.sh
# usage: tools/gpu_ab.sh <variant>...      (no variant: tests only)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${TESTS:-tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py tests/test_golden.py}
timeout -k 10 900 python -u -m pytest $T -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_ab.txt 2>&1 \
  || { tail -30 $O/pytest_ab.txt; exit 1; }
tail -1 $O/pytest_ab.txt
if [ -n "$VTESTS" ]; then
  cp plonky3_eon_amd/libeonhip.so $O/.keep_default.so
  for V in "$@"; do
    cp variants/libeonhip_$V.so plonky3_eon_amd/libeonhip.so
    timeout -k 10 900 python -u -m pytest $VTESTS -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_ab_$V.txt 2>&1 \
      || { tail -30 $O/pytest_ab_$V.txt; cp $O/.keep_default.so plonky3_eon_amd/libeonhip.so; exit 1; }
    echo "$V: $(tail -1 $O/pytest_ab_$V.txt)"
  done
  cp $O/.keep_default.so plonky3_eon_amd/libeonhip.so && rm -f $O/.keep_default.so
fi
[ $# -ge 1 ] || exit 0
timeout -k 10 1500 bash tools/gpu_probe.sh "$@" || exit 1
for f in default "$@" default2; do
  [ -f $O/probe_prove_$f.json ] || continue
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], 'clk', d.get('gpu_clock_inkernel_mhz'), {n: round(v['total_ms'], 1) for n, v in k.items() if 'piece' in n or 'ntt' in n or 'bucket' in n or 'sort' in n})"
done
