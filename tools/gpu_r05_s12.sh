#!/bin/bash
# Round 5, session 12: radix-2^29 products with each column's multiply-adds in one asm statement
# (field29.h madcol, EON_MAD_BLOCKS=1) -- the whole GPU suite, then the same-call A/B against one
# asm statement per multiply-add (variants/libeonhip_mb0.so) on msm, prove, lde and quotient.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 tools/sort_check > $O/sort_check12.txt 2>&1 && ! grep -q '"ok":0' $O/sort_check12.txt || { tail -5 $O/sort_check12.txt; exit 1; }
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_s12.txt 2>&1 \
  || { tail -30 $O/pytest_s12.txt; exit 1; }
tail -1 $O/pytest_s12.txt
PROBE_WORKLOADS="msm prove lde quotient" timeout -k 10 1000 bash tools/gpu_probe.sh mb0 || exit 1
