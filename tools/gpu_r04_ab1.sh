#!/bin/bash
# Round-4 A/B session 1: generic quotient interpreter (VGPR register file + forwarding vs LDS),
# cooperative table gathers in k_piece_sum29 (variants/libeonhip_coop.so) with MSM parity under
# the variant, then the msm / prove A/B (tools/gpu_probe.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_air_program.py tests/test_gpu_quotient.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_air.txt 2>&1 || { tail -30 $O/pytest_air.txt; exit 1; }
tail -1 $O/pytest_air.txt
EON_LIB=$PWD/variants/libeonhip_coop.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py \
  tests/test_gpu_msm_batches.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_msm_coop.txt 2>&1 \
  || { tail -30 $O/pytest_msm_coop.txt; exit 1; }
tail -1 $O/pytest_msm_coop.txt
for m in vgpr lds vgpr lds; do
  EON_AIR_REGS=$m timeout -k 10 300 python3 bench.py --workload quotient --air generic --no-cpu-baseline \
    > $O/bench_qgen_$m.json 2> $O/bench_qgen_$m.err || { tail -20 $O/bench_qgen_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_qgen_$m.json')); print('generic', '$m', d['value'], d['roofline'].get('valu'))"
done
timeout -k 10 300 python3 bench.py --workload quotient --air fused --no-cpu-baseline > $O/bench_qfused.json \
  2> $O/bench_qfused.err && python3 -c "import json; d=json.load(open('$O/bench_qfused.json')); print('fused', d['value'])" &&
PROBE_WORKLOADS="msm prove" timeout -k 10 900 tools/gpu_probe.sh coop
