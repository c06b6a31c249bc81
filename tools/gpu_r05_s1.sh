#!/bin/bash
# Round 5, session 1: the new GPU tests (clock probe, trim, worst-case quotient inputs, pairing
# after the PoolScope change), a short default bench line with the in-kernel clock, and the PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE, FLAT/scratch instructions) of k_piece_sum29 in the
# serialized prove -> gpurun_out/traffic_prove.json (EON_COMMIT names the measured build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_diag.py tests/test_gpu_quotient.py tests/test_gpu_air_program.py \
  tests/test_gpu_pairing.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_s1.txt 2>&1 \
  || { tail -30 $O/pytest_s1.txt; exit 1; }
tail -2 $O/pytest_s1.txt
timeout -k 10 600 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_prove.json 2> $O/bench_prove.err \
  || { tail -20 $O/bench_prove.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_prove.json')); r=d['roofline']
print('prove', d['value'], 'sclk', d['gpu_sclk'].get('median_mhz'), 'inkernel', d['gpu_clock_inkernel_mhz'], d['gpu_clock_probe'])
print('valu', r['valu'])"
B="python3 bench.py --serial --steps 1 --warmup 0 --no-cpu-baseline --no-clock-probe"
R="--kernel-include-regex k_piece_sum29"
pass() {  # name counters...
  local n=$1; shift
  rm -rf $O/pmc_$n
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace $R -d $O/pmc_$n -o p --output-format csv -- $B \
    > $O/pmc_$n.log 2>&1 || { tail -5 $O/pmc_$n.log; return 1; }
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && pass flat SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES \
  && python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write k_piece_sum $O/bench_prove.json $O/traffic_prove.json \
  && python3 tools/pmc_table.py k_piece_sum29 $O/pmc_flat.json $O/pmc_flat
