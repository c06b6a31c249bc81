#!/bin/bash
# Validation + measurement of the committed build on one MI355X (EON_COMMIT names it): sort_check,
# the whole GPU suite (slow tests included), smoke, the default bench line (CPU baselines, in-kernel
# clock), the serialized rocprofv3 kernel summary of the same workload, the PMC traffic passes of
# k_piece_sum29 (raw FETCH_SIZE + WRITE_SIZE, tools/pmc_traffic.py), the emulated 8-rank prove and
# every other workload's bench line (tools/gpu_bench_all.sh).  Everything lands in gpurun_out/.
#   SKIP_TESTS=1 skips sort_check / pytest / smoke (a re-measurement of an already validated build)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export EON_TEST_HEARTBEAT=$PWD/gpurun_out/heartbeat.txt
O=gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 120 tools/sort_check > $O/sort_check.txt 2>&1 && ! grep -q '"ok":0' $O/sort_check.txt \
    || { tail -5 $O/sort_check.txt; exit 1; }
  timeout -k 10 1500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
    || { tail -30 $O/pytest_gpu.txt; exit 1; }
  tail -1 $O/pytest_gpu.txt
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 \
    || { tail -20 $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
timeout -k 10 600 python3 bench.py > $O/bench_prove.json 2> $O/bench_prove.err || { tail -20 $O/bench_prove.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_prove.json')); r=d['roofline']; v=r['valu']
print('prove', d['value'], 'sclk', (d['gpu_sclk'] or {}).get('median_mhz'), 'inkernel', d['gpu_clock_inkernel_mhz'],
      'valu', v['frac'], v.get('frac_live'), 'issue_floor', v.get('issue_floor', {}).get('frac'), 'hbm', r['frac'])"
rm -rf $O/stats_prove
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_prove -o s -- \
  python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline --no-clock-probe > $O/stats_prove.json 2> $O/stats_prove.err \
  || { tail -20 $O/stats_prove.err; exit 1; }
B="python3 bench.py --serial --steps 1 --warmup 0 --no-cpu-baseline --no-clock-probe"
R="--kernel-include-regex k_piece_sum29"
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/pmc_$c
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace $R -d $O/pmc_$c -o p --output-format csv -- $B > $O/pmc_$c.log 2>&1 \
    || { tail -5 $O/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE k_piece_sum $O/bench_prove.json $O/traffic_prove.json || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --emulate-world 8 --steps 5 > $O/bench_emul8.json 2> $O/bench_emul8.err &&
  python3 -c "import json; d=json.load(open('$O/bench_emul8.json')); print('emul8', d['value'], d['throughput']['stage_ms'])" || exit 1
[ -n "$NO_BENCH_ALL" ] && exit 0  # the other workloads in a call of their own (gpurun caps a call at 20 min)
timeout -k 10 1200 bash tools/gpu_bench_all.sh
