#!/bin/bash
# Round-4 final validation of the committed build: the whole GPU suite and smoke, the default bench
# line (CPU baselines included), the serialized rocprofv3 kernel summary, the emulated 8-rank prove
# and the generic / fused quotient benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
  || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python3 bench.py > $O/bench_prove.json 2> $O/bench_prove.err || { tail -20 $O/bench_prove.err; exit 1; }
cut -c1-300 $O/bench_prove.json
rm -rf $O/stats_prove
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_prove -o s -- \
  python3 bench.py --serial --steps 2 --warmup 1 --no-cpu-baseline > $O/stats_prove.json 2> $O/stats_prove.err \
  || { tail -20 $O/stats_prove.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --emulate-world 8 --steps 5 > $O/bench_emul8.json 2> $O/bench_emul8.err &&
  python3 -c "import json; d=json.load(open('$O/bench_emul8.json')); print('emul8', d['value'], d['throughput']['stage_ms'])" &&
for a in generic fused; do
  timeout -k 10 300 python3 bench.py --workload quotient --air $a --no-cpu-baseline > $O/bench_q_$a.json 2> $O/bench_q_$a.err &&
  python3 -c "import json; d=json.load(open('$O/bench_q_$a.json')); print('quotient $a', d['value'])" || exit 1
done
