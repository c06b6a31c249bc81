#!/bin/bash
# Full GPU session: smoke, parity tests, the three bench workloads, rocprof summaries.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 \
  && cat gpurun_out/smoke.txt \
  && timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.txt 2>&1 \
  && tail -2 gpurun_out/pytest_gpu.txt \
  && timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
  && timeout -k 10 400 python bench.py --workload lde > gpurun_out/bench_lde.json 2> gpurun_out/bench_lde.err \
  && timeout -k 10 400 python bench.py --workload msm > gpurun_out/bench_msm.json 2> gpurun_out/bench_msm.err \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_prove -o prove --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prove_prof.json 2> gpurun_out/prof_prove.err \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o lde --output-format csv -- python3 bench.py --workload lde $B > gpurun_out/bench_prof.json 2> gpurun_out/prof.err \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_msm -o msm --output-format csv -- python3 bench.py --workload msm $B > gpurun_out/bench_msm_prof.json 2> gpurun_out/prof_msm.err
rc=$?
tail -3 gpurun_out/pytest_gpu.txt
for f in bench.json bench_lde.json bench_msm.json; do python3 -c "
import json,sys; d=json.load(open('gpurun_out/$f')); r=d['roofline']
print('$f', d['ms_per_step'], 'ms |', r['kernel'], r['avg_launch_ms'], 'ms/launch |', r.get('valu',{}).get('frac'), '| cpu', (d['cpu_baseline'] or {}).get('value'))" 2>/dev/null; done
exit $rc
