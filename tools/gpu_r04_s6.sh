#!/bin/bash
# Round-4 session 6: transcript absorb microbench on the box's host, MSM tests after the
# grid-stride digit kernel, headline prove, kernel trace of the emulated 8-rank prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for i in 1 2 3; do timeout -k 10 60 tools/ubench_transcript; done | tee $O/ubench_transcript.json &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_prove_full.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_msm.txt 2>&1 || { tail -30 $O/pytest_msm.txt; exit 1; }
tail -1 $O/pytest_msm.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_prove.json 2> $O/bench_prove.err &&
  python3 -c "
import json; d=json.load(open('$O/bench_prove.json')); print('prove', d['value'], d['throughput']['stage_ms'])
ks=d['roofline']['kernels']; print({k: round(v['total_ms'], 2) for k, v in ks.items()})" &&
rm -rf $O/trace8 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace8 -o t -- python3 bench.py --steps 1 \
  --warmup 1 --no-cpu-baseline --emulate-world 8 > $O/trace8_bench.json 2> $O/trace8.err || { tail -20 $O/trace8.err; exit 1; }
f=$(find $O/trace8 -name '*kernel_trace.csv' | head -1)
python3 tools/phases.py $f 0.3 > $O/phases8.txt && tail -45 $O/phases8.txt
