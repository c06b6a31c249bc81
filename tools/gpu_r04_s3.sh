#!/bin/bash
# Round-4 session 3: host permutation A/B (old / new build of the transcript), the generic
# quotient with prefetched operands, and a kernel trace of the emulated 8-rank prove.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for i in 1 2; do tools/perm_bench_old; tools/perm_bench_new; done | tee $O/perm_ab.txt &&
timeout -k 10 60 tools/ubench_transcript | tee $O/ubench_transcript.json &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_air_program.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_air.txt 2>&1 || { tail -30 $O/pytest_air.txt; exit 1; }
tail -1 $O/pytest_air.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload quotient --air generic --no-cpu-baseline \
    > $O/bench_qgen_$i.json 2> $O/bench_qgen_$i.err || { tail -20 $O/bench_qgen_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_qgen_$i.json')); print('generic', d['value'], d['roofline'].get('valu'))"
done
rm -rf $O/trace8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace8 -o t -- python3 bench.py --steps 1 \
  --warmup 1 --no-cpu-baseline --emulate-world 8 > $O/trace8_bench.json 2> $O/trace8.err || { tail -20 $O/trace8.err; exit 1; }
f=$(find $O/trace8 -name '*kernel_trace.csv' | head -1)
python3 tools/phases.py $f 0.3 > $O/phases8.txt && tail -40 $O/phases8.txt
