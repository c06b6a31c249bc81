#!/bin/bash
# Round-4 session 7 (HEAD after the scratch-free team pairings and the one-body generic quotient):
# transcript microbench on the box's host, pairing / AIR-program / MSM tests, smoke, verify bench,
# generic-quotient A/B against the old four-slot body (variants/libeonhip_airold.so), headline
# prove, emulated 8-rank prove, kernel traces of both (phases / exposure).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for i in 1 2 3; do timeout -k 10 60 tools/ubench_transcript; done | tee $O/ubench_transcript.json &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_air_program.py tests/test_gpu_msm.py tests/test_gpu_msm_batches.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_msm_air.txt 2>&1 || { tail -30 $O/pytest_msm_air.txt; exit 1; }
tail -1 $O/pytest_msm_air.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
qgen() {  # name [EON_LIB]
  EON_LIB=$2 timeout -k 10 300 python3 bench.py --workload quotient --air generic --no-cpu-baseline \
    > $O/bench_qgen_$1.json 2> $O/bench_qgen_$1.err || { tail -20 $O/bench_qgen_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/bench_qgen_$1.json')); print('qgen $1', d['value'], d['roofline']['valu']['frac'])"
}
timeout -k 10 300 python3 bench.py --workload verify --no-cpu-baseline > $O/bench_verify.json 2> $O/bench_verify.err &&
  python3 -c "import json; d=json.load(open('$O/bench_verify.json')); print('verify', d['value'], {k: v['total_ms'] for k, v in d['roofline']['kernels'].items()})" &&
qgen new && qgen old $PWD/variants/libeonhip_airold.so && qgen new2 && qgen old2 $PWD/variants/libeonhip_airold.so &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_prove.json 2> $O/bench_prove.err &&
  python3 -c "
import json; d=json.load(open('$O/bench_prove.json')); print('prove', d['value'], d['throughput']['stage_ms'], d.get('gpu_sclk'))" &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --emulate-world 8 --steps 5 > $O/bench_emul8.json 2> $O/bench_emul8.err &&
  python3 -c "import json; d=json.load(open('$O/bench_emul8.json')); print('emul8', d['value'], d['throughput']['stage_ms'])" &&
rm -rf $O/trace8 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace8 -o t -- python3 bench.py --steps 1 \
  --warmup 1 --no-cpu-baseline --emulate-world 8 > $O/trace8_bench.json 2> $O/trace8.err || { tail -20 $O/trace8.err; exit 1; }
f=$(find $O/trace8 -name '*kernel_trace.csv' | head -1)
python3 tools/phases.py $f 0.3 > $O/phases8.txt && tail -12 $O/phases8.txt &&
rm -rf $O/trace &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o prove -- python3 bench.py --steps 1 \
  --warmup 1 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 tools/exposure.py $f > $O/prove_exposure.txt && cat $O/prove_exposure.txt
