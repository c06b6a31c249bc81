#!/bin/bash
# Round-4 session 5: team-parallel pairing tests first (new kernels, short limit), then the full
# GPU suite, sort/scan check, headline bench, emulated 8-rank prove, generic quotient, verify.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_pairing.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_pairing.txt 2>&1 || { tail -30 $O/pytest_pairing.txt; exit 1; }
tail -1 $O/pytest_pairing.txt
timeout -k 10 120 tools/sort_check > $O/sort_check.txt 2>&1 && grep -c '"ok":1' $O/sort_check.txt && ! grep -q '"ok":0' $O/sort_check.txt &&
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python3 bench.py --workload verify --no-cpu-baseline > $O/bench_verify.json 2> $O/bench_verify.err &&
  python3 -c "import json; d=json.load(open('$O/bench_verify.json')); print('verify', d['value'], {k: v['total_ms'] for k, v in d['roofline']['kernels'].items()})" &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_prove.json 2> $O/bench_prove.err &&
  python3 -c "import json; d=json.load(open('$O/bench_prove.json')); print('prove', d['value'], d['throughput']['stage_ms'], d.get('gpu_sclk'))" &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --emulate-world 8 --steps 5 > $O/bench_emul8.json 2> $O/bench_emul8.err &&
  python3 -c "import json; d=json.load(open('$O/bench_emul8.json')); print('emul8', d['value'], d['throughput']['stage_ms'])" &&
timeout -k 10 300 python3 bench.py --workload quotient --air generic --no-cpu-baseline > $O/bench_qgen.json 2> $O/bench_qgen.err &&
  python3 -c "import json; d=json.load(open('$O/bench_qgen.json')); print('qgen', d['value'], d['roofline']['valu']['frac'])"
