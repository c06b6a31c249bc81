#!/bin/bash
# Round 5, session 28: rehearsal of the N > 1 bench path on one GPU (two ranks sharing the device,
# gloo process group, torch collective): the lane-sharded prove end to end with this build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
EON_BENCH_BACKEND=gloo EON_BENCH_ONE_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-clock-probe > $O/bench_n2_rehearsal.json 2> $O/bench_n2_rehearsal.err || { tail -20 $O/bench_n2_rehearsal.err; exit 1; }
cat $O/bench_n2_rehearsal.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['scaling'], d['config'])"
