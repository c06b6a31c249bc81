#!/bin/bash
# bench.py --workload W under several tuning knobs (each argument: space-separated env assignments,
# "-" for the defaults); one summary line per setting in gpurun_out/knobs_W.txt
# usage: tools/knob_bench.sh <workload> <setting>...
set -o pipefail
mkdir -p gpurun_out
W=${1:?workload}
shift
OUT=gpurun_out/knobs_$W.txt
: > $OUT
for kv in "$@"; do
  [ "$kv" = - ] && kv=""
  env $kv timeout -k 10 200 python3 bench.py --workload $W --no-cpu-baseline --steps 5 --warmup 2 \
    > gpurun_out/knob.json 2> gpurun_out/knob.err || { tail -5 gpurun_out/knob.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/knob.json')); print(sys.argv[1], d['ms_per_step'], d['roofline'].get('achieved'), d['roofline'].get('valu', {}).get('frac') if isinstance(d['roofline'].get('valu'), dict) else d['roofline'].get('valu'))" "[$kv]" >> $OUT
done
cat $OUT
