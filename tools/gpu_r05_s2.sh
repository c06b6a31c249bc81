#!/bin/bash
# Round 5, session 2: kernel-trace summaries of the single MSM (configs[2]), the LDE (configs[1])
# and the 2^24 sharded MSM in serial mode, for the tail / NTT work.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for w in msm lde msm-shard; do
  rm -rf $O/stats_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$w -o s -- \
    python3 bench.py --workload $w --serial --steps 3 --warmup 1 --no-cpu-baseline --no-clock-probe \
    > $O/stats_$w.json 2> $O/stats_$w.err || { tail -20 $O/stats_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/stats_$w.json')); print('$w', d['value'])"
done
