#!/bin/bash
# Every bench.py workload line of DESIGN.md section 0 on one MI355X -> gpurun_out/bench_<name>.json
set -o pipefail
mkdir -p gpurun_out
run() {  # name args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err \
    || { tail -5 gpurun_out/bench_$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline'].get('valu', {}).get('frac'), d['roofline'].get('frac'))" \
    gpurun_out/bench_$n.json $n
}
run lde --workload lde && run lde_bitrev --workload lde --order bitrev && run msm --workload msm \
  && run msm_small --workload msm --msm-scalars small && run ntt4 --workload ntt4 \
  && run msm_shard --workload msm-shard && run quotient_fused --workload quotient \
  && run quotient_generic --workload quotient --air generic && run verify --workload verify
