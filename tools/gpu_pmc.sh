#!/bin/bash
# PMC passes (counters only, with kernel-trace; FETCH_SIZE and WRITE_SIZE in separate passes) for
# the dominant kernel of each bench workload -> profiles/traffic_<workload>.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
pmc() {  # workload kernel steps
  local w=$1 k=$2 st=$3
  timeout -k 10 300 python3 bench.py --workload $w --steps $st --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$w.json 2> gpurun_out/pmc_$w.err \
  && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_${w}_fetch -o f --output-format csv -- python3 bench.py --workload $w --steps $st --warmup 1 --no-cpu-baseline > /dev/null 2>> gpurun_out/pmc_$w.err \
  && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_${w}_write -o w --output-format csv -- python3 bench.py --workload $w --steps $st --warmup 1 --no-cpu-baseline > /dev/null 2>> gpurun_out/pmc_$w.err \
  && python3 tools/pmc_traffic.py gpurun_out/pmc_${w}_fetch gpurun_out/pmc_${w}_write "$k" gpurun_out/pmc_$w.json gpurun_out/traffic_$w.json
}
pmc prove k_piece_sum 1 && pmc lde "k_ntt_pass29<false, 3>" 2 && pmc msm k_piece_sum 2
rc=$?; tail -2 gpurun_out/pmc_*.err; exit $rc
