#!/bin/bash
# Instruction-cache and scalar-cache PMC passes (SQ block, kernel-trace only) for one kernel of one
# bench.py workload -> gpurun_out/icache_<name>_{i,s}/ (counter CSVs) and a one-line summary.
# usage: [BENCH_EXTRA="--air generic"] tools/gpu_icache.sh <workload> <kernel-regex> <name>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W=${1:?workload}; K=${2:?kernel regex}; N=${3:?name}
B="python3 bench.py --workload $W --serial --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_EXTRA}"
pass() {  # pass-name counters...
  local n=$1; shift
  rm -rf gpurun_out/icache_${N}_$n
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "$K" -d gpurun_out/icache_${N}_$n -o p \
    --output-format csv -- $B > gpurun_out/icache_${N}_$n.log 2>&1 || { tail -5 gpurun_out/icache_${N}_$n.log; return 1; }
}
pass i SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES \
  SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
 && pass s SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQ_INST_LEVEL_SMEM \
  SQ_INSTS_SMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
 && python3 - "$K" gpurun_out/icache_${N}_i gpurun_out/icache_${N}_s <<'PY'
import csv, collections, re, sys
k = re.compile(sys.argv[1])
tot = collections.defaultdict(float)
for d in sys.argv[2:]:
    for r in csv.DictReader(open(d + "/p_counter_collection.csv")):
        if k.search(r["Kernel_Name"]):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
t = dict(tot)
out = {c: t[c] for c in sorted(t)}
if t.get("SQC_ICACHE_REQ"):
    out["icache_hit_rate"] = t["SQC_ICACHE_HITS"] / t["SQC_ICACHE_REQ"]
if t.get("SQC_DCACHE_REQ"):
    out["dcache_hit_rate"] = t["SQC_DCACHE_HITS"] / t["SQC_DCACHE_REQ"]
print(sys.argv[1], out)
PY
