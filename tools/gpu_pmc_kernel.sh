#!/bin/bash
# Issue/LDS/VALU PMC passes (each alone, kernel-trace only, within the gfx950 slot limits) for one
# kernel of one bench.py workload (serialized) -> gpurun_out/pmc_<name>.json via tools/pmc_table.py.
# usage: [BENCH_EXTRA="--air generic"] tools/gpu_pmc_kernel.sh <workload> <kernel-regex> <name>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W=${1:?workload}; K=${2:?kernel regex}; N=${3:?name}
B="python3 bench.py --workload $W --serial --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_EXTRA}"
pass() {  # pass-name counters...
  local n=$1; shift
  rm -rf gpurun_out/pmc_${N}_$n
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "$K" -d gpurun_out/pmc_${N}_$n -o p \
    --output-format csv -- $B > gpurun_out/pmc_${N}_$n.log 2>&1 || { tail -5 gpurun_out/pmc_${N}_$n.log; return 1; }
}
pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
 && pass b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_THREAD_CYCLES_VALU \
  SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
 && python3 tools/pmc_table.py "$K" gpurun_out/pmc_$N.json gpurun_out/pmc_${N}_a gpurun_out/pmc_${N}_b > /dev/null \
 && python3 - gpurun_out/pmc_$N.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t = d["per_dispatch_mean"]
cu = 256
g = t.get("GRBM_GUI_ACTIVE") or 1
out = {"VALUBusy %": 100 * t["SQ_ACTIVE_INST_VALU"] / cu / g,
       "LDS active % (IDX_ACTIVE / CU / cycles)": 100 * t.get("SQ_LDS_IDX_ACTIVE", 0) / cu / g,
       "LDS bank conflict / IDX_ACTIVE": t.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, t.get("SQ_LDS_IDX_ACTIVE", 1)),
       "VALU insts per LDS inst": t["SQ_INSTS_VALU"] / max(1, t.get("SQ_INSTS_LDS", 1)),
       "wait_inst_lds / wave_cycles": t.get("SQ_WAIT_INST_LDS", 0) / t["SQ_WAVE_CYCLES"],
       "wait_any / wave_cycles": t["SQ_WAIT_ANY"] / t["SQ_WAVE_CYCLES"],
       "wait_inst_any / wave_cycles": t["SQ_WAIT_INST_ANY"] / t["SQ_WAVE_CYCLES"],
       "active_any / wave_cycles": t["SQ_ACTIVE_INST_ANY"] / t["SQ_WAVE_CYCLES"],
       "mean waves resident per SIMD": t["SQ_WAVE_CYCLES"] / (cu * 4) / (g / 4)}
d["derived"].update({k: round(v, 4) for k, v in out.items()})
json.dump(d, open(sys.argv[1], "w"), indent=1)
print(json.dumps(d["derived"], indent=1))
PY
