#!/bin/bash
# PMC passes (each alone, kernel-trace only, counters per pass within the gfx950 slot limits) for
# k_piece_sum29 in the serialized configs[3] prove -> profiles/r02/pmc_piece_sum29.json via
# tools/pmc_table.py.  Stall breakdown (SQ), L2 hit rate and TA/TCP stalls, HBM bytes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --serial --steps 1 --warmup 0 --no-cpu-baseline"
R="--kernel-include-regex k_piece_sum29"
pass() {  # name counters...
  local n=$1; shift
  rm -rf gpurun_out/pmc_$n
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace $R -d gpurun_out/pmc_$n -o p --output-format csv -- $B \
    > gpurun_out/pmc_$n.log 2>&1 || { tail -5 gpurun_out/pmc_$n.log; return 1; }
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM \
 && pass sq2 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_LEVEL_WAVES TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum \
 && pass mem TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_BUSY_max \
 && pass fetch FETCH_SIZE \
 && pass write WRITE_SIZE \
 && python3 tools/pmc_table.py k_piece_sum29 gpurun_out/pmc_piece_sum29.json gpurun_out/pmc_sq gpurun_out/pmc_sq2 gpurun_out/pmc_mem gpurun_out/pmc_fetch gpurun_out/pmc_write
