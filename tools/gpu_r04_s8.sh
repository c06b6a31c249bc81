#!/bin/bash
# Round-4 session 8: issue/stall PMC of the generic quotient interpreter (old four-slot body) and
# of the fused Poseidon2 quotient kernel, same counters (tools/gpu_pmc_kernel.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
EON_LIB=$PWD/variants/libeonhip_airold.so BENCH_EXTRA="--air generic" timeout -k 10 400 bash tools/gpu_pmc_kernel.sh quotient k_air_quotient qgen_old &&
timeout -k 10 400 bash tools/gpu_pmc_kernel.sh quotient k_p2_quotient qfused
