#!/bin/bash
# Round-4 session 12: issue PMC of the radix-2^29 generic interpreter and the radix-2^29 fused
# quotient (tools/gpu_pmc_kernel.sh; compare profiles/r04/s8 for the radix-2^32 kernels).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_EXTRA="--air generic" timeout -k 10 400 bash tools/gpu_pmc_kernel.sh quotient k_air_quotient qgen29 &&
timeout -k 10 400 bash tools/gpu_pmc_kernel.sh quotient k_p2_quotient qfused29
