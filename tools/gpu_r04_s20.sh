#!/bin/bash
# Round-4 session 20: issue/stall PMC of the digit sort pass and the bucket reduction on the prove
# (tools/gpu_pmc_kernel.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 bash tools/gpu_pmc_kernel.sh prove k_sort_pass sortpass &&
timeout -k 10 500 bash tools/gpu_pmc_kernel.sh prove k_bucket_reduce29 bucketred
