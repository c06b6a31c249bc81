#!/bin/bash
# PMC passes (counters only with kernel-trace; one counter group per pass) for both workloads.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W_LDE=$(python3 -c "print('configs[1]: batched LDE NTT, coset_lde_batch 2^20 rows x 64 cols over BN254 Fr, added_bits=1, shift=5, natural output (per GPU; column-sharded)')")
W_MSM=$(python3 -c "print('configs[2]: KZG commit MSM, 2^20 BN254 G1 SRS points (alpha=12345, fixed-base window table built untimed) x uniform Fr scalars (per GPU)')")
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_lde_fetch -o f --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc1.err \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_lde_write -o w --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc2.err \
 && python3 tools/pmc_traffic.py gpurun_out/pmc_lde_fetch gpurun_out/pmc_lde_write "k_ntt_pass<false, 3>" "$W_LDE" gpurun_out/traffic_lde.json \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_msm_fetch -o f --output-format csv -- python3 bench.py --workload msm --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc3.err \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_msm_write -o w --output-format csv -- python3 bench.py --workload msm --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc4.err \
 && python3 tools/pmc_traffic.py gpurun_out/pmc_msm_fetch gpurun_out/pmc_msm_write "k_piece_sum" "$W_MSM" gpurun_out/traffic_msm.json
rc=$?; tail -3 gpurun_out/pmc*.err; exit $rc
