set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 bash tools/gpu_pmc_kernel.sh prove k_sort_pass sortp > gpurun_out/pmc_sortp_out.txt 2>&1 || exit 1
B="python3 bench.py --serial --steps 1 --warmup 0 --no-cpu-baseline --no-clock-probe"
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmcs_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex k_sort_pass -d gpurun_out/pmcs_$c -o p --output-format csv -- $B > gpurun_out/pmcs_$c.log 2>&1 || { tail -5 gpurun_out/pmcs_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py gpurun_out/pmcs_FETCH_SIZE gpurun_out/pmcs_WRITE_SIZE k_sort_pass prove gpurun_out/traffic_sort.json
cat gpurun_out/pmc_sortp_out.txt gpurun_out/traffic_sort.json
