#!/bin/bash
# Round 5, session 5: (1) digit-sort pass variants (tools/gpu_r05_s4.sh); (2) k_bucket_reduce29
# with its segments handed out in piece-count order per 256-thread block (EON_BR_BALANCE) --
# MSM / open / prove tests, then the same-call A/B against the unbalanced 64-thread form
# (variants/libeonhip_brold.so) on the prove, with the bucket reductions' profiled time.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu_r05_s4.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_batches.py tests/test_gpu_kzg_open.py tests/test_gpu_prove.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s5.txt 2>&1 || { tail -30 $O/pytest_s5.txt; exit 1; }
tail -1 $O/pytest_s5.txt
PROBE_WORKLOADS=prove timeout -k 10 1000 bash tools/gpu_probe.sh brold || exit 1
for f in default brold default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_prove_$f.json')); k=d['roofline']['kernels']
print('$f', d['value'], {n: round(v['total_ms'], 2) for n, v in k.items() if 'bucket' in n or 'finish' in n})"
done
# (3) the single MSM's bucket sums + radix-2^29 segment sums (EON_MSM_SUMS29) against the combine
# path (variants/libeonhip_sumsold.so), configs[2]
cp $O/probe_summary.txt $O/probe_summary_br.txt
PROBE_WORKLOADS=msm timeout -k 10 600 bash tools/gpu_probe.sh sumsold c16 || exit 1
for f in default sumsold c16 default2; do
  python3 -c "
import json; d=json.load(open('$O/probe_msm_$f.json')); k=d['roofline']['kernels']
print('msm $f', d['value'], {n: round(v['total_ms'] / v['launches'], 3) for n, v in k.items()})"
done
# (4) NTT passes with the stage count a template constant (EON_NTT_FIXED_K) against the runtime
# form (variants/libeonhip_nttk0.so): DFT tests at the forced small-pass plans, then the LDE A/B
cp $O/probe_summary.txt $O/probe_summary_sums.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_dft_small.py tests/test_gpu_dft_large.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_s5_dft.txt 2>&1 || { tail -30 $O/pytest_s5_dft.txt; exit 1; }
tail -1 $O/pytest_s5_dft.txt
PROBE_WORKLOADS=lde timeout -k 10 600 bash tools/gpu_probe.sh nttk0 ntttwg || exit 1
# (5) research A/B: batch-affine additions with one inversion shared by the W waves of a block
timeout -k 10 300 tools/ubench_batch_affine > $O/ubench_batch_affine.txt 2>&1 || { tail -5 $O/ubench_batch_affine.txt; exit 1; }
cat $O/ubench_batch_affine.txt
