set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.txt 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 \
 && tail -2 gpurun_out/pytest_gpu.txt \
 && timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err \
 && cat gpurun_out/bench.json
rc=$?
tail -3 gpurun_out/smoke.txt gpurun_out/pytest_gpu.txt
exit $rc
