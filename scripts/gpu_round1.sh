set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "start $(date)"; rocm-smi --showproductname 2>&1 | head -20 > gpurun_out/smi.txt
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench_dma.log 2>&1 || exit $?
tail -2 gpurun_out/bench_dma.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --input-mode zerocopy --no-unloaded-probe > gpurun_out/bench_zc.log 2>&1 || exit $?
tail -2 gpurun_out/bench_zc.log
echo "done $(date)"
