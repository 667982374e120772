set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu2.log 2>&1 || { tail -30 gpurun_out/pytest_gpu2.log; exit 1; }
tail -3 gpurun_out/pytest_gpu2.log
timeout -k 10 300 python bench/roofline.py > gpurun_out/roofline.json 2>&1 || exit $?
cat gpurun_out/roofline.json
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log
timeout -k 10 300 python bench.py --model gbdt --batch 65536 --batches-per-step 16 --no-unloaded-probe > gpurun_out/bench_gbdt.log 2>&1 || exit $?
tail -1 gpurun_out/bench_gbdt.log
timeout -k 10 300 python bench.py --model lr --no-unloaded-probe > gpurun_out/bench_lr.log 2>&1 || exit $?
tail -1 gpurun_out/bench_lr.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python bench.py --steps 20 --warmup 3 --no-unloaded-probe > gpurun_out/prof2.log 2>&1 || exit $?
cat gpurun_out/prof2/run_kernel_stats.csv | head -5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2dma -o run -- python bench.py --steps 20 --warmup 3 --no-unloaded-probe --input-mode dma > gpurun_out/prof2dma.log 2>&1 || exit $?
cat gpurun_out/prof2dma/run_kernel_stats.csv | head -5
