set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r45


timeout -k 10 600 python bench/train_bench.py --out gpurun_out/r45/train_bench.json > gpurun_out/r45/train_bench.log 2>&1 || { tail -30 gpurun_out/r45/train_bench.log; exit 1; }
cat gpurun_out/r45/train_bench.json
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r45/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/r45/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/r45/pytest_gpu_all.log
