set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r47
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r47/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/r47/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/r47/pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r47/smoke.log 2>&1 || { tail -30 gpurun_out/r47/smoke.log; exit 1; }
tail -1 gpurun_out/r47/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r47/bench.log 2>&1 || { tail -30 gpurun_out/r47/bench.log; exit 1; }
tail -2 gpurun_out/r47/bench.log
