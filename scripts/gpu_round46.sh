set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r46
timeout -k 10 300 python -m pytest tests/test_rccl_gpu.py -x -q > gpurun_out/r46/pytest_rccl.log 2>&1 || { tail -40 gpurun_out/r46/pytest_rccl.log; exit 1; }
tail -1 gpurun_out/r46/pytest_rccl.log
