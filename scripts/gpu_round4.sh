set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu4.log 2>&1 || { tail -30 gpurun_out/pytest_gpu4.log; exit 1; }
tail -2 gpurun_out/pytest_gpu4.log
timeout -k 10 120 python bench/roofline.py > gpurun_out/r4_roofline.json 2>&1 || exit $?
cat gpurun_out/r4_roofline.json
timeout -k 10 600 python bench/engine_sweep.py --rounds 2 --batches 1024 --modes zerocopy:zerocopy,dma:zerocopy --depths 4,8 --streams 1,2,4,8 > gpurun_out/r4_sweep.log 2>&1 || exit $?
grep tx_per gpurun_out/r4_sweep.log
