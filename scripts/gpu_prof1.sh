set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench/engine_sweep.py --rounds 3 --batches 512 > gpurun_out/sweep1.log 2>&1 || exit $?
cat gpurun_out/sweep1.log | grep tx_per
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python bench.py --steps 20 --warmup 3 --no-unloaded-probe > gpurun_out/prof1.log 2>&1 || exit $?
ls -R gpurun_out/prof1 | head -20
