set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r48
export TMPDIR=/tmp
timeout -k 10 300 python bench/kernel_sol.py --out gpurun_out/r48/kernel_sol.json > gpurun_out/r48/kernel_sol.log 2>&1 || { tail -30 gpurun_out/r48/kernel_sol.log; exit 1; }
cat gpurun_out/r48/kernel_sol.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r48/prof -o run -- python3 bench/kernel_sol.py --sizes 1048576,16777216 --iters 5 > gpurun_out/r48/prof.log 2>&1 || { tail -30 gpurun_out/r48/prof.log; exit 1; }
find gpurun_out/r48/prof -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-200
