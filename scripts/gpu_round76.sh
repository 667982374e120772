set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/r76; mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-unloaded-probe > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
grep '"metric"' $O/prof_bench.log | cut -c1-200
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sol -o run -- python3 $R/bench/kernel_sol.py --sizes 16777216 --iters 5 > $O/prof_sol.log 2>&1 || { tail -20 $O/prof_sol.log; exit 1; }
grep -h -o '"model": "[a-z]*", "wire": "[a-z0-9]*".*"G_rows_per_s": [0-9.]*' $O/prof_sol.log
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e2e -o run -- python3 $R/bench/e2e.py --broker inproc --fmt json --seconds 5 --warmup 2 > $O/prof_e2e.log 2>&1 || { tail -20 $O/prof_e2e.log; exit 1; }
find $O -name '*kernel_stats.csv' | sort
