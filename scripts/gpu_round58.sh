set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/r58; mkdir -p $O
export CCFD_DIST_BACKEND=gloo CCFD_DEVICE_MODULO=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 3 --no-unloaded-probe > $O/bench_dp2_gloo.log 2>&1 || { tail -30 $O/bench_dp2_gloo.log; exit 1; }
grep '"metric"' $O/bench_dp2_gloo.log | cut -c1-330
unset CCFD_DIST_BACKEND CCFD_DEVICE_MODULO
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-unloaded-probe > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sol -o run -- python3 $R/bench/kernel_sol.py --sizes 16777216 --iters 5 > $O/prof_sol.log 2>&1 || { tail -20 $O/prof_sol.log; exit 1; }
find $O -name '*kernel_stats.csv' | sort
