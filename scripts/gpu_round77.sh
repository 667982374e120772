set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r77; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k gbdt --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 120 python bench/kernel_sol.py --cases gbdt:f32 --sizes 1048576,16777216 --tag tb4 > $O/sol_$i.log 2>&1 || { tail -30 $O/sol_$i.log; exit 1; }
grep -h -o '"rows": [0-9]*.*"G_rows_per_s": [0-9.]*' $O/sol_$i.log
done
timeout -k 10 300 python bench.py --model gbdt --steps 30 --warmup 5 --no-unloaded-probe > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
tail -1 $O/bench_gbdt.log | cut -c1-250
