set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r52; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gbdt or strided" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
K="timeout -k 10 120 python bench/kernel_sol.py"
CCFD_GBDT_R=1 $K --cases gbdt:f32 --tag gbdt_v2_r1 >> $O/sweep.jsonl 2>>$O/err.log || exit 1
CCFD_GBDT_R=2 $K --cases gbdt:f32 --tag gbdt_v2_r2 >> $O/sweep.jsonl 2>>$O/err.log || exit 1
CCFD_GBDT_KERNEL=v1 $K --cases gbdt:f32 --tag gbdt_v1 >> $O/sweep.jsonl 2>>$O/err.log || exit 1
cat $O/sweep.jsonl
timeout -k 10 300 python bench.py --model gbdt --batch 65536 --batches-per-step 16 --steps 20 --warmup 3 > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
tail -1 $O/bench_gbdt.log
