set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r55; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="timeout -k 10 120 python bench/kernel_sol.py"
$K --cases lr:w64,mlp:w64 --tag wirebody >> $O/sweep.jsonl 2>>$O/err.log || exit 1
cat $O/sweep.jsonl
timeout -k 10 300 python bench.py --model lr --steps 50 > $O/bench_lr.log 2>&1 || { tail -30 $O/bench_lr.log; exit 1; }
tail -1 $O/bench_lr.log | cut -c1-400
