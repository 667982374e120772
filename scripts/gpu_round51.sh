set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r51; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
K="timeout -k 10 120 python bench/kernel_sol.py"
$K --cases mlp:w64 --tag histlanes >> $O/sweep.jsonl 2>>$O/err.log || exit 1
$K --cases mlp:w64 --sizes 1048576,16777216 --flags 16 --tag histlanes_nocnt >> $O/sweep.jsonl 2>>$O/err.log || exit 1
cat $O/sweep.jsonl
