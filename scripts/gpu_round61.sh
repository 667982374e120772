set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r61; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gbdt or strided" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python bench/kernel_sol.py --cases gbdt:f32 --sizes 1048576,16777216 --tag gbdt_v2_prefetch >> $O/sweep.jsonl 2>>$O/err.log || exit 1
cat $O/sweep.jsonl
