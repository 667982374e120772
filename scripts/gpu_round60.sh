set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r60; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64"
for pf in 2 4; do CCFD_MLP_PF=$pf $K --tag pair_pf$pf >> $O/sweep.jsonl 2>>$O/err.log || exit 1; done
cat $O/sweep.jsonl
