set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r57; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64 --sizes 1048576,16777216"
for pf in 1 2 4; do CCFD_MLP_PF=$pf $K --tag wpe_pf$pf >> $O/sweep.jsonl 2>>$O/err.log || exit 1; done
cat $O/sweep.jsonl
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
