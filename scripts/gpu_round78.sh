set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r78; mkdir -p $O
CCFD_MLP_REGW=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_wire.py -x -q -k "wire or w64" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64 --sizes 1048576,16777216 --tag lds > $O/lds_$i.log 2>&1 || { tail -30 $O/lds_$i.log; exit 1; }
grep -h -o '"rows": [0-9]*.*"G_rows_per_s": [0-9.]*' $O/lds_$i.log
CCFD_MLP_REGW=1 timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64 --sizes 1048576,16777216 --tag regw > $O/regw_$i.log 2>&1 || { tail -30 $O/regw_$i.log; exit 1; }
grep -h -o '"rows": [0-9]*.*"G_rows_per_s": [0-9.]*' $O/regw_$i.log
CCFD_MLP_REGW=1 CCFD_MLP_PF=4 timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64 --sizes 1048576,16777216 --tag regw_pf4 > $O/regw4_$i.log 2>&1 || { tail -30 $O/regw4_$i.log; exit 1; }
grep -h -o '"rows": [0-9]*.*"G_rows_per_s": [0-9.]*' $O/regw4_$i.log
done
