set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r82; mkdir -p $O
CCFD_LR_WAVES=16 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_wire.py -x -q -k "lr" --timeout 120 --timeout-method thread > $O/pytest16.log 2>&1 || { tail -40 $O/pytest16.log; exit 1; }
tail -1 $O/pytest16.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_wire.py -x -q -k "lr" --timeout 120 --timeout-method thread > $O/pytest8.log 2>&1 || { tail -40 $O/pytest8.log; exit 1; }
tail -1 $O/pytest8.log
for w in 4 8 16; do
CCFD_LR_WAVES=$w timeout -k 10 120 python bench/kernel_sol.py --cases lr:w64 --sizes 65536,262144,1048576,4194304,16777216 > $O/sol_$w.log 2>&1 || { tail -30 $O/sol_$w.log; exit 1; }
echo "w$w $(grep -h -o '"G_rows_per_s": [0-9.]*' $O/sol_$w.log | awk '{printf "%s ", $2}')"
done
