set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r80; mkdir -p $O
CCFD_MLP_WAVES=16 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_wire.py -x -q -k "wire or w64" --timeout 120 --timeout-method thread > $O/pytest16.log 2>&1 || { tail -40 $O/pytest16.log; exit 1; }
tail -1 $O/pytest16.log
CCFD_MLP_WAVES=8 CCFD_MLP_REGW=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_wire.py -x -q -k "wire or w64" --timeout 120 --timeout-method thread > $O/pytest8r.log 2>&1 || { tail -40 $O/pytest8r.log; exit 1; }
tail -1 $O/pytest8r.log
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64 --sizes 65536,262144,1048576,4194304,16777216 --tag $tag > $O/sol_$tag.log 2>&1 || { tail -30 $O/sol_$tag.log; exit 1; }; echo "$tag $(grep -h -o '"G_rows_per_s": [0-9.]*' $O/sol_$tag.log | awk '{printf "%s ", $2}')"; }
run w4 CCFD_MLP_WAVES=4
run w8 CCFD_MLP_WAVES=8
run w16 CCFD_MLP_WAVES=16
run w4r CCFD_MLP_WAVES=4 CCFD_MLP_REGW=1
run w8r CCFD_MLP_WAVES=8 CCFD_MLP_REGW=1
timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64 --sizes 65536,262144,1048576,4194304,16777216 --flags 64 --tag nofence > $O/sol_nofence.log 2>&1 || exit 1
echo "w4 nofence $(grep -h -o '"G_rows_per_s": [0-9.]*' $O/sol_nofence.log | awk '{printf "%s ", $2}')"
