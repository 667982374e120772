set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r79; mkdir -p $O
for v in 0 1; do
CCFD_MLP_REGW=$v timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64 --sizes 32768,65536,262144,1048576,4194304 --tag regw$v > $O/sol_$v.log 2>&1 || { tail -30 $O/sol_$v.log; exit 1; }
echo "REGW=$v"; grep -h -o '"rows": [0-9]*.*"G_rows_per_s": [0-9.]*' $O/sol_$v.log
done
for v in 0 1 0 1; do
CCFD_MLP_REGW=$v timeout -k 10 300 python bench.py --exec-mode launch --no-unloaded-probe > $O/launch_$v.log 2>&1 || { tail -30 $O/launch_$v.log; exit 1; }
echo "launch REGW=$v $(tail -1 $O/launch_$v.log | cut -c100-200)"
done
