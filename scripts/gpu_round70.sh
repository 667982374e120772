set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r70; mkdir -p $O
for fl in 0 16 32 48; do
  timeout -k 10 120 python bench/kernel_sol.py --cases lr:w64,mlp:w64 --sizes 16777216 --flags $fl --tag abl$fl > $O/abl_$fl.log 2>&1 || { tail -30 $O/abl_$fl.log; exit 1; }
done
grep -h -o '"tag": "[a-z0-9]*".*"G_rows_per_s": [0-9.]*' $O/abl_*.log
