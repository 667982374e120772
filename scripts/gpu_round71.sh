set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r71; mkdir -p $O
for fl in 0 128 256 384 0; do
  timeout -k 10 120 python bench/kernel_sol.py --cases lr:w64,mlp:w64 --sizes 16777216 --flags $fl --tag st$fl > $O/st_$fl.log 2>&1 || { tail -30 $O/st_$fl.log; exit 1; }
  grep -h -o '"tag": "[a-z0-9]*".*"G_rows_per_s": [0-9.]*' $O/st_$fl.log
done
