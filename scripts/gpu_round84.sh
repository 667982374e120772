set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r84; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_all.log 2>&1 || { tail -60 $O/pytest_gpu_all.log; exit 1; }
tail -1 $O/pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 120 python bench/kernel_sol.py --sizes 1048576,16777216 --out $O/kernel_sol.json > $O/sol.log 2>&1 || { tail -30 $O/sol.log; exit 1; }
grep -h -o '"model": "[a-z]*", "wire": "[a-z0-9]*", "rows": [0-9]*.*"G_rows_per_s": [0-9.]*' $O/sol.log
