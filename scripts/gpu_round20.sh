set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu20.log 2>&1 || { tail -40 gpurun_out/pytest_gpu20.log; exit 1; }
tail -1 gpurun_out/pytest_gpu20.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke20.log 2>&1 || { tail -20 gpurun_out/smoke20.log; exit 1; }
tail -2 gpurun_out/smoke20.log
timeout -k 10 300 python bench.py --out gpurun_out/bench_default.json > gpurun_out/bench20.log 2>&1 || { tail -20 gpurun_out/bench20.log; exit 1; }
tail -1 gpurun_out/bench20.log
timeout -k 10 300 python bench.py --model lr --out gpurun_out/bench_lr.json > gpurun_out/bench20_lr.log 2>&1 || { tail -20 gpurun_out/bench20_lr.log; exit 1; }
timeout -k 10 300 python bench.py --model gbdt --batch 65536 --batches-per-step 16 --coalesce 1 --depth 8 --out gpurun_out/bench_gbdt.json > gpurun_out/bench20_gbdt.log 2>&1 || { tail -20 gpurun_out/bench20_gbdt.log; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof20" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-unloaded-probe > "$R/gpurun_out/prof20.log" 2>&1 || { tail -20 "$R/gpurun_out/prof20.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof20db" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-unloaded-probe > "$R/gpurun_out/prof20db.log" 2>&1 || { tail -20 "$R/gpurun_out/prof20db.log"; exit 1; }
find "$R/gpurun_out/prof20" -name "*.csv" | head
