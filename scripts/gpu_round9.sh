set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu9.log 2>&1 || { tail -40 gpurun_out/pytest_gpu9.log; exit 1; }
tail -2 gpurun_out/pytest_gpu9.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r9_$name.log 2>&1 || { tail -20 gpurun_out/r9_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r9_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["ms_per_step"], d["rows_scored"]==d["rows_expected"])')"; }
run w_auto
CCFD_MLP_WAVES=4 run w4
CCFD_MLP_WAVES=2 run w2 --no-unloaded-probe
run w_auto_s8 --streams 8 --no-unloaded-probe
run w_auto_d16 --depth 16 --no-unloaded-probe
run lr --model lr --no-unloaded-probe
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof9" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-unloaded-probe > "$GRAFT_REPO_ROOT/gpurun_out/prof9.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof9.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof9" -name "*stats.csv" | head -5
