set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_engine_service_gpu.py -x -q > gpurun_out/pytest_gpu10.log 2>&1 || { tail -40 gpurun_out/pytest_gpu10.log; exit 1; }
tail -2 gpurun_out/pytest_gpu10.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r10_$name.log 2>&1 || { tail -20 gpurun_out/r10_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r10_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["ms_per_step"], d["rows_scored"]==d["rows_expected"])')"; }
run coh_w4
CCFD_COHERENT_OUT=0 run nc_w4 --no-unloaded-probe
CCFD_MLP_WAVES=1 run coh_w1 --no-unloaded-probe
CCFD_MLP_WAVES=2 run coh_w2 --no-unloaded-probe
run coh_w4_s8 --streams 8 --no-unloaded-probe
run coh_lr --model lr --no-unloaded-probe
run coh_gbdt --model gbdt --batch 65536 --batches-per-step 16 --no-unloaded-probe
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof10" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-unloaded-probe > "$GRAFT_REPO_ROOT/gpurun_out/prof10.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof10.log"; exit 1; }
echo prof-ok
