set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu16.log 2>&1 || { tail -40 gpurun_out/pytest_gpu16.log; exit 1; }
tail -2 gpurun_out/pytest_gpu16.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r16_$name.log 2>&1 || { tail -20 gpurun_out/r16_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r16_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
run c1
run c2 --coalesce 2 --no-unloaded-probe
run c4 --coalesce 4
run c8 --coalesce 8 --depth 16 --no-unloaded-probe
run c4_s8_d16 --coalesce 4 --streams 8 --depth 16 --no-unloaded-probe
run c4_d16 --coalesce 4 --depth 16 --no-unloaded-probe
run c1_s8_d16 --streams 8 --depth 16 --no-unloaded-probe
