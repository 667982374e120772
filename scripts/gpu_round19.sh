set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu19.log 2>&1 || { tail -40 gpurun_out/pytest_gpu19.log; exit 1; }
tail -1 gpurun_out/pytest_gpu19.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r19_$name.log 2>&1 || { tail -20 gpurun_out/r19_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r19_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
run c4_d16 --coalesce 4 --depth 16
run c8_d32 --coalesce 8 --depth 32 --no-unloaded-probe
run c4_d32 --coalesce 4 --depth 32 --no-unloaded-probe
run c2_d16 --coalesce 2 --depth 16 --no-unloaded-probe
CCFD_MLP_TPW=8 run tpw8_c4_d16 --coalesce 4 --depth 16 --no-unloaded-probe
CCFD_MLP_TPW=8 run tpw8_c8_d32 --coalesce 8 --depth 32 --no-unloaded-probe
run c1_d8 --no-unloaded-probe
run lr_c1 --model lr --no-unloaded-probe
run f32_c8_d32 --wire f32 --coalesce 8 --depth 32 --no-unloaded-probe
