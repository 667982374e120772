set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu18.log 2>&1 || { tail -40 gpurun_out/pytest_gpu18.log; exit 1; }
tail -1 gpurun_out/pytest_gpu18.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r18_$name.log 2>&1 || { tail -20 gpurun_out/r18_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r18_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
run base --coalesce 4 --depth 16 --no-unloaded-probe
CCFD_MLP_TPW=2 run tpw2 --coalesce 4 --depth 16
CCFD_MLP_TPW=4 run tpw4 --coalesce 4 --depth 16 --no-unloaded-probe
CCFD_MLP_TPW=2 run tpw2_c8_d32 --coalesce 8 --depth 32 --no-unloaded-probe
GPU_MAX_HW_QUEUES=8 run q8_s8 --coalesce 4 --depth 16 --streams 8 --no-unloaded-probe
GPU_MAX_HW_QUEUES=8 CCFD_MLP_TPW=2 run q8_s8_tpw2 --coalesce 4 --depth 32 --streams 8 --no-unloaded-probe
