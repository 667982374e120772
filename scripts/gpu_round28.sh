set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r28_$name.log 2>&1 || { tail -20 gpurun_out/r28_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r28_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
run base --no-unloaded-probe
CCFD_ABLATE=64 run no_fence --no-unloaded-probe
CCFD_ABLATE=32 run no_out --no-unloaded-probe
CCFD_ABLATE=112 run none --no-unloaded-probe
run s8 --streams 8 --no-unloaded-probe
GPU_MAX_HW_QUEUES=8 run q8s8 --streams 8 --no-unloaded-probe
run d64 --depth 64 --no-unloaded-probe
CCFD_MLP_TPW=4 run tpw4 --no-unloaded-probe
