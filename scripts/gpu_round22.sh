set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu22.log 2>&1 || { tail -40 gpurun_out/pytest_gpu22.log; exit 1; }
tail -1 gpurun_out/pytest_gpu22.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r22_$name.log 2>&1 || { tail -20 gpurun_out/r22_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r22_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
run mlp_default
run lr_default --model lr
run lr_f32 --model lr --wire f32 --no-unloaded-probe
