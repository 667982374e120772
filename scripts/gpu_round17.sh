set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r17_$name.log 2>&1 || { tail -20 gpurun_out/r17_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r17_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
run base --coalesce 4 --depth 16 --no-unloaded-probe
CCFD_ABLATE=112 run ablate_all --coalesce 4 --depth 16 --no-unloaded-probe
CCFD_ABLATE=64 run no_fence --coalesce 4 --depth 16 --no-unloaded-probe
CCFD_MLP_WEIGHTS=global run gw --coalesce 4 --depth 16 --no-unloaded-probe
run lr --model lr --depth 16 --no-unloaded-probe
run c4_d32 --coalesce 4 --depth 32 --streams 8 --no-unloaded-probe
run c8_d32 --coalesce 8 --depth 32 --streams 4 --no-unloaded-probe
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof17" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-unloaded-probe --coalesce 4 --depth 16 > "$R/gpurun_out/prof17.log" 2>&1 || { tail -20 "$R/gpurun_out/prof17.log"; exit 1; }
echo prof-ok
