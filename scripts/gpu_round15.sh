set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r15_$name.log 2>&1 || { tail -20 gpurun_out/r15_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r15_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["step_us_per_batch"], d["host_us_per_batch"])')"; }
run f32 --no-unloaded-probe
run w64 --wire w64 --no-unloaded-probe
run w64_s2 --wire w64 --streams 2 --no-unloaded-probe
run w64_s8_d16 --wire w64 --streams 8 --depth 16 --no-unloaded-probe
run w64_p128 --wire w64 --exec-mode persistent --persist-grid 128 --no-unloaded-probe
