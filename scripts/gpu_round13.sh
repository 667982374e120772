set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu13.log 2>&1 || { tail -40 gpurun_out/pytest_gpu13.log; exit 1; }
tail -2 gpurun_out/pytest_gpu13.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r13_$name.log 2>&1 || { tail -20 gpurun_out/r13_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r13_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["ms_per_step"], d["rows_scored"]==d["rows_expected"])')"; }
run f32 --no-unloaded-probe
run w64
run w64_s8 --streams 8 --no-unloaded-probe
run w64_d16 --depth 16 --no-unloaded-probe
run w64_p128 --exec-mode persistent --persist-grid 128 --no-unloaded-probe
run w64_p256 --exec-mode persistent --persist-grid 256 --no-unloaded-probe
run w64_lr --model lr --no-unloaded-probe
