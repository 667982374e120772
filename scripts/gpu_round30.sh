set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu30.log 2>&1 || { tail -40 gpurun_out/pytest_gpu30.log; exit 1; }
tail -1 gpurun_out/pytest_gpu30.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r30_$name.log 2>&1 || { tail -20 gpurun_out/r30_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r30_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
CCFD_PERSIST_ITEM_ROWS=256 run p256_g256_d8 --exec-mode persistent --persist-grid 256 --depth 8
CCFD_PERSIST_ITEM_ROWS=256 run p256_g256_d16 --exec-mode persistent --persist-grid 256 --depth 16 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=128 run p128_g256_d8 --exec-mode persistent --persist-grid 256 --depth 8 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=256 run p256_g512_d8 --exec-mode persistent --persist-grid 512 --depth 8 --no-unloaded-probe
