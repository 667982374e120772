set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r32_$name.log 2>&1 || { tail -20 gpurun_out/r32_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r32_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
CCFD_PERSIST_ITEM_ROWS=512 run p512_g128_d24 --exec-mode persistent --persist-grid 128 --depth 24 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=512 run p512_g128_d32 --exec-mode persistent --persist-grid 128 --depth 32 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=256 run p256_g128_d24 --exec-mode persistent --persist-grid 128 --depth 24 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=512 run p512_g192_d20 --exec-mode persistent --persist-grid 192 --depth 20 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=512 run p512_g128_d16_b --exec-mode persistent --persist-grid 128 --depth 16
run launch_default --no-unloaded-probe
