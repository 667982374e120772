set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r31_$name.log 2>&1 || { tail -20 gpurun_out/r31_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r31_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["step_us_per_batch"], d["host_us_per_batch"], d["rows_scored"]==d["rows_expected"])')"; }
CCFD_PERSIST_ITEM_ROWS=512 run p512_g256_d8 --exec-mode persistent --persist-grid 256 --depth 8
CCFD_PERSIST_ITEM_ROWS=512 run p512_g256_d16 --exec-mode persistent --persist-grid 256 --depth 16 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=1024 run p1024_g256_d16 --exec-mode persistent --persist-grid 256 --depth 16 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=512 run p512_g128_d16 --exec-mode persistent --persist-grid 128 --depth 16 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=256 run p256_g256_d12 --exec-mode persistent --persist-grid 256 --depth 12 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=256 run p256_g256_d24 --exec-mode persistent --persist-grid 256 --depth 24 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=256 run p256_g384_d16 --exec-mode persistent --persist-grid 384 --depth 16 --no-unloaded-probe
