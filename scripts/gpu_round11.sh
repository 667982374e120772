set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu11.log 2>&1 || { tail -40 gpurun_out/pytest_gpu11.log; exit 1; }
tail -2 gpurun_out/pytest_gpu11.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r11_$name.log 2>&1 || { tail -20 gpurun_out/r11_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r11_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["ms_per_step"], d["rows_scored"]==d["rows_expected"])')"; }
run launch
CCFD_COHERENT_OUT=0 run launch_nc --no-unloaded-probe
run p_g128 --exec-mode persistent --persist-grid 128
run p_g256 --exec-mode persistent --persist-grid 256 --no-unloaded-probe
run p_g512 --exec-mode persistent --persist-grid 512 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=128 run p_i128_g256 --exec-mode persistent --persist-grid 256 --no-unloaded-probe
CCFD_PERSIST_ITEM_ROWS=256 run p_i256_g512 --exec-mode persistent --persist-grid 512 --no-unloaded-probe
run p_g256_d16 --exec-mode persistent --persist-grid 256 --depth 16 --no-unloaded-probe
GPU_MAX_HW_QUEUES=8 run launch_q8_s8 --streams 8 --no-unloaded-probe
