set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py tests/test_engine_service_gpu.py -x -q > gpurun_out/pytest_gpu8.log 2>&1 || { tail -40 gpurun_out/pytest_gpu8.log; exit 1; }
tail -2 gpurun_out/pytest_gpu8.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r8_$name.log 2>&1 || { tail -20 gpurun_out/r8_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r8_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["ms_per_step"], d["rows_scored"]==d["rows_expected"])')"; }
for ir in 64 128; do
  for g in 128 256; do
    CCFD_PERSIST_ITEM_ROWS=$ir run p_i${ir}_g$g --persist-grid $g
  done
done
CCFD_PERSIST_ITEM_ROWS=64 run p_i64_g256_d16 --persist-grid 256 --depth 16 --no-unloaded-probe
run launch --exec-mode launch --no-unloaded-probe
