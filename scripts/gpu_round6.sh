set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu6.log 2>&1 || { tail -40 gpurun_out/pytest_gpu6.log; exit 1; }
tail -2 gpurun_out/pytest_gpu6.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r6_$name.log 2>&1 || { tail -20 gpurun_out/r6_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r6_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["ms_per_step"], d["rows_scored"]==d["rows_expected"])')"; }
run persist_default
run persist_d16 --depth 16 --no-unloaded-probe
run persist_g512 --persist-grid 512 --no-unloaded-probe
run launch --exec-mode launch --no-unloaded-probe
run lr_persist --model lr --no-unloaded-probe
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench/engine_sweep.py --rounds 2 --batches 1024 --modes zerocopy:zerocopy --depths 8,16 --streams 8,16 > gpurun_out/r6_sweep_q$q.log 2>&1 || exit $?
  echo "== GPU_MAX_HW_QUEUES=$q"; grep tx_per gpurun_out/r6_sweep_q$q.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['depth'], d['streams'], d['tx_per_s_median'], d['p50_us'], d['us_per_batch'], d['host_submit_us'], d['host_wait_us'])"
done
