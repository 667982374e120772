set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench/engine_sweep.py --rounds 2 --batches 1024 --modes zerocopy:zerocopy --depths 8,16 --streams 4,8,16 > gpurun_out/r5_sweep_q$q.log 2>&1 || exit $?
  echo "== GPU_MAX_HW_QUEUES=$q"; grep tx_per gpurun_out/r5_sweep_q$q.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['depth'], d['streams'], d['tx_per_s_median'], d['p50_us'], d['us_per_batch'], d['host_submit_us'], d['host_wait_us'])"
done
