set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
nproc > gpurun_out/r3_env.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/r3_env.txt; ls /sys/devices/system/node/ >> gpurun_out/r3_env.txt; cat /sys/devices/system/node/node*/cpulist >> gpurun_out/r3_env.txt 2>/dev/null
cat gpurun_out/r3_env.txt
run() { name=$1; shift; timeout -k 10 300 python bench.py --no-unloaded-probe "$@" > gpurun_out/r3_$name.log 2>&1 || exit $?; echo "$name $(tail -1 gpurun_out/r3_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["ms_per_step"])')"; }
run default
CCFD_NO_NUMA_BIND=1 run nonuma
run p1 --partitions-per-rank 1
run d16 --depth 16
run s8 --streams 8 --depth 16
run bps1024 --batches-per-step 1024 --steps 30
run dma --input-mode dma
timeout -k 10 300 python bench/engine_sweep.py --rounds 2 --batches 512 --modes zerocopy:zerocopy --depths 8,16 --streams 4,8 > gpurun_out/r3_sweep.log 2>&1 || exit $?
grep tx_per gpurun_out/r3_sweep.log
