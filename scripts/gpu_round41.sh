set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r41
CCFD_GBDT_LEAVES=global timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k gbdt > gpurun_out/r41/pytest_gbdt_global.log 2>&1 || { tail -30 gpurun_out/r41/pytest_gbdt_global.log; exit 1; }
tail -1 gpurun_out/r41/pytest_gbdt_global.log
run() { name=$1; shift; timeout -k 10 300 python bench.py --model gbdt --batch 65536 --batches-per-step 16 --coalesce 1 --no-unloaded-probe --steps 60 --warmup 5 "$@" > gpurun_out/r41/$name.log 2>&1 || { tail -20 gpurun_out/r41/$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r41/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "Mtx/s dev_exec_us", d.get("device_exec_us_mean"), "step_us", d.get("step_us_per_batch"))')"; }
run lds_d8 --depth 8
CCFD_GBDT_LEAVES=global run glob_d8 --depth 8
run lds_d16_s8 --depth 16 --streams 8
CCFD_GBDT_LEAVES=global run glob_d16_s8 --depth 16 --streams 8
run lds_d4_s2 --depth 4 --streams 2
run lds_b16k --depth 16 --batch 16384 --batches-per-step 64
