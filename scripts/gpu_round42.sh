set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r42
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k gbdt > gpurun_out/r42/pytest_gbdt.log 2>&1 || { tail -30 gpurun_out/r42/pytest_gbdt.log; exit 1; }
tail -1 gpurun_out/r42/pytest_gbdt.log
CCFD_GBDT_CPW=1 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k gbdt > gpurun_out/r42/pytest_gbdt_cpw1.log 2>&1 || { tail -30 gpurun_out/r42/pytest_gbdt_cpw1.log; exit 1; }
tail -1 gpurun_out/r42/pytest_gbdt_cpw1.log
run() { name=$1; shift; timeout -k 10 300 python bench.py --model gbdt --batch 65536 --batches-per-step 16 --coalesce 1 --no-unloaded-probe --steps 60 --warmup 5 "$@" > gpurun_out/r42/$name.log 2>&1 || { tail -20 gpurun_out/r42/$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r42/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "Mtx/s dev_exec_us", d.get("device_exec_us_mean"), "step_us", d.get("step_us_per_batch"), "p50", d.get("p50_latency_us"))')"; }
run default_d8 --depth 8
CCFD_GBDT_CPW=1 run cpw1_d8 --depth 8
CCFD_GBDT_CPW=4 run cpw4_d8 --depth 8
CCFD_GBDT_CPW=8 run cpw8_d8 --depth 8
CCFD_GBDT_CPW=16 run cpw16_d8 --depth 8
run default_d4 --depth 4
run default_d16 --depth 16
