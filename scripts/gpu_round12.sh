set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu12.log 2>&1 || { tail -40 gpurun_out/pytest_gpu12.log; exit 1; }
tail -2 gpurun_out/pytest_gpu12.log
run() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r12_$name.log 2>&1 || { tail -20 gpurun_out/r12_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/r12_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["p50_latency_us"], d["p50_latency_us_unloaded"], d["ms_per_step"], d["rows_scored"]==d["rows_expected"])')"; }
run base --no-unloaded-probe
CCFD_ABLATE=16 run no_cnt --no-unloaded-probe
CCFD_ABLATE=32 run no_out --no-unloaded-probe
CCFD_ABLATE=64 run no_fence --no-unloaded-probe
CCFD_ABLATE=112 run no_all --no-unloaded-probe
run b8k --batch 8192 --batches-per-step 128 --no-unloaded-probe
run b16k --batch 16384 --batches-per-step 64 --no-unloaded-probe
run b64k --batch 65536 --batches-per-step 16 --no-unloaded-probe
run dma_in --input-mode dma --no-unloaded-probe
