set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r44
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py tests/test_engine_service_gpu.py -x -q > gpurun_out/r44/pytest.log 2>&1 || { tail -40 gpurun_out/r44/pytest.log; exit 1; }
tail -1 gpurun_out/r44/pytest.log
timeout -k 10 300 python bench.py --out gpurun_out/r44/bench_default.json > gpurun_out/r44/bench_default.log 2>&1 || { tail -20 gpurun_out/r44/bench_default.log; exit 1; }
cat gpurun_out/r44/bench_default.json
export CCFD_DIST_BACKEND=gloo CCFD_DEVICE_MODULO=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29617 bench/e2e.py --seconds 6 --warmup 2 --flush-us 100 --out gpurun_out/r44/e2e_dp4.json > gpurun_out/r44/e2e_dp4.log 2>&1 || { tail -40 gpurun_out/r44/e2e_dp4.log; exit 1; }
cat gpurun_out/r44/e2e_dp4.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29619 bench.py --gpus 4 --steps 20 --warmup 3 --out gpurun_out/r44/bench_dp4_gloo.json > gpurun_out/r44/bench_dp4.log 2>&1 || { tail -40 gpurun_out/r44/bench_dp4.log; exit 1; }
cat gpurun_out/r44/bench_dp4_gloo.json
