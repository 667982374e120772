set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export CCFD_DIST_BACKEND=gloo CCFD_DEVICE_MODULO=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench/e2e.py --seconds 6 --warmup 2 --flush-us 100 --out gpurun_out/e2e_dp2.json > gpurun_out/e2e_dp2.log 2>&1 || { tail -40 gpurun_out/e2e_dp2.log; exit 1; }
cat gpurun_out/e2e_dp2.json
