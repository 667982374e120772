set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export CCFD_DIST_BACKEND=gloo CCFD_DEVICE_MODULO=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 3 --log-rows 1048576 > gpurun_out/dp2_rehearsal.log 2>&1 || { tail -40 gpurun_out/dp2_rehearsal.log; exit 1; }
tail -1 gpurun_out/dp2_rehearsal.log
