set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r67; mkdir -p $O
# the driver's N>1 launch line at N=1, with the process group forced on so X1/X2/X3 run over
# real RCCL next to the persistent scoring kernel
CCFD_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 100 --warmup 10 > $O/bench_forced_rccl.log 2>&1 || { tail -40 $O/bench_forced_rccl.log; exit 1; }
tail -1 $O/bench_forced_rccl.log
