set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r72; mkdir -p $O
for i in 1 2; do for e in 1 8; do
timeout -k 10 300 python bench.py --no-unloaded-probe --x2-every $e > $O/plain_e${e}_$i.log 2>&1 || { tail -30 $O/plain_e${e}_$i.log; exit 1; }
CCFD_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 2962$e bench.py --gpus 1 --no-unloaded-probe --x2-every $e > $O/forced_e${e}_$i.log 2>&1 || { tail -40 $O/forced_e${e}_$i.log; exit 1; }
done; done
for f in $O/*.log; do echo $f; tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_latency_us'], d['host_us_per_step_x2'], d['ms_per_step'], d['rows_scored']==d['rows_expected'])"; done
