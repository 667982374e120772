#!/usr/bin/env bash
# Rehearse the N-rank bench path on a one-GPU box: N ranks share the GPU
# (CCFD_DEVICE_MODULO=1) and run their collectives over gloo.  First checks that bench.py
# REFUSES that topology without --rehearsal, then runs it with --rehearsal.
#   bash scripts/rehearse_dp.sh OUTDIR NPROC [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O="gpurun_out/$1"; N=$2; shift 2
mkdir -p "$O"
export CCFD_DIST_BACKEND=gloo CCFD_DEVICE_MODULO=1
run() {
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus "$N" "$@"
}
if run --steps 3 --warmup 1 --log-rows 1048576 > "$O/refuse.log" 2>&1; then
  echo "[rehearse] bench.py accepted a gloo / shared-GPU topology without --rehearsal"; exit 1
fi
grep -m3 "topology check failed" "$O/refuse.log" || { tail -20 "$O/refuse.log"; exit 1; }
# the rehearsal itself goes through bench.py's own launcher, exactly as the driver invokes
# config 2: `python bench.py --gpus N` spawns the N ranks (launch/local_ranks.py); --rehearsal
# makes the parent hand its children the gloo / shared-GPU env
unset CCFD_DIST_BACKEND CCFD_DEVICE_MODULO
timeout -k 10 300 python bench.py --gpus "$N" --rehearsal --out "$O/bench_dp${N}_rehearsal.json" "$@" \
  > "$O/rehearsal.log" 2>&1 || { tail -40 "$O/rehearsal.log"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('rehearsal dp%d' % d['n_gpus'], '%.4g tx/s' % d['value'], 'p50', d['p50_latency_us'], 'timed', d['timed_region_s'], [ (r['rank'], r['tx_s'], r['h2d_zerocopy_GBps']) for r in d['per_rank']])" "$O/bench_dp${N}_rehearsal.json"
