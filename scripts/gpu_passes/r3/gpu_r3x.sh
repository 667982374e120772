#!/bin/bash
# Round-3 GPU pass X: the final tree in the deployed topology (config 5, JSON per message at
# 1.2e6 tx/s for 60 s; TXB1 open loop 30 s) and a 60 s sustained headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
step() { echo "[r3x] $(date +%T) $*"; }
step pytest probes
timeout -k 10 200 python -u -m pytest tests/test_probes_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_probes.log 2>&1 || { tail -40 $O/pytest_probes.log; exit 1; }
tail -1 $O/pytest_probes.log
step deploy topology mlp json 1.2e6 60 s
timeout -k 30 420 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1200000 --fmt json \
    --log-dir $O/topo_json --out $O/topo_json.json > $O/topo_json.log 2>&1 || { tail -40 $O/topo_json.log; exit 1; }
tail -c 1200 $O/topo_json.json; echo
step deploy topology mlp txb1 open loop 30 s
timeout -k 30 360 python bench/deploy_topology.py --seconds 30 --producers 4 --rate 0 --fmt txb1 \
    --log-dir $O/topo_txb1 --out $O/topo_txb1.json > $O/topo_txb1.log 2>&1 || { tail -40 $O/topo_txb1.log; exit 1; }
tail -c 1200 $O/topo_txb1.json; echo
step bench 60 s sustained
timeout -k 10 400 python bench.py --min-timed-s 60 --out $O/bench_60s.json > $O/bench_60s.log 2>&1 || { tail -30 $O/bench_60s.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_60s.json')); print(d['value'], d['p50_latency_us'], d['p99_latency_us'], d['timed_region_s'], d['rows_scored']==d['rows_expected'])"
du -sh gpurun_out
step done
bash scripts/gpu_passes/r3/gpu_r3y.sh
