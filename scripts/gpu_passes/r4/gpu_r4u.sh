#!/bin/bash
# Round 4: is the durable TXB1 deployed rate producer-bound?  4 / 6 / 8 producer processes,
# open loop, durable broker.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
step() { echo "[r4u] $(date +%T) $*"; }
for np in 4 6 8; do
  step txb1 $np producers
  timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers $np --rate 0 --fmt txb1 \
    --log-dir $O/p$np --out $O/txb1_p$np.json > $O/txb1_p$np.log 2>&1 || { tail -40 $O/txb1_p$np.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/txb1_p$np.json'))
print($np, d['value'], d['min_sample_tx_s'], [s['tx_s'] for s in d['samples']], d['producers_tx_s'], d['checks_passed'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'])
print(d['produce_to_scored_us']); print(d['scored_to_process_started_us']); print(d.get('ingest_attribution'))"
done
step done
