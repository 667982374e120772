#!/bin/bash
# Round 4, the committed tree: the deployed topology with the GBDT model (G20 rows binned at
# ingest by the native consumer): TXB1 open loop and JSON at 1.2e6/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4w
mkdir -p $O
step() { echo "[r4w] $(date +%T) $*"; }
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['model'], d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'checks', d['checks_passed'], 'a->s', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'])
print('produce->scored', d['produce_to_scored_us']); print('scored->started', d['scored_to_process_started_us'])" "$1"; }
run() {
  local n=$1; shift
  step $n
  timeout -k 30 300 python bench/deploy_topology.py --seconds 30 "$@" --log-dir $O/$n --out $O/$n.json > $O/$n.log 2>&1 \
    || { tail -40 $O/$n.log; exit 1; }
  show $O/$n.json
}
run gbdt_txb1 --model gbdt --producers 4 --rate 0 --fmt txb1
run gbdt_json --model gbdt --producers 3 --rate 1200000 --fmt json
step done
