#!/bin/bash
# Round 4: what the durable broker costs and where the broker share of produce -> scored
# comes from: JSON 1.2e6/s and TXB1 open loop with fsync=interval (default) / never / the
# in-memory broker (--kafka-memory); JSON with 1024-message produce requests (the batch's
# serial parse is part of produce -> scored).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
step() { echo "[r4m] $(date +%T) $*"; }
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'checks', d['checks_passed'], 'durable', d.get('kafka_durable'))
print('produce->scored', d['produce_to_scored_us'])
print('scored->started', d['scored_to_process_started_us'])" "$1"; }
run() {
  local n=$1; shift
  step $n
  timeout -k 30 300 python bench/deploy_topology.py --seconds 30 "$@" --log-dir $O/$n --out $O/$n.json > $O/$n.log 2>&1 \
    || { tail -40 $O/$n.log; exit 1; }
  show $O/$n.json
}
run json_interval --producers 3 --rate 1200000 --fmt json
run json_never --producers 3 --rate 1200000 --fmt json --fsync never
run json_memory --producers 3 --rate 1200000 --fmt json --kafka-memory
run json_batch1024 --producers 3 --rate 1200000 --fmt json --batch 1024
run txb1_interval --producers 4 --rate 0 --fmt txb1
run txb1_memory --producers 4 --rate 0 --fmt txb1 --kafka-memory
step done
