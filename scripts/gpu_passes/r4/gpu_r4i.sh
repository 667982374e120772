#!/bin/bash
# Round 4: deployed topology with the small-young-generation GC policy (KIE pauses) and
# attribution maxima placed in time (max_at vs window_wall): TXB1 open loop x3 (journal on
# TMPDIR, /dev/shm, TMPDIR again: is the journal's disk a throughput factor or run order?),
# JSON at 1.2e6/s, process mode at 2e5/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
step() { echo "[r4i] $(date +%T) $*"; }
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'arrival->scored', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], 'checks', d['checks_passed'], d.get('kie_standard_plus_fraud_equals_incoming'))
print('window', d.get('window_wall'), 'drained', d.get('drained_wall'), 'samples', [s['tx_s'] for s in d['samples']])
print('produce->scored', d['produce_to_scored_us'])
print('scored->started', d['scored_to_process_started_us'])
print('engine handoff', d.get('handoff_engine_us'))
print('kie', d.get('kie_handoff_attribution'))" "$1"; }
run() {   # name, extra args...
  local n=$1; shift
  step $n
  timeout -k 30 300 python bench/deploy_topology.py --seconds 30 "$@" --log-dir $O/$n --out $O/$n.json > $O/$n.log 2>&1 \
    || { tail -40 $O/$n.log; exit 1; }
  show $O/$n.json
}
run txb1_tmp --producers 4 --rate 0 --fmt txb1
run txb1_shm --producers 4 --rate 0 --fmt txb1 --journal-dir /dev/shm
run txb1_tmp2 --producers 4 --rate 0 --fmt txb1
run json --producers 3 --rate 1200000 --fmt json
run json_process --producers 2 --rate 200000 --fmt json --standard-mode process
step done
