#!/bin/bash
# Round 4: deployed topology after the pooled TXB1 producer and the KIE journal fix, with GC /
# journal-write attribution at KIE: TXB1 open loop (4 producers) with the KIE journal on the
# broker's disk ($TMPDIR) and on /dev/shm; JSON at 1.2e6/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
step() { echo "[r4h] $(date +%T) $*"; }
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'arrival->scored', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], 'checks', d['checks_passed'])
print('samples', [s['tx_s'] for s in d['samples']])
print('produce->scored', d['produce_to_scored_us'])
print('scored->started', d['scored_to_process_started_us'])
print('engine handoff', d.get('handoff_engine_us'))
print('kie', d.get('kie_handoff_attribution'))" "$1"; }
step txb1 open loop, 4 producers, journal on TMPDIR
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 4 --rate 0 --fmt txb1 \
  --log-dir $O/txb1 --out $O/topo_txb1_4p.json > $O/topo_txb1_4p.log 2>&1 || { tail -40 $O/topo_txb1_4p.log; exit 1; }
show $O/topo_txb1_4p.json
step txb1 open loop, 4 producers, journal on /dev/shm
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 4 --rate 0 --fmt txb1 --journal-dir /dev/shm \
  --log-dir $O/txb1_shm --out $O/topo_txb1_4p_shm.json > $O/topo_txb1_4p_shm.log 2>&1 || { tail -40 $O/topo_txb1_4p_shm.log; exit 1; }
show $O/topo_txb1_4p_shm.json
step json 1.2e6
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 3 --rate 1200000 --fmt json \
  --log-dir $O/json --out $O/topo_json.json > $O/topo_json.log 2>&1 || { tail -40 $O/topo_json.log; exit 1; }
show $O/topo_json.json
step done
