#!/bin/bash
# Round-3 GPU pass C: config 5 in the deployed topology (separate processes) on one MI355X,
# the 4-rank gloo rehearsal of the same topology, GBDT consumer-only e2e attribution.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
step() { echo "[r3c] $(date +%T) $*"; }
step deploy topology 1 GPU json 60 s
timeout -k 30 420 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1200000 --fmt json \
    --log-dir $O/topo1 --out $O/topo1.json > $O/topo1.log 2>&1 || { tail -40 $O/topo1.log; tail -30 $O/topo1/engine.log; exit 1; }
tail -c 3000 $O/topo1.json
step deploy topology 4-rank rehearsal
timeout -k 30 360 python bench/deploy_topology.py --ranks 4 --rehearsal --seconds 20 --producers 2 --rate 300000 \
    --fmt json --log-dir $O/topo4 --out $O/topo4.json > $O/topo4.log 2>&1 || { tail -40 $O/topo4.log; tail -30 $O/topo4/engine.log; exit 1; }
step gbdt e2e consumer-only attribution
timeout -k 10 300 python bench/e2e.py --model gbdt --broker kafka-lite --fmt txb1 --prefill-s 8 --seconds 8 \
    --out $O/e2e_gbdt_prefill.json > $O/e2e_gbdt.log 2>&1 || { tail -30 $O/e2e_gbdt.log; exit 1; }
step done
