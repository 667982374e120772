#!/bin/bash
# Round-3 GPU pass D: 4-rank gloo rehearsal of the deployed topology, open-loop capacity of
# the deployed topology, GBDT consumer-only e2e attribution.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
step() { echo "[r3d] $(date +%T) $*"; }
step deploy topology 4-rank rehearsal
timeout -k 30 360 python bench/deploy_topology.py --ranks 4 --rehearsal --seconds 20 --producers 2 --rate 300000 \
    --fmt json --log-dir $O/topo4 --out $O/topo4.json > $O/topo4.log 2>&1 || { tail -40 $O/topo4.log; grep -v "^W1017\|^I1017" $O/topo4/engine.log | tail -30; exit 1; }
tail -c 1500 $O/topo4.json
step deploy topology open loop 30 s
timeout -k 30 360 python bench/deploy_topology.py --seconds 30 --producers 4 --rate 0 --fmt json \
    --log-dir $O/topo1max --out $O/topo1max.json > $O/topo1max.log 2>&1 || { tail -40 $O/topo1max.log; exit 1; }
tail -c 1500 $O/topo1max.json
step gbdt e2e consumer-only attribution
timeout -k 10 300 python bench/e2e.py --model gbdt --broker kafka-lite --fmt txb1 --prefill-s 8 --seconds 8 \
    --out $O/e2e_gbdt_prefill.json > $O/e2e_gbdt.log 2>&1 || { tail -30 $O/e2e_gbdt.log; exit 1; }
cat $O/e2e_gbdt_prefill.json
step done
