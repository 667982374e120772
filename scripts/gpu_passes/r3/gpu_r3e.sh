#!/bin/bash
# Round-3 GPU pass E: GBDT ingest attribution (consumer-only e2e), GBDT in the deployed
# topology (JSON per message -> G20 rows binned at ingest), MLP deployed-topology capacity
# with more producers.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
step() { echo "[r3e] $(date +%T) $*"; }
step gbdt e2e consumer-only attribution
timeout -k 10 300 python bench/e2e.py --model gbdt --broker kafka-lite --fmt txb1 --prefill-s 8 --seconds 8 \
    --out $O/e2e_gbdt_prefill.json > $O/e2e_gbdt.log 2>&1 || { tail -30 $O/e2e_gbdt.log; exit 1; }
cat $O/e2e_gbdt_prefill.json
step deploy topology gbdt json 30 s
timeout -k 30 360 python bench/deploy_topology.py --model gbdt --seconds 30 --producers 3 --rate 1200000 --fmt json \
    --log-dir $O/topo_gbdt --out $O/topo_gbdt.json > $O/topo_gbdt.log 2>&1 || { tail -40 $O/topo_gbdt.log; exit 1; }
tail -c 1200 $O/topo_gbdt.json
step deploy topology mlp open loop 6 producers 30 s
timeout -k 30 360 python bench/deploy_topology.py --seconds 30 --producers 6 --rate 0 --fmt json \
    --log-dir $O/topo_max6 --out $O/topo_max6.json > $O/topo_max6.log 2>&1 || { tail -40 $O/topo_max6.log; exit 1; }
tail -c 1200 $O/topo_max6.json
step done
