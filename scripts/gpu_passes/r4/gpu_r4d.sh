#!/bin/bash
# Round 4: GPU tests of the new paths + traced deployed-topology runs (tail attribution).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
step() { echo "[r4d] $(date +%T) $*"; }
step pytest subset
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  -k "scored or engine_service or handoff" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step txb1 open loop traced
timeout -k 30 300 python bench/deploy_topology.py --seconds 20 --producers 3 --rate 0 --fmt txb1 --trace \
  --log-dir $O/txb1 --out $O/topo_txb1.json > $O/topo_txb1.log 2>&1 || { tail -40 $O/topo_txb1.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_txb1.json')); print(d['value'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], d['checks_passed']); print(json.dumps(d.get('tail_attribution'))[:1500])"
step json process-mode traced
timeout -k 30 300 python bench/deploy_topology.py --seconds 20 --producers 2 --rate 200000 --fmt json --trace \
  --standard-mode process --log-dir $O/json_proc --out $O/topo_json_process.json > $O/topo_json_process.log 2>&1 || { tail -40 $O/topo_json_process.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_json_process.json')); print(d['value'], d['checks_passed'], d.get('kie_standard_plus_fraud_equals_incoming'), d['kie']); print(json.dumps(d.get('tail_attribution'))[:1500])"
step done
