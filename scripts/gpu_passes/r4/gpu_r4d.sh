#!/bin/bash
# Round 4: GPU tests of the new paths + traced deployed-topology runs (tail attribution:
# the round-3 Python scoring thread vs the native serving thread), process mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
step() { echo "[r4d] $(date +%T) $*"; }
step pytest subset
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  -k "scored or engine_service or handoff or serve" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for serving in python native; do
  step txb1 open loop traced, $serving serving
  timeout -k 30 300 python bench/deploy_topology.py --seconds 20 --producers 3 --rate 0 --fmt txb1 --trace \
    --serving $serving --log-dir $O/txb1_$serving --out $O/topo_txb1_$serving.json > $O/topo_txb1_$serving.log 2>&1 \
    || { tail -40 $O/topo_txb1_$serving.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/topo_txb1_$serving.json')); print(d['value'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], d['checks_passed']); print(json.dumps(d.get('tail_attribution'))[:1200])"
done
step json process-mode traced
timeout -k 30 300 python bench/deploy_topology.py --seconds 20 --producers 2 --rate 200000 --fmt json --trace \
  --standard-mode process --log-dir $O/json_proc --out $O/topo_json_process.json > $O/topo_json_process.log 2>&1 || { tail -40 $O/topo_json_process.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_json_process.json')); print(d['value'], d['checks_passed'], d.get('kie_standard_plus_fraud_equals_incoming'), d['kie']); print(json.dumps(d.get('tail_attribution'))[:1200])"

step counters list
timeout -k 10 120 rocprofv3 -L > $O/rocprofv3_counters.txt 2>&1 || true
head -3 $O/rocprofv3_counters.txt
step done
