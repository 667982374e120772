#!/bin/bash
# Round 4: the native consumer's parallel JSON parse as the default (4 threads): smoke, the GPU
# tests that drive the native consumer / engine service, and the JSON deployed topology.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
step() { echo "[r4p] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step pytest gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step json topology
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 3 --rate 1200000 --fmt json \
  --log-dir $O/json --out $O/json.json > $O/json.log 2>&1 || { tail -40 $O/json.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/json.json'))
print(d['value'], d['min_sample_tx_s'], d['checks_passed'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'])
print(d['produce_to_scored_us']); print(d['scored_to_process_started_us'])"
step done
