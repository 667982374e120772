#!/bin/bash
# Round-3 GPU pass M: engine / service GPU tests with pipelined persistent items as the service
# default, then the deployed topology (JSON per message, 1.2e6 tx/s) pipelined vs claimed items.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
step() { echo "[r3m] $(date +%T) $*"; }
step pinned pages probe
timeout -k 10 120 python bench/experiments/pinned_pages.py --mb 1024 > $O/pinned_pages.jsonl 2>$O/pinned_pages.err || { tail -20 $O/pinned_pages.err; exit 1; }
cat $O/pinned_pages.jsonl
step engine + service GPU tests
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_rules_gpu.py tests/test_engine_service_gpu.py -x -q --timeout 180 --timeout-method thread > $O/pytest_engine.log 2>&1 || { tail -40 $O/pytest_engine.log; exit 1; }
tail -3 $O/pytest_engine.log
for mode in pipelined claimed; do
  step deploy topology json 30 s items=$mode
  CCFD_PERSIST_ITEMS=$mode timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 3 --rate 1200000 --fmt json \
      --log-dir $O/topo_$mode --out $O/topo_json_$mode.json > $O/topo_$mode.log 2>&1 || { tail -40 $O/topo_$mode.log; exit 1; }
  python - "$O/topo_json_$mode.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = [k for k in d if any(s in k for s in ("tx_s", "p50", "p99", "ok", "checks"))]
print({k: d[k] for k in keys})
PY
done
step done
