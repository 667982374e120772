#!/bin/bash
# Round-3 GPU pass F: the full GPU suite after the round's changes, the deployed topology with
# a KIE crash (SIGKILL) and restart from its journal mid-stream, default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
step() { echo "[r3f] $(date +%T) $*"; }
step pytest
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step deploy topology with KIE crash + journal restart
timeout -k 30 420 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1200000 --fmt json \
    --kie-outage-at 20 --kie-outage-s 5 --log-dir $O/topo_kie_crash --out $O/topo_kie_crash.json > $O/topo_kie_crash.log 2>&1 \
    || { tail -40 $O/topo_kie_crash.log; exit 1; }
tail -c 1500 $O/topo_kie_crash.json
step bench default
timeout -k 10 300 python bench.py --out $O/bench_default.json > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
step done
