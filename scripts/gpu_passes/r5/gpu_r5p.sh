#!/usr/bin/env bash
# Round-5 pass P (item 4): where the replicated JSON produce -> scored tail comes from -- the
# same 60 s JSON run at RF 1 (no replication: the leaders' own path) and RF 2, next to pass M's
# RF 3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/${R5P_OUT:-r5p}; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r5p] $(date +%T) $*"; }
for rf in ${R5P_RFS:-1 2}; do
  st rf$rf
  timeout -k 10 300 python bench/deploy_topology.py --kafka-replicated --kafka-rf $rf --producer-acks -1 \
      --producer-max-in-flight 5 --seconds 60 --producers 3 --rate 1.2e6 --fmt json --log-dir $O/rf$rf \
      --out $O/repl_json_60s_rf$rf.json > $O/rf$rf.log 2>&1; rc=$?
  st "rf$rf rc=$rc"; [ $rc -ge 2 ] && { tail -30 $O/rf$rf.log; exit $rc; }
  python -c "import json; d=json.load(open('$O/repl_json_60s_rf$rf.json')); print($rf, d['value'], d['produce_to_scored_us'], d['checks_passed'], d.get('cpu_s_by_service'))"
done
st done
