#!/usr/bin/env bash
# Round-6 final pass 1: the whole GPU suite + smoke on the tree, then 60 s sustained runs of
# config 2 and config 4 on the collector-thread hand-off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6final; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6final] $(date +%T) $*"; }
st pytest
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
st smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for m in mlp gbdt; do
  st sustained $m
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 5 --min-timed-s 60 --out $O/bench_${m}_60s.json > $O/bench_${m}_60s.log 2>&1 || { tail -30 $O/bench_${m}_60s.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${m}_60s.json'));print({k:d.get(k) for k in ('value','ms_per_step','p50_latency_us','p99_latency_us','fraud_routed','flagged_handed_off','handoff_stalls','h2d_zerocopy_ceiling_tx_s_rank0')})"
done
st done
