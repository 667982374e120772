#!/usr/bin/env bash
# Round-6 pass K: config 4's operating point re-swept on the collector-thread harness
# (micro-batch rows x batches in flight; persistent grid).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6k; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6k] $(date +%T) $*"; }
for cfg in 65536-4-0 65536-5-0 49152-5-0 32768-8-0 65536-4-256; do
  b=${cfg%%-*}; rest=${cfg#*-}; d=${rest%%-*}; gr=${rest#*-}
  st $cfg
  timeout -k 10 300 python -u bench.py --model gbdt --steps 20 --warmup 5 --batch $b --depth $d --persist-grid $gr \
    --no-f32-probe --out $O/bench_gbdt_$cfg.json > $O/bench_gbdt_$cfg.log 2>&1 || { tail -30 $O/bench_gbdt_$cfg.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_gbdt_$cfg.json'));print('$cfg',{k:d.get(k) for k in ('value','p50_latency_us','p99_latency_us','flagged_handed_off','fraud_routed','h2d_zerocopy_ceiling_tx_s_rank0')})"
done
st done
