#!/usr/bin/env bash
# Round-6 pass I: the fraud hand-off on a collector thread beside the pump (FlaggedDrainer).
# Pump-only driver with and without it, the lossless hand-off GPU tests, then bench.py
# config 4 and config 2 (the driver's) on the new harness.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6i; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6i] $(date +%T) $*"; }
run() { n=$1; shift; st $n; timeout -k 10 180 python3 -u bench/pmc_persist.py --batches 200000 --segments 10 "$@" > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }; cat $O/$n.json; }
# (pump-only A/B done in the first pass I run)

st tests
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_handoff_lossless_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
st bench gbdt
timeout -k 10 300 python3 -u bench.py --model gbdt --steps 20 --warmup 5 --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_gbdt.json'));print({k:d.get(k) for k in ('value','vs_baseline','p50_latency_us','p99_latency_us','fraud_routed','flagged_handed_off','handoff_stalls','h2d_zerocopy_ceiling_tx_s_rank0')})"
st bench mlp
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --out $O/bench_mlp.json > $O/bench_mlp.log 2>&1 || { tail -30 $O/bench_mlp.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_mlp.json'));print({k:d.get(k) for k in ('value','vs_baseline','p50_latency_us','p99_latency_us','fraud_routed','flagged_handed_off','handoff_stalls','h2d_zerocopy_ceiling_tx_s_rank0')})"
st done
