#!/usr/bin/env bash
# Round-6 final pass 2: the committed tree as the driver runs it -- whole GPU suite, smoke,
# then bench.py with no flags (config 2) and config 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6final2; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6final2] $(date +%T) $*"; }
st pytest
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
st smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
st bench default
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log || { tail -30 $O/bench_default.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('value','steps','ms_per_step','p50_latency_us','p99_latency_us','fraud_routed','flagged_handed_off','handoff_stalls','h2d_zerocopy_ceiling_tx_s_rank0')})"
st bench gbdt
timeout -k 10 300 python -u bench.py --model gbdt --steps 20 --warmup 5 --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_gbdt.json'));print({k:d.get(k) for k in ('value','p50_latency_us','p99_latency_us','fraud_routed','flagged_handed_off','handoff_stalls','h2d_zerocopy_ceiling_tx_s_rank0')})"
st done
