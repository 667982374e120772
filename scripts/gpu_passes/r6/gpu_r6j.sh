#!/usr/bin/env bash
# Round-6 pass J: bench.py's multi-rank path with the collector-thread hand-off, rehearsed on
# one GPU (ranks share it, gloo collectives, labelled rehearsal): dp2 and dp4, configs 2 and 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6j; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6j] $(date +%T) $*"; }
st pytest handoff
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_handoff_lossless_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for n in 2 4; do
  for m in mlp gbdt; do
    st dp$n $m
    timeout -k 10 400 python bench.py --gpus $n --rehearsal --model $m --steps 10 --warmup 3 --out $O/bench_${m}_dp${n}r.json > $O/bench_${m}_dp${n}r.out 2> $O/bench_${m}_dp${n}r.log || { tail -30 $O/bench_${m}_dp${n}r.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${m}_dp${n}r.json'));print({k:d.get(k) for k in ('value','n_gpus','p50_latency_us','rows_scored','rows_expected','fraud_routed','flagged_handed_off','handoff_stalls')}, d['config'].get('parallelism'))"
  done
done
st done
