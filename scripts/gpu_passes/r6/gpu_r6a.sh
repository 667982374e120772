#!/usr/bin/env bash
# Round-6 pass A: lossless hand-off -- the new GPU tests, the engine / serving tests, then
# config 2 and config 4 benches with flagged_handed_off == fraud_routed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6a; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6a] $(date +%T) $*"; }
st pytest
timeout -k 10 600 python -u -m pytest tests/test_handoff_lossless_gpu.py tests/test_engine_gpu.py tests/test_serve_gpu.py \
  tests/test_gbdt_g20_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
st bench mlp
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp.json 2> $O/bench_mlp.log || { tail -30 $O/bench_mlp.log; exit 1; }
st bench gbdt
timeout -k 10 300 python bench.py --model gbdt --steps 20 --warmup 5 > $O/bench_gbdt.json 2> $O/bench_gbdt.log || { tail -30 $O/bench_gbdt.log; exit 1; }
python - $O <<'PY'
import json, sys
for n in ("mlp", "gbdt"):
    d = json.load(open(f"{sys.argv[1]}/bench_{n}.json"))
    p = d["precision_vs_fp32"]
    print(n, d["value"], d["p50_latency_us"], d["p99_latency_us"], "flips", p["route_flips_outside_1e-2_band"],
          "rows_ok", d["rows_scored"] == d["rows_expected"], "handed", d["flagged_handed_off"], "routed",
          d["fraud_routed"], "stalls", d["handoff_stalls"], "ceiling", d["h2d_zerocopy_ceiling_tx_s_rank0"])
PY
st done
