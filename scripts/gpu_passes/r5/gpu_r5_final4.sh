#!/usr/bin/env bash
# Round-5 final pass 4: the libraries rebuilt after the pass-AF revert -- GPU suite,
# smoke, config 2 once and config 4 three times as the driver runs them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5final4; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r5final4] $(date +%T) $*"; }
st pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
st smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
st bench
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp.json 2> $O/bench_mlp.log || { tail -30 $O/bench_mlp.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model gbdt --steps 20 --warmup 5 > $O/bench_gbdt_$i.json 2> $O/bench_gbdt_$i.log || { tail -30 $O/bench_gbdt_$i.log; exit 1; }
done
python - $O <<'PY'
import json, sys
for n in ("mlp", "gbdt_1", "gbdt_2", "gbdt_3"):
    d = json.load(open(f"{sys.argv[1]}/bench_{n}.json"))
    p = d["precision_vs_fp32"]
    print(n, d["value"], d["p50_latency_us"], d["p99_latency_us"], "flips", p["route_flips_outside_1e-2_band"],
          "rows_ok", d["rows_scored"] == d["rows_expected"], "ceiling", d["h2d_zerocopy_ceiling_tx_s_rank0"])
PY
st done
