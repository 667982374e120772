#!/usr/bin/env bash
# Round-5 pass N: regression of the tree after the round-5 work (persist_dev ABI grew per-XCD
# counters; experiment-only blocks in the kernels; replicated kafka-lite): the whole GPU suite,
# smoke, config 2 as the driver runs it, config 4 default and at grid 257 x depth 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/${R5N_OUT:-r5n}; mkdir -p $O; export TMPDIR=/tmp
st() { echo "[r5n] $(date +%T) $*"; }
st pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
st smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
st bench
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp.json 2> $O/bench_mlp.log || { tail -30 $O/bench_mlp.log; exit 1; }
timeout -k 10 300 python bench.py --model gbdt --steps 20 --warmup 5 > $O/bench_gbdt.json 2> $O/bench_gbdt.log || { tail -30 $O/bench_gbdt.log; exit 1; }
timeout -k 10 300 python bench.py --model gbdt --steps 20 --warmup 5 --persist-grid 257 --depth 8 > $O/bench_gbdt_g257_d8.json 2> $O/bench_gbdt_g257_d8.log || { tail -30 $O/bench_gbdt_g257_d8.log; exit 1; }
python - $O <<'PY'
import json, sys
for n in ("mlp", "gbdt", "gbdt_g257_d8"):
    d = json.load(open(f"{sys.argv[1]}/bench_{n}.json"))
    p = d["precision_vs_fp32"]
    print(n, d["value"], d["p50_latency_us"], d["p99_latency_us"], "flips", p["route_flips"], p["route_flips_outside_1e-2_band"],
          "ceiling", d["h2d_zerocopy_ceiling_tx_s_rank0"], "diag", d.get("diagnostic"), d["config"]["parallelism"])
PY
st done
