#!/usr/bin/env bash
# Round-5 pass A: GPU suite + smoke after the ablation switches left the kernels; config 2 / 4
# benches as the driver runs them; config 4 with the pipelined static-item G20 kernel (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $O/bench_mlp.json > $O/bench_mlp.log 2>&1 || { tail -30 $O/bench_mlp.log; exit 1; }
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
CCFD_PERSIST_PIPE=1 timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt_pipe.json > $O/bench_gbdt_pipe.log 2>&1 || { tail -30 $O/bench_gbdt_pipe.log; exit 1; }
CCFD_PERSIST_PIPE=1 timeout -k 10 300 python bench.py --model gbdt --persist-grid 256 --out $O/bench_gbdt_pipe_g256.json > $O/bench_gbdt_pipe_g256.log 2>&1 || { tail -30 $O/bench_gbdt_pipe_g256.log; exit 1; }
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt_b.json > $O/bench_gbdt_b.log 2>&1 || { tail -30 $O/bench_gbdt_b.log; exit 1; }
python - <<'PY'
import json
for n in ("mlp", "gbdt", "gbdt_pipe", "gbdt_pipe_g256", "gbdt_b"):
    d = json.load(open(f"gpurun_out/r5a/bench_{n}.json"))
    p = d["precision_vs_fp32"]
    print(n, d["value"], d["p50_latency_us"], d["p99_latency_us"], "flips", p["route_flips"], p["route_flips_outside_1e-2_band"], "ceiling", d["h2d_zerocopy_ceiling_tx_s_rank0"])
PY
