#!/bin/bash
# Round-3 GPU pass R: global-address-space row loads / output stores (no FLAT instructions
# on the hot path) and the 16-byte G20 fetch.  Probe, GPU suite, benches, latency sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
step() { echo "[r3r] $(date +%T) $*"; }
step load-width probe
timeout -k 10 120 python bench/experiments/load_width_probe.py --out $O/load_width.jsonl > $O/load_width.log 2>&1 || { tail -20 $O/load_width.log; exit 1; }
cat $O/load_width.jsonl
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
summ() { python3 -c "import json; d=json.load(open('$1')); print('$1', '%.4g' % d['value'], 'p50', d['p50_latency_us'], 'p99', d.get('p99_latency_us'), 't', d['timed_region_s'])"; }
step bench mlp
timeout -k 10 300 python bench.py --out $O/bench_mlp.json > $O/bench_mlp.log 2>&1 || { tail -30 $O/bench_mlp.log; exit 1; }
summ $O/bench_mlp.json
step bench gbdt x4 fetch
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt_x4.json > $O/bench_gbdt_x4.log 2>&1 || { tail -30 $O/bench_gbdt_x4.log; exit 1; }
summ $O/bench_gbdt_x4.json
step bench gbdt dword fetch
CCFD_G20_FETCH_DWORD=1 timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt_dw.json > $O/bench_gbdt_dw.log 2>&1 || { tail -30 $O/bench_gbdt_dw.log; exit 1; }
summ $O/bench_gbdt_dw.json
step latency sweep claimed
timeout -k 10 300 python bench/experiments/latency_breakdown.py --pipe 0 --items 128,256,512 --grids 64,128 --depths 1,4,8,12 --batches 3000 --out $O/lat_claimed.jsonl > $O/lat_claimed.log 2>&1 || { tail -20 $O/lat_claimed.log; exit 1; }
step latency sweep pipelined
timeout -k 10 300 python bench/experiments/latency_breakdown.py --pipe 1 --items 64,128 --grids 128,256 --depths 1,4,8,12 --batches 3000 --out $O/lat_pipe.jsonl > $O/lat_pipe.log 2>&1 || { tail -20 $O/lat_pipe.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r3r/lat_claimed.jsonl", "gpurun_out/r3r/lat_pipe.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(f.split("_")[-1][:5], d["item_rows"], d["grid"], "depth", d["depth"], "tx %.3g" % d["tx_s"],
              "p50", d["p50_total_us"], "dev", d["p50_dev_exec_us"], "out", d["p50_outside_us"])
PY
step done
