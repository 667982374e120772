set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r59; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="timeout -k 10 120 python bench/kernel_sol.py --cases mlp:w64"
$K --tag l3mfma >> $O/sweep.jsonl 2>>$O/err.log || exit 1
cat $O/sweep.jsonl
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
python3 -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print({k: d[k] for k in ('p50_latency_us','p99_latency_us','p50_latency_us_unloaded','device_exec_us_mean')})"
