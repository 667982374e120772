set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu38.log 2>&1 || { tail -40 gpurun_out/pytest_gpu38.log; exit 1; }
tail -1 gpurun_out/pytest_gpu38.log
timeout -k 10 300 python bench.py --out gpurun_out/bench38.json > gpurun_out/bench38.log 2>&1 || { tail -20 gpurun_out/bench38.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench38.json')); print(round(d['value']/1e6,1), d['p50_latency_us'], d['p50_latency_us_unloaded'], d['device_exec_us_mean'], d['device_exec_us_p50'])"
