set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu33.log 2>&1 || { tail -40 gpurun_out/pytest_gpu33.log; exit 1; }
tail -1 gpurun_out/pytest_gpu33.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke33.log 2>&1 || { tail -20 gpurun_out/smoke33.log; exit 1; }
tail -1 gpurun_out/smoke33.log
timeout -k 10 300 python bench.py --out gpurun_out/bench33.json > gpurun_out/bench33.log 2>&1 || { tail -20 gpurun_out/bench33.log; exit 1; }
tail -1 gpurun_out/bench33.log
timeout -k 10 300 python bench.py --model lr --out gpurun_out/bench33_lr.json > gpurun_out/bench33_lr.log 2>&1 || { tail -20 gpurun_out/bench33_lr.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench33_lr.json')); print('lr', d['value'], d['p50_latency_us'])"
