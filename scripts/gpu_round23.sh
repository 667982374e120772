set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu23.log 2>&1 || { tail -40 gpurun_out/pytest_gpu23.log; exit 1; }
tail -1 gpurun_out/pytest_gpu23.log
timeout -k 10 300 python bench.py --out gpurun_out/bench23.json > gpurun_out/bench23.log 2>&1 || { tail -20 gpurun_out/bench23.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench23.json')); print(round(d['value']/1e6,1), d['p50_latency_us'], d['device_exec_us_mean'], d['device_exec_us_p50'])"
timeout -k 10 200 python bench/baseline_cpu.py --seconds 10 --out gpurun_out/rest_cpu_lr.json > gpurun_out/rest_cpu.log 2>&1 || { tail -20 gpurun_out/rest_cpu.log; exit 1; }
timeout -k 10 200 python bench/baseline_cpu.py --seconds 10 --scorer gpu --model mlp --max-batch 4096 --max-delay-us 200 --pool 64 --out gpurun_out/rest_gpu_mlp.json > gpurun_out/rest_gpu.log 2>&1 || { tail -20 gpurun_out/rest_gpu.log; exit 1; }
cat gpurun_out/rest_cpu_lr.json gpurun_out/rest_gpu_mlp.json | cut -c1-160
