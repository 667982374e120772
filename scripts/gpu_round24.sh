set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python bench/e2e.py --seconds 10 --warmup 3 --out gpurun_out/e2e_inproc.json > gpurun_out/e2e_inproc.log 2>&1 || { tail -30 gpurun_out/e2e_inproc.log; exit 1; }
cat gpurun_out/e2e_inproc.json
timeout -k 10 200 python bench/e2e.py --seconds 10 --warmup 3 --broker kafka-lite --out gpurun_out/e2e_kafka.json > gpurun_out/e2e_kafka.log 2>&1 || { tail -30 gpurun_out/e2e_kafka.log; exit 1; }
cat gpurun_out/e2e_kafka.json
