set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu27.log 2>&1 || { tail -40 gpurun_out/pytest_gpu27.log; exit 1; }
tail -1 gpurun_out/pytest_gpu27.log
e2e() { name=$1; shift; timeout -k 10 120 python bench/e2e.py --seconds 6 --warmup 2 "$@" --out gpurun_out/e2e_$name.json > gpurun_out/e2e_$name.log 2>&1 || { tail -30 gpurun_out/e2e_$name.log; exit 1; }; python -c "import json; d=json.load(open('gpurun_out/e2e_$name.json')); print('$name', round(d['value']/1e6,3), d['ring_arrival_to_scored_p50_us'], d['ring_arrival_to_scored_p99_us'], d['fraud_processes_started_rank0'], d['prometheus_transaction_incoming_total_rank0'] == d['rows_scored_rank0_total'])"; }
e2e r1e4 --rate 10000 --batch 256 --flush-us 100
e2e r1e5 --rate 100000 --batch 1024 --flush-us 100
e2e r1e6 --rate 1000000 --batch 4096 --flush-us 100
e2e max_inproc --flush-us 100
e2e max_kafka --broker kafka-lite --flush-us 100
