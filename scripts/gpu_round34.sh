set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_engine_service_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/pytest_gpu34.log 2>&1 || { tail -40 gpurun_out/pytest_gpu34.log; exit 1; }
tail -1 gpurun_out/pytest_gpu34.log
e2e() { name=$1; shift; timeout -k 10 120 python bench/e2e.py --seconds 6 --warmup 2 "$@" --out gpurun_out/e2e_$name.json > gpurun_out/e2e_$name.log 2>&1 || { tail -30 gpurun_out/e2e_$name.log; exit 1; }; python -c "import json; d=json.load(open('gpurun_out/e2e_$name.json')); print('$name', round(d['value']/1e6,3), d['ring_arrival_to_scored_p50_us'], d['ring_arrival_to_scored_p99_us'], d['fraud_processes_started_rank0'], d['prometheus_transaction_incoming_total_rank0'] == d['rows_scored_rank0_total'], d['ingest'])"; }
e2e kafka_txb1_native --broker kafka-lite --flush-us 100
e2e kafka_txb1_python --broker kafka-lite --flush-us 100 --python-ingest
e2e kafka_json_native --broker kafka-lite --flush-us 100 --fmt json
e2e kafka_json_python --broker kafka-lite --flush-us 100 --fmt json --python-ingest
