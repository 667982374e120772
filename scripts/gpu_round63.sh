set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r63; mkdir -p $O
b() { name=$1; shift; timeout -k 10 300 python bench.py "$@" --out $O/bench_$name.json > $O/bench_$name.log 2>&1 || { tail -30 $O/bench_$name.log; exit 1; }; python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', round(d['value']/1e6,1), 'Mtx/s p50', d['p50_latency_us'], 'unloaded', d['p50_latency_us_unloaded'])"; }
b default
b lr --model lr
b gbdt --model gbdt --batch 65536 --batches-per-step 16 --depth 8 --coalesce 1
b mlp_f32 --wire f32
e2e() { name=$1; shift; timeout -k 10 150 python bench/e2e.py --seconds 6 --warmup 2 "$@" --out $O/e2e_$name.json > $O/e2e_$name.log 2>&1 || { tail -30 $O/e2e_$name.log; exit 1; }; python3 -c "import json; d=json.load(open('$O/e2e_$name.json')); print('e2e_$name', round(d['value']/1e6,3), 'Mtx/s p50', d['ring_arrival_to_scored_p50_us'], d['prometheus_transaction_incoming_total_rank0'] == d['rows_scored_rank0_total'])"; }
e2e inproc
e2e kafka --broker kafka-lite
