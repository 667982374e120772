set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r85; mkdir -p $O
for cfg in "inproc txb1 6" "kafka-lite txb1 6" "inproc json 8"; do
  set -- $cfg
  timeout -k 10 200 python bench/e2e.py --broker $1 --fmt $2 --seconds $3 --out $O/e2e_$1_$2.json > $O/e2e_$1_$2.log 2>&1 || { tail -30 $O/e2e_$1_$2.log; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e_$1_$2.json')); print('$1 $2', d['value'], d['ring_arrival_to_scored_p50_us'], d['prometheus_transaction_incoming_total_rank0']==d['rows_scored_rank0_total'])"
done
