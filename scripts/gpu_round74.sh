set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r74; mkdir -p $O
timeout -k 10 200 python bench/e2e.py --broker inproc --fmt json --seconds 10 --out $O/e2e_inproc_json.json > $O/e2e_inproc_json.log 2>&1 || { tail -30 $O/e2e_inproc_json.log; exit 1; }
tail -1 $O/e2e_inproc_json.log | cut -c1-600
timeout -k 10 200 python bench/e2e.py --broker kafka-lite --fmt json --seconds 10 --out $O/e2e_kafka_json.json > $O/e2e_kafka_json.log 2>&1 || { tail -30 $O/e2e_kafka_json.log; exit 1; }
tail -1 $O/e2e_kafka_json.log | cut -c1-600
