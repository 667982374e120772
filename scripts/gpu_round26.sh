set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
e2e() { name=$1; shift; timeout -k 10 120 python bench/e2e.py --seconds 6 --warmup 2 "$@" --out gpurun_out/e2e_$name.json > gpurun_out/e2e_$name.log 2>&1 || { tail -30 gpurun_out/e2e_$name.log; exit 1; }; python -c "import json; d=json.load(open('gpurun_out/e2e_$name.json')); print('$name', round(d['value']/1e6,3), d['ring_arrival_to_scored_p50_us'], d['ring_arrival_to_scored_p99_us'])"; }
e2e r1e4_f100 --rate 10000 --batch 256 --flush-us 100
e2e r1e5_f100 --rate 100000 --batch 1024 --flush-us 100
e2e r1e6_f100 --rate 1000000 --batch 4096 --flush-us 100
e2e r1e6_f500 --rate 1000000 --batch 4096 --flush-us 500
e2e r1e7 --rate 10000000 --batch 4096 --flush-us 100
