#!/bin/bash
# Round 4: config 4 in launch mode (one launch per 65536-row G20 micro-batch over 4 streams)
# against the persistent default -- the launch-mode kernel streams 94.7 % of the link at 16 M
# rows per launch (profiles/r4/g20/), the persistent one 87 %.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
step() { echo "[r4k] $(date +%T) $*"; }
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g tx/s' % d['value'], 'p50', d['p50_latency_us'], 'p99', d['p99_latency_us'], d['config'].get('exec_mode'), d['config'].get('depth'), d['config'].get('streams'))" "$1" "$2"; }
for cfg in "persistent 4 4" "launch 4 4" "launch 8 4" "launch 16 8" "launch 32 8"; do
  set -- $cfg
  step gbdt $1 depth $2 streams $3
  timeout -k 10 300 python bench.py --model gbdt --exec-mode $1 --depth $2 --streams $3 --no-f32-probe \
    --out $O/gbdt_$1_d$2_s$3.json > $O/gbdt_$1_d$2_s$3.log 2>&1 || { tail -30 $O/gbdt_$1_d$2_s$3.log; exit 1; }
  summ $O/gbdt_$1_d$2_s$3.json $1_d$2_s$3
done
step done
