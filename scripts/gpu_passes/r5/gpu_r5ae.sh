#!/usr/bin/env bash
# Round-5 pass AE: why config 4 measured 2.69e9 under rocprofv3 --kernel-trace (pass AD) against
# 2.56e9 without -- the same bench with and without the profiler, at --steps 5 and 20.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
O=$R/gpurun_out/r5ae; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
st() { echo "[r5ae] $(date +%T) $*"; }
show() { python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['p50_latency_us'], d['p99_latency_us'], round(d['value']/d['h2d_zerocopy_ceiling_tx_s_rank0'],4), d['ms_per_step'])"; }
b() {  # b <name> <steps> <warmup> [prof]
  st "$1"
  if [ "$4" = prof ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$1 -o $1 -- python3 $R/bench.py --model gbdt --steps $2 --warmup $3 \
        > $O/$1.json 2> $O/$1.log || { tail -20 $O/$1.log; exit 1; }
  else
    timeout -k 10 300 python3 $R/bench.py --model gbdt --steps $2 --warmup $3 > $O/$1.json 2> $O/$1.log || { tail -20 $O/$1.log; exit 1; }
  fi
  show $1
}
b plain_s20 20 5
b plain_s5 5 2
b prof_s5 5 2 prof
b prof_s20 20 5 prof
b plain_s20_b 20 5
find $O -name "*.db" -delete
st done
