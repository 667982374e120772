#!/usr/bin/env bash
# Round-6 pass M: rocprofv3 kernel trace + stats of configs 2 and 4 on the final harness
# (fraud hand-off on a collector thread beside the pump).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
O=$R/gpurun_out/r6m; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
st() { echo "[r6m] $(date +%T) $*"; }
st trace mlp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mlp -o mlp -- python3 $R/bench.py --steps 5 --warmup 2 \
    > $O/bench_mlp.json 2> $O/mlp.log || { tail -30 $O/mlp.log; exit 1; }
st trace gbdt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gbdt -o gbdt -- python3 $R/bench.py --model gbdt --steps 5 --warmup 2 \
    > $O/bench_gbdt.json 2> $O/gbdt.log || { tail -30 $O/gbdt.log; exit 1; }
find $O -name "*.db" -size +20M -delete
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -6 "$f" | cut -c1-220; done
st done
