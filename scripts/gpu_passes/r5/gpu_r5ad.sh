#!/usr/bin/env bash
# Round-5 pass AD: rocprofv3 kernel trace + stats of config 2 (MLP, W64 rows) and config 4 (GBDT,
# G20 rows) on the final tree, persistent kernels, as the driver runs them.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
O=$R/gpurun_out/r5ad; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
st() { echo "[r5ad] $(date +%T) $*"; }
st mlp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mlp -o mlp -- python3 $R/bench.py --steps 5 --warmup 2 \
    > $O/bench_mlp.json 2> $O/mlp.log || { tail -30 $O/mlp.log; exit 1; }
st gbdt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gbdt -o gbdt -- python3 $R/bench.py --model gbdt --steps 5 --warmup 2 \
    > $O/bench_gbdt.json 2> $O/gbdt.log || { tail -30 $O/gbdt.log; exit 1; }
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -8 "$f" | cut -c1-220; done
find $O -name "*.db" -size +20M -delete
st done
