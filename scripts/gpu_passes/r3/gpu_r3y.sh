#!/bin/bash
# Round-3 GPU pass Y: GBDT 100x6 on G20 rows, persistent-kernel operating sweep on the final
# tree (item rows x chunk ring vs whole item in flight x grid x depth), 3 s timed regions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
summ() { python3 -c "import json; d=json.load(open('$1')); r=d['per_rank'][0]; print('$1', '%.4g' % d['value'], 'p50', d['p50_latency_us'], 'p99', d.get('p99_latency_us'), 'h2d', r.get('h2d_zerocopy_GBps'))"; }
run() {   # tag, env..., -- bench args
  local tag=$1; shift
  echo "[r3y] $(date +%T) $tag"
  env "$@" timeout -k 10 200 python bench.py --model gbdt --min-timed-s 3 --out $O/$tag.json > $O/$tag.log 2>&1 || { tail -30 $O/$tag.log; exit 1; }
  summ $O/$tag.json
}
run base             CCFD_G32_INFLIGHT=0
run inflight512      CCFD_G32_INFLIGHT=1
run ring1024         CCFD_G32_INFLIGHT=0 CCFD_PERSIST_ITEM_ROWS=1024
run inflight1024     CCFD_G32_INFLIGHT=1 CCFD_PERSIST_ITEM_ROWS=1024
run ring256          CCFD_G32_INFLIGHT=0 CCFD_PERSIST_ITEM_ROWS=256
run base_again       CCFD_G32_INFLIGHT=0
for g in 128 256 320; do
  echo "[r3y] $(date +%T) grid $g"
  timeout -k 10 200 python bench.py --model gbdt --min-timed-s 3 --persist-grid $g --out $O/grid$g.json > $O/grid$g.log 2>&1 || { tail -30 $O/grid$g.log; exit 1; }
  summ $O/grid$g.json
done
for d in 3 5 6; do
  echo "[r3y] $(date +%T) depth $d"
  timeout -k 10 200 python bench.py --model gbdt --min-timed-s 3 --depth $d --out $O/depth$d.json > $O/depth$d.log 2>&1 || { tail -30 $O/depth$d.log; exit 1; }
  summ $O/depth$d.json
done
echo "[r3y] done"
