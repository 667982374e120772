#!/bin/bash
# Round-3 GPU pass U (diagnostic): does the per-row output traffic (proba f32 + route u8 to
# host memory) cost link throughput?  Same-box A/B with CCFD_ABLATE=32 (no proba/route
# stores; timing only -- incomplete results by design).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
step() { echo "[r3u] $(date +%T) $*"; }
summ() { python3 -c "import json; d=json.load(open('$1')); r=d['per_rank'][0]; print('$1', '%.4g' % d['value'], 'p50', d['p50_latency_us'], 'h2d', r.get('h2d_zerocopy_GBps'), r.get('pci'))"; }
for m in mlp gbdt; do
  for i in 1 2; do
    step $m default $i
    timeout -k 10 300 python bench.py --model $m --min-timed-s 3 --out $O/${m}_def_$i.json > $O/${m}_def_$i.log 2>&1 || { tail -30 $O/${m}_def_$i.log; exit 1; }
    summ $O/${m}_def_$i.json
    step $m no-outputs $i
    CCFD_ABLATE=32 timeout -k 10 300 python bench.py --model $m --min-timed-s 3 --out $O/${m}_noout_$i.json > $O/${m}_noout_$i.log 2>&1 || { tail -30 $O/${m}_noout_$i.log; exit 1; }
    summ $O/${m}_noout_$i.json
  done
done
step done
