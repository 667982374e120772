#!/bin/bash
# Round 4: config 3's launch path with 8 ranks, rehearsed on one GPU (gloo collectives, ranks
# share the card): python bench.py --gpus 8 --rehearsal -- the parent spawns the 8 ranks, rank
# 0 prints the line; the host-DRAM ceiling is aggregated per NUMA node.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
step() { echo "[r4s] $(date +%T) $*"; }
step bench dp8 rehearsal
timeout -k 10 600 python bench.py --gpus 8 --rehearsal --steps 10 --warmup 3 > $O/bench_dp8r.json 2> $O/bench_dp8r.log || { tail -40 $O/bench_dp8r.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_dp8r.json').read().strip().splitlines()[-1])
print(d['metric'], d['value'], d['n_gpus'], d['config'].get('parallelism'), d.get('rehearsal'), d.get('world_size'))
for k in ('host_numa_read_GBps', 'host_dram_ceiling_tx_s', 'host_node_probe_GBps'):
    print(k, d.get(k))
print([ (r.get('rank'), r.get('rows')) for r in d.get('per_rank', [])])"
step done
