#!/bin/bash
# Round 4 final-tree profiles: rocprofv3 kernel stats of the config-2 and config-4 benches
# (the resident persistent kernel is one long dispatch; the table shows what else runs next to
# it), and the 4-rank deployed topology rehearsal (gloo on one GPU) with the round-4 services.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
step() { echo "[r4l] $(date +%T) $*"; }
step rocprof mlp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python3 bench.py --steps 10 --warmup 3 --out $O/bench_mlp_traced.json > $O/prof_mlp.log 2>&1 || { tail -30 $O/prof_mlp.log; exit 1; }
find $O/prof_mlp -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -6 {} | cut -c1-200'
step rocprof gbdt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt -o gbdt -- python3 bench.py --model gbdt --steps 10 --warmup 3 --out $O/bench_gbdt_traced.json > $O/prof_gbdt.log 2>&1 || { tail -30 $O/prof_gbdt.log; exit 1; }
find $O/prof_gbdt -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -6 {} | cut -c1-200'
step deployed topology, 4 ranks rehearsal, JSON
timeout -k 30 400 python bench/deploy_topology.py --ranks 4 --rehearsal --seconds 20 --producers 3 --rate 600000 --fmt json \
  --log-dir $O/topo4 --out $O/topo4_json.json > $O/topo4_json.log 2>&1 || { tail -40 $O/topo4_json.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/topo4_json.json'))
print(d['value'], d['checks_passed'], d['partition_owners'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'])
print(d['produce_to_scored_us']); print(d['scored_to_process_started_us']); print(d['reference_dashboards']['matched'], '/', d['reference_dashboards']['selectors'])"
step done
