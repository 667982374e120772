#!/bin/bash
# Round-3 GPU pass G: the deployed topology with TXB1 batches (the hot-path wire format),
# MLP and GBDT (G20 binned at ingest), open loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
step() { echo "[r3g] $(date +%T) $*"; }
step deploy topology mlp txb1 open loop 30 s
timeout -k 30 360 python bench/deploy_topology.py --seconds 30 --producers 4 --rate 0 --fmt txb1 \
    --log-dir $O/topo_txb1_mlp --out $O/topo_txb1_mlp.json > $O/topo_txb1_mlp.log 2>&1 || { tail -40 $O/topo_txb1_mlp.log; exit 1; }
tail -c 1500 $O/topo_txb1_mlp.json
step deploy topology gbdt txb1 open loop 30 s
timeout -k 30 360 python bench/deploy_topology.py --model gbdt --seconds 30 --producers 4 --rate 0 --fmt txb1 \
    --log-dir $O/topo_txb1_gbdt --out $O/topo_txb1_gbdt.json > $O/topo_txb1_gbdt.log 2>&1 || { tail -40 $O/topo_txb1_gbdt.log; exit 1; }
tail -c 1500 $O/topo_txb1_gbdt.json
step deploy topology with KIE crash + journal restart
timeout -k 30 420 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1200000 --fmt json \
    --kie-outage-at 20 --kie-outage-s 5 --log-dir $O/topo_kie_crash --out $O/topo_kie_crash.json > $O/topo_kie_crash.log 2>&1 \
    || { tail -40 $O/topo_kie_crash.log; exit 1; }
tail -c 600 $O/topo_kie_crash.json
step bench default
timeout -k 10 300 python bench.py --out $O/bench_default.json > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
step encoder microbench, AVX-512 16-row G20 path vs AVX2 on the box host
timeout -k 10 300 python bench/encode_bench.py --rows 2000000 --threads 8 --out $O/encode_g20.json > $O/encode.log 2>&1 || { tail -30 $O/encode.log; exit 1; }
cat $O/encode_g20.json
step bench gbdt
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
du -sh gpurun_out
step done
