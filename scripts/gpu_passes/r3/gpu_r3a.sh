#!/bin/bash
# Round-3 GPU pass A: GPU tests, default bench (5 s timed), X2 on/off A/B, RCCL one-rank probe,
# kernel-traced X2 overlap run, GBDT bench.  Every GPU step has its own time limit; the
# first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
step() { echo "[r3a] $(date +%T) $*"; }
step pytest
timeout -k 10 300 python -u -m pytest tests/test_watchdog.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step bench default
timeout -k 10 300 python bench.py --out $O/bench_default.json > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
step bench x2 off
timeout -k 10 300 python bench.py --x2-every 1000000000 --out $O/bench_x2off.json > $O/bench_x2off.log 2>&1 || { tail -30 $O/bench_x2off.log; exit 1; }
step rccl one-rank probe
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rccl1 -o probe -- python3 scripts/rccl_one_rank_probe.py > $O/rccl1.log 2>&1 || { tail -30 $O/rccl1.log; exit 1; }
step x2 traced
CCFD_FORCE_PG=1 CCFD_X2_ONE_RANK_KERNEL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x2 -o x2 -- python3 bench.py --out $O/bench_x2_traced.json > $O/x2.log 2>&1 || { tail -30 $O/x2.log; exit 1; }
python bench/x2_overlap.py $O/x2 > $O/x2_overlap.json 2>&1 || true
step bench gbdt
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
step encode bench
timeout -k 10 300 python bench/encode_bench.py --rows 2000000 --threads 8 --out $O/encode_g20.json > $O/encode.log 2>&1
timeout -k 10 300 python bench/encode_bench.py --rows 2000000 --threads 8 --trained --out $O/encode_g20_trained.json >> $O/encode.log 2>&1
step done
