#!/bin/bash
# Round-3 GPU pass B: the full GPU suite (exec_mode auto = persistent is now the engine
# service default; persistent EngineService + KIE outage test), kernel-traced X2 run with
# the one-rank RCCL kernel probe, default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
step() { echo "[r3b] $(date +%T) $*"; }
step pytest
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step x2 traced
CCFD_FORCE_PG=1 CCFD_X2_ONE_RANK_KERNEL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x2 -o x2 -- python3 bench.py --out $O/bench_x2_traced.json > $O/x2.log 2>&1 || { tail -30 $O/x2.log; exit 1; }
python bench/x2_overlap.py $O/x2 > $O/x2_overlap.json 2>&1 || true
step bench default
timeout -k 10 300 python bench.py --out $O/bench_default.json > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
step done
