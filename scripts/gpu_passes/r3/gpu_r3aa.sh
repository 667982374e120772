#!/bin/bash
# Round-3 GPU pass AA: the pipelined (latency-mode) persistent kernel with the 4-byte-lane +
# DPP-transpose fetch (compile-time CCFD_PIPE_FETCH_Q4, _native/ab/pipeq4.so) vs the default:
# exactness, then the light-load latency sweep, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3aa
mkdir -p $O
V=$PWD/ccfd_demo_summit_amd/_native/ab/pipeq4.so
step() { echo "[r3aa] $(date +%T) $*"; }
step pytest pipeq4 exactness
CCFD_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_rules_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "persistent" > $O/pytest_pipeq4.log 2>&1 || { tail -40 $O/pytest_pipeq4.log; exit 1; }
tail -1 $O/pytest_pipeq4.log
for v in def q4 def2 q42; do
  step latency $v
  if [ ${v:0:2} = q4 ]; then export CCFD_LIB_PATH=$V; else unset CCFD_LIB_PATH; fi
  timeout -k 10 300 python bench/experiments/latency_breakdown.py --pipe 1 --items 64,128 --grids 128,256 --depths 1,2,4,8 --batches 3000 --out $O/lat_$v.jsonl > $O/lat_$v.log 2>&1 || { tail -20 $O/lat_$v.log; exit 1; }
done
unset CCFD_LIB_PATH
python3 - <<'PY'
import json
rows = {}
for v in ("def", "q4", "def2", "q42"):
    for l in open(f"gpurun_out/r3aa/lat_{v}.jsonl"):
        d = json.loads(l)
        rows.setdefault((d["item_rows"], d["grid"], d["depth"]), {})[v] = (d["tx_s"], d["p50_total_us"])
for k, r in sorted(rows.items(), key=lambda x: str(x[0])):
    print(k, "  ".join(f"{v}: {r[v][0]:.3g} @ {r[v][1]} us" for v in ("def", "q4", "def2", "q42") if v in r))
PY
step done
