#!/bin/bash
# Round-3 GPU pass O: same-box A/B of the LDS-staged flag list (flags 0) vs per-ballot
# reservation (flags 1024 = CCFD_ARG_FLAG_DIRECT), alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
for rep in 1 2; do
  for fl in 0 1024; do
    echo "[r3o] $(date +%T) rep $rep flags $fl"
    timeout -k 10 200 python bench/kernel_sol.py --cases mlp:w64,lr:w64 --sizes 1048576,16777216 --flags $fl --tag "ab$rep" >> $O/ab.jsonl 2>>$O/ab.err || { tail -20 $O/ab.err; exit 1; }
  done
done
cat $O/ab.jsonl
