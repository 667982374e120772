set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r49; mkdir -p $O
export TMPDIR=/tmp
K="timeout -k 10 120 python bench/kernel_sol.py"
for f in 0 16 32 48; do
  $K --cases mlp:w64,lr:w64 --sizes 1048576,16777216 --flags $f --tag ablate$f >> $O/sweep.jsonl 2>>$O/err.log || exit 1
done
for c in 1 4 16; do
  CCFD_GBDT_CPW=$c $K --cases gbdt:f32 --sizes 1048576,16777216 --tag gbdt_cpw$c >> $O/sweep.jsonl 2>>$O/err.log || exit 1
done
for t in 1 2 4; do
  CCFD_MLP_TPW=$t $K --cases mlp:w64,lr:w64 --sizes 1048576,16777216 --tag tpw$t >> $O/sweep.jsonl 2>>$O/err.log || exit 1
done
CCFD_MLP_WEIGHTS=global $K --cases mlp:w64 --sizes 1048576,16777216 --tag gweights >> $O/sweep.jsonl 2>>$O/err.log || exit 1
cat $O/sweep.jsonl
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d "$GRAFT_REPO_ROOT/$O/pmc1" -o run -- python3 "$GRAFT_REPO_ROOT/bench/kernel_sol.py" --cases mlp:w64 --sizes 16777216 --iters 2 > "$GRAFT_REPO_ROOT/$O/pmc1.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$O/pmc1.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --output-format csv -d "$GRAFT_REPO_ROOT/$O/pmc2" -o run -- python3 "$GRAFT_REPO_ROOT/bench/kernel_sol.py" --cases mlp:w64 --sizes 16777216 --iters 2 > "$GRAFT_REPO_ROOT/$O/pmc2.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$O/pmc2.log"; exit 1; }
ls -R "$GRAFT_REPO_ROOT/$O" | head
