set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r69; mkdir -p $O
for occ in 4 8; do for pf in 2 4 8; do
  CCFD_LR_OCC=$occ CCFD_LR_PF=$pf timeout -k 10 120 python bench/kernel_sol.py --cases lr:w64 --sizes 1048576,16777216 \
    --tag lr_occ${occ}_pf${pf} --out $O/lr_sweep.jsonl > $O/lr_${occ}_${pf}.log 2>&1 || { tail -30 $O/lr_${occ}_${pf}.log; exit 1; }
done; done
cut -c1-220 $O/lr_sweep.jsonl
