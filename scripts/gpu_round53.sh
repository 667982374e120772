set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r53; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gbdt or strided" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="timeout -k 10 120 python bench/kernel_sol.py --sizes 65536,1048576,16777216"
CCFD_GBDT_R=1 $K --cases gbdt:f32 --tag gbdt_v2_r1 >> $O/sweep.jsonl 2>>$O/err.log || exit 1
CCFD_GBDT_R=2 $K --cases gbdt:f32 --tag gbdt_v2_r2 >> $O/sweep.jsonl 2>>$O/err.log || exit 1
cat $O/sweep.jsonl
B="timeout -k 10 200 python bench.py --model gbdt --batch 65536 --batches-per-step 16 --steps 20 --warmup 3 --depth 8 --no-unloaded-probe"
for v in v1 v2r1 v2r2; do
  case $v in v1) E="CCFD_GBDT_KERNEL=v1";; v2r1) E="CCFD_GBDT_R=1";; v2r2) E="CCFD_GBDT_R=2";; esac
  env $E $B > $O/bench_$v.log 2>&1 || { tail -30 $O/bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), 'Mtx/s p50', d['p50_latency_us'], 'devexec', d['device_exec_us_mean'])"
done
