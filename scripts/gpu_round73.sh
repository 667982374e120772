set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r73; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in 4 8; do
  timeout -k 10 200 python bench/rest_native.py --model mlp --conns 64,256,1024 --seconds 3 --workers $w --out $O/rest_native_gpu_mlp_w$w.json > $O/rest_w$w.log 2>&1 || { tail -30 $O/rest_w$w.log; exit 1; }
  echo "workers=$w"; grep req_per_s $O/rest_w$w.log
done
