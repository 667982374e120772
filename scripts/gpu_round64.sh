set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r64; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench/rest_native.py --model mlp --conns 1,16,64,256 --seconds 4 --out $O/rest_native_gpu_mlp.json > $O/rest.log 2>&1 || { tail -30 $O/rest.log; exit 1; }
cat $O/rest.log
timeout -k 10 200 python bench/rest_native.py --model lr --device cpu --conns 1,16,64 --seconds 3 --out $O/rest_native_cpu_lr.json > $O/rest_cpu.log 2>&1 || { tail -30 $O/rest_cpu.log; exit 1; }
cat $O/rest_cpu.log
