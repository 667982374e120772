set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r75; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_service_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench/e2e.py --broker inproc --fmt json --seconds 10 --out $O/e2e_inproc_json.json > $O/e2e_inproc_json.log 2>&1 || { tail -30 $O/e2e_inproc_json.log; exit 1; }
tail -1 $O/e2e_inproc_json.log | cut -c1-700
timeout -k 10 200 python bench/e2e.py --broker inproc --seconds 6 --out $O/e2e_inproc_txb1.json > $O/e2e_inproc_txb1.log 2>&1 || { tail -30 $O/e2e_inproc_txb1.log; exit 1; }
tail -1 $O/e2e_inproc_txb1.log | cut -c1-300
