cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/d3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dsd or c5 or format" > gpurun_out/d3/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/d3/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 scripts/bench_configs.py dsd3 dsd1 c5 --inflight 3 > gpurun_out/d3/rates.jsonl 2> gpurun_out/d3/rates.err; rc=$?
echo "rates rc=$rc"; cut -c1-400 gpurun_out/d3/rates.jsonl; exit $rc
