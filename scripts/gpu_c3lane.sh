# Lane kernel on the 16-term list: its GPU tests, then C3 on both kernels.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/c3l
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c3l/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/c3l/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 scripts/bench_configs.py c3 --kernel lane --inflight 20 > gpurun_out/c3l/rates.jsonl 2> gpurun_out/c3l/rates.err; rc=$?
echo "rates rc=$rc"; cut -c1-500 gpurun_out/c3l/rates.jsonl; tail -3 gpurun_out/c3l/rates.err; exit $rc
