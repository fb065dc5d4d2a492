# Lane kernel GPU tests (mono included), C5 on both kernels, the DSD call/seek tests.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/lm
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_lane.py tests/test_gpu_c5.py tests/test_api_mirror.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lm/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^FAILED|^ERROR|Error" gpurun_out/lm/pytest.log | head -5; tail -3 gpurun_out/lm/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 scripts/bench_configs.py c5 c3 c1 --kernel lane --inflight 20 > gpurun_out/lm/rates.jsonl 2> gpurun_out/lm/rates.err; rc=$?
echo "rates rc=$rc"; cut -c1-420 gpurun_out/lm/rates.jsonl; exit $rc
