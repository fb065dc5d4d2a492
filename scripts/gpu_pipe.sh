cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "pipe or c3_full or corrupted" > gpurun_out/pytest_pipe.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_pipe.log
exit $rc
