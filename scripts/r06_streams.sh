cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g/t_streams.log 2>&1; rc=$?; tail -15 gpurun_out/g/t_streams.log; exit $rc
