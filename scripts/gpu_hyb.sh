cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 scripts/bench_configs.py c4 c1 > gpurun_out/hyb.jsonl 2> gpurun_out/hyb.err || { tail -5 gpurun_out/hyb.err; exit 1; }
cat gpurun_out/hyb.jsonl
