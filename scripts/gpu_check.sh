# GPU round check: smoke -> GPU parity tests -> bench; stops at the first fault.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"
if [ $rc -ne 0 ]; then tail -30 gpurun_out/smoke.log; exit $rc; fi
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q --maxfail=30 -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --check --cpu-reps 3 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
