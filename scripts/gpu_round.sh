# GPU check + experiments in one call: smoke -> GPU parity -> bench -> placement probe.
# Stops at the first failing GPU step (no retries).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
B=$PWD/wavpackdecoder_amd/build
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --check --cpu-reps 3 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$EXPS" ]; then
  WVG_LIB=$B/exp5/libwvgpu.so timeout -k 10 200 python scripts/exp_place.py 1024 > gpurun_out/exp5.log 2>&1; rc=$?
  echo "exp5 rc=$rc"; grep -v Warn gpurun_out/exp5.log
  [ $rc -ne 0 ] && exit $rc
  WVG_PROF=4 WVG_LIB=$B/exp4/libwvgpu.so timeout -k 10 200 python scripts/exp_time.py 1024 > gpurun_out/exp4.log 2>&1; rc=$?
  echo "exp4 rc=$rc"; grep -v Warn gpurun_out/exp4.log
fi
exit $rc
