# Lane-per-block kernel check: GPU parity with WVG_LANE_KERNEL=1, then C2 at several
# batches-in-flight depths for the lane and the two-wave kernel.  Stops at the
# first failing GPU step.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/lane
if [ -z "$NO_TESTS" ]; then
  WVG_LANE_KERNEL=1 timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/lane/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/lane/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CFGS:-1:3 1:8 1:16 0:3}; do
  lk=${cfg%%:*}; inf=${cfg##*:}
  WVG_LANE_KERNEL=$lk timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu --inflight $inf --check > gpurun_out/lane/b_${lk}_${inf}.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/lane/b_${lk}_${inf}.log; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/lane/b_${lk}_${inf}.log').read().strip().splitlines()[-1])
print('lane=$lk inflight=$inf', d['value'], d.get('value_one_batch_at_a_time'), d['launch_ms'], d['ms_per_step'])"
done
exit 0
