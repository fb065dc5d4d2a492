cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for n in 1 2 3 4 6; do
  timeout -k 10 300 python bench.py --steps 24 --warmup 4 --inflight $n --no-cpu > gpurun_out/bench_if$n.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_if$n.log').read().strip().splitlines()[-1]); print($n, d['value'], d['ms_per_step'], d['launch_ms'])"
done
