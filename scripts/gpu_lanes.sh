# Stream / hardware-queue mapping A/B: C5 (single batch + 3 in flight) and C2 for
# combinations of WVG_LANES (streams per decode) and GPU_MAX_HW_QUEUES.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/lanes
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/lanes/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "^FAILED|^ERROR" gpurun_out/lanes/pytest.log | head -20; tail -2 gpurun_out/lanes/pytest.log
  if [ $rc -ne 0 ]; then
    if [ $rc -ne 1 ] || grep -qiE "hipError|HSA_STATUS|memory access fault|Aborted|Segmentation|Timeout" gpurun_out/lanes/pytest.log; then exit $rc; fi
  fi
fi
i=0
for combo in "11 4" "11 8" "11 16" "4 4" "4 8"; do
  set -- $combo
  i=$((i+1))
  WVG_LANES=$1 GPU_MAX_HW_QUEUES=$2 timeout -k 10 400 python scripts/bench_configs.py c5 dsd1 --inflight 3 > gpurun_out/lanes/c$i.log 2>&1 || { tail -3 gpurun_out/lanes/c$i.log; exit 1; }
  WVG_LANES=$1 GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/lanes/b$i.log 2>&1 || { tail -3 gpurun_out/lanes/b$i.log; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/lanes/b$i.log').read().strip().splitlines()[-1])
c=[json.loads(l) for l in open('gpurun_out/lanes/c$i.log') if l.startswith('{')]
print('lanes=$1 hwq=$2 C2', d['value'], d['launch_ms']['in_flight_mean'])
for x in c: print('   ', x['config'][:24], x['kernel_ms'], x['Mframes_per_s'], x.get('Mframes_per_s_inflight'), x.get('group_end_ms'))"
done
exit 0
