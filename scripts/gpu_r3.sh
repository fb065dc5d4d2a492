# Round-3 GPU check in one call: GPU parity, then A/B of two builds (C2 bench +
# per-config rates), the device-framing phase trace and the issue microbenchmarks.
# LIBS / CFGS as in gpu_ab_cfg.sh.  Stops at the first failing GPU step.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3
LIBS=${LIBS:-"build/libwvgpu.so"}
CFGS=${CFGS:-"dsd3 dsd0 dsd1 c4 c5"}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "^FAILED|^ERROR" gpurun_out/r3/pytest.log | head -20; tail -2 gpurun_out/r3/pytest.log
  # assertion failures (rc 1) still let the measurements run; anything that looks like a
  # device fault, a crash or a timeout stops here
  if [ $rc -ne 0 ]; then
    if [ $rc -ne 1 ] || grep -qiE "hipError|HSA_STATUS|memory access fault|Aborted|Segmentation|Timeout" gpurun_out/r3/pytest.log; then exit $rc; fi
  fi
fi
i=0
for L in $LIBS; do
  i=$((i+1))
  WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/r3/b$i.log 2>&1 || { tail -3 gpurun_out/r3/b$i.log; exit 1; }
  WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 600 python scripts/bench_configs.py $CFGS --inflight 3 > gpurun_out/r3/c$i.log 2>&1 || { tail -3 gpurun_out/r3/c$i.log; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/r3/b$i.log').read().strip().splitlines()[-1])
c=[json.loads(l) for l in open('gpurun_out/r3/c$i.log') if l.startswith('{')]
print('$L', 'C2', d['value'], d.get('value_one_batch_at_a_time'), d['launch_ms'], d['pcie_inclusive']['ms'], d['pcie_inclusive']['device_framing']['ms'])
for x in c: print('   ', x['config'][:24], x['kernel_ms'], x['Mframes_per_s'], x.get('Mframes_per_s_inflight'), x.get('group_end_ms'))"
done
if [ -z "$NO_EXTRA" ]; then
  WVG_DFRAME_TRACE=1 timeout -k 10 300 python scripts/dframe_time.py > gpurun_out/r3/dframe.log 2> gpurun_out/r3/dframe.err || { tail -3 gpurun_out/r3/dframe.err; exit 1; }
  cat gpurun_out/r3/dframe.log; tail -8 gpurun_out/r3/dframe.err
  timeout -k 10 120 ./scripts/micro/issue > gpurun_out/r3/issue.log 2>&1 || { tail -3 gpurun_out/r3/issue.log; exit 1; }
  grep "blocks=   1" gpurun_out/r3/issue.log
fi
exit 0
