# Measurement builds: parser-only C2 (no-op reconstruction) and DSD mode 1 on the
# host framing's tables, against the product build.  Not part of the test suite.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/exp
export GPU_MAX_HW_QUEUES=16
for L in build/libwvgpu.so build/varN/libwvgpu.so; do
  WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/exp/b.log 2>&1 || { tail -3 gpurun_out/exp/b.log; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/exp/b.log').read().strip().splitlines()[-1])
print('$L C2', d['value'], d.get('value_one_batch_at_a_time'), d['launch_ms']['in_flight_mean'], d['launch_ms']['alone'])"
done
for L in build/libwvgpu.so build/varT/libwvgpu.so; do
  WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 300 python scripts/bench_configs.py dsd1 --inflight 3 > gpurun_out/exp/c.log 2>&1 || { tail -3 gpurun_out/exp/c.log; exit 1; }
  echo "$L"; cat gpurun_out/exp/c.log
done
exit 0
