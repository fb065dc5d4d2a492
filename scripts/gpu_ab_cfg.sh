# GPU parity with the product build, then C2 (bench.py) and C4/C3 (bench_configs.py)
# rates for experiment builds: LIBS="build/base/libwvgpu.so build/libwvgpu.so"
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/abc
LIBS=${LIBS:-"build/libwvgpu.so"}
CFGS=${CFGS:-"c4"}
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/abc/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/abc/pytest.log
[ $rc -ne 0 ] && exit $rc
i=0
for rep in 1 2; do
  for L in $LIBS; do
    i=$((i+1))
    WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 300 python bench.py --steps 30 --warmup 4 --no-cpu > gpurun_out/abc/b$i.log 2>&1 || { tail -3 gpurun_out/abc/b$i.log; exit 1; }
    WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 300 python scripts/bench_configs.py $CFGS --inflight 3 > gpurun_out/abc/c$i.log 2>&1 || { tail -3 gpurun_out/abc/c$i.log; exit 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/abc/b$i.log').read().strip().splitlines()[-1])
c=[json.loads(l) for l in open('gpurun_out/abc/c$i.log') if l.startswith('{')]
print('$L', 'C2', d['value'], ' '.join('%s %s/%s' % (x['config'][:3], x['Mframes_per_s'], x.get('Mframes_per_s_inflight')) for x in c))"
  done
done
