# GPU parity with the product build, then the bench line for experiment builds
# of the same source (WVG_LIB=<path>), e.g. compile-time constants:
#   LIBS="build/libwvgpu.so build/exp_s6/libwvgpu.so" bash scripts/gpu_variants.sh
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/var
LIBS=${LIBS:-"build/libwvgpu.so"}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/var/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 gpurun_out/var/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for rep in 1 2; do
  for L in $LIBS; do
    i=$((i+1))
    WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 300 python bench.py --steps 30 --warmup 4 --no-cpu ${BENCH_ARGS} > gpurun_out/var/b$i.log 2>&1 || { tail -3 gpurun_out/var/b$i.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/var/b$i.log').read().strip().splitlines()[-1]); print('$L', d['value'], d.get('value_one_batch_at_a_time'), d.get('launch_ms',{}).get('in_flight_mean'), d.get('launch_ms',{}).get('alone'), d['pcie_inclusive']['value'], d['pcie_inclusive'].get('pipelined'))"
  done
done
