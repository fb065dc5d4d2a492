# A/B of the kernel choice on one config at 20 in flight (CFG, KERNELS) -> gpurun_out/ab/
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
for k in ${KERNELS:-lane auto}; do
  timeout -k 10 200 python3 scripts/bench_configs.py ${CFG:-c4} --kernel $k --inflight 20 > gpurun_out/ab/${CFG:-c4}_$k.json 2> gpurun_out/ab/${CFG:-c4}_$k.err || { tail -3 gpurun_out/ab/${CFG:-c4}_$k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/${CFG:-c4}_$k.json').read().strip().splitlines()[-1]); print('$k', d['kernel_ms'], d['Mframes_per_s_inflight'])"
done
