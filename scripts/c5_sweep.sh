# C5 at 20 batches in flight by streams per decode (WVG_LANES; "auto": the library's
# in-flight policy) and hardware queues -> gpurun_out/c5s/
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/c5s
for q in ${QUEUES:-24}; do for l in ${LANESET:-auto 1 2 11}; do
  if [ $l = auto ]; then unset WVG_LANES; else export WVG_LANES=$l; fi
  WVG_BENCH_HW_QUEUES=$q timeout -k 10 120 python3 scripts/bench_configs.py ${CFG:-c5} --kernel lane --inflight 20 > gpurun_out/c5s/q${q}_l${l}.json 2> gpurun_out/c5s/q${q}_l${l}.err || { echo "q=$q l=$l failed"; tail -3 gpurun_out/c5s/q${q}_l${l}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5s/q${q}_l${l}.json').read().strip().splitlines()[-1]); print('q=$q l=$l', d['kernel_ms'], d['Mframes_per_s_inflight'], d['crc_errors'], d.get('group_end_ms'))"
done; done
