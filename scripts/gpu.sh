# One parameterised GPU runner (run through gpurun from the repo root):
#   gpurun --timeout 1200 -- 'STEPS="smoke tests bench" bash scripts/gpu.sh'
# STEPS (in order, the first failing GPU step ends the call):
#   smoke    __graft_entry__.smoke()
#   tests    pytest -m gpu (TESTS: files, default tests/; PYTEST_ARGS: extra args, e.g. -k)
#   bench    bench.py (BENCH_ARGS, default the driver's --steps 20 --warmup 5) -> gpurun_out/g/bench.log
#   ab       for each build in LIBS (paths under wavpackdecoder_amd/): bench.py --no-cpu and
#            bench_configs.py $CFGS, via WVG_LIB (A/B of experiment builds)
#   configs  bench_configs.py $CFGS --kernel $KERNEL --inflight $INFLIGHT -> gpurun_out/g/configs.jsonl
#   diag     scripts/lane_diag.py (the lane kernel's ST_REDO reasons, DIAG_ARGS) -> gpurun_out/g/diag.log
#   profile  scripts/profile.sh (rocprofv3 kernel trace + FETCH/WRITE passes of the bench, TAG)
#   pmc_sq   scripts/pmc_sq.sh (SQ instruction counters; PROG / ARGS, KSUB: kernel name substring)
#   micro    scripts/micro/issue.hip issue-cost microbenchmarks (built here, in gpurun_out/g)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
STEPS=${STEPS:-"smoke tests bench"}
G=gpurun_out/g
fail() { echo "$1 failed (rc=$2)"; tail -5 "$3"; exit "$2"; }
for step in $STEPS; do
  case $step in
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $G/smoke.log 2>&1 || fail smoke $? $G/smoke.log
    tail -1 $G/smoke.log ;;
  tests)
    timeout -k 10 1000 python -u -m pytest ${TESTS:-tests/} -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $G/pytest.log 2>&1 || fail tests $? $G/pytest.log
    tail -2 $G/pytest.log ;;
  bench)
    timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > $G/bench.log 2>&1 || fail bench $? $G/bench.log
    tail -1 $G/bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('bench', d['value'], 'alone', d['launch_ms']['alone'], 'in-flight', d['launch_ms']['in_flight_mean'],
      'one-at-a-time', d.get('value_one_batch_at_a_time'), 'verified', d.get('verified'))" ;;
  ab)
    i=0
    for L in ${LIBS:-build/libwvgpu.so}; do
      i=$((i+1))
      WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu ${AB_ARGS} > $G/ab_b$i.log 2>&1 || fail "ab bench $L" $? $G/ab_b$i.log
      if [ -n "$CFGS" ]; then
        WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 600 python scripts/bench_configs.py $CFGS --kernel ${KERNEL:-lane} --inflight ${INFLIGHT:-20} > $G/ab_c$i.jsonl 2> $G/ab_c$i.err || fail "ab configs $L" $? $G/ab_c$i.err
      fi
      python3 -c "
import json, os
d = json.loads(open('$G/ab_b$i.log').read().strip().splitlines()[-1])
print('$L', 'C2', d['value'], 'alone', d['launch_ms']['alone'], 'redo', d['verified']['redo_blocks'])
p = '$G/ab_c$i.jsonl'
for x in ([json.loads(l) for l in open(p) if l.startswith('{')] if os.path.exists(p) else []):
    print('   ', x['config'][:28], x.get('kernel_ms'), x.get('Mframes_per_s'), x.get('Mframes_per_s_inflight'))"
    done ;;
  configs)
    timeout -k 10 900 python scripts/bench_configs.py ${CFGS:-c1 c3 c4 c5} --kernel ${KERNEL:-lane} --inflight ${INFLIGHT:-20} > $G/configs.jsonl 2> $G/configs.err || fail configs $? $G/configs.err
    cut -c1-400 $G/configs.jsonl ;;
  diag)
    timeout -k 10 300 python scripts/lane_diag.py ${DIAG_ARGS} > $G/diag.log 2>&1 || fail diag $? $G/diag.log
    tail -20 $G/diag.log ;;
  profile)
    TAG=${TAG:-r04} bash scripts/profile.sh || exit 1 ;;
  pmc_sq)
    bash scripts/pmc_sq.sh > /dev/null || exit 1
    python3 scripts/pmc_sq_sum.py "${KSUB:-wv_pcm_lane<false, 0, 17, 17>}" > $G/pmc_sq.txt && cat $G/pmc_sq.txt ;;
  micro)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/micro/issue.hip -o $G/issue && timeout -k 10 120 $G/issue > $G/micro.log 2>&1 || fail micro $? $G/micro.log
    cat $G/micro.log ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
