cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/lane
NO_TESTS=1 bash scripts/gpu_lane_diag.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/lane/bench_default.log 2>&1 || { tail -5 gpurun_out/lane/bench_default.log; exit 1; }
tail -1 gpurun_out/lane/bench_default.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('DEFAULT', d['value'], d['kernel'], d['config']['batches_in_flight'], d['launch_ms'], d['two_wave'], d['roofline']['frac'], d['roofline'].get('node_frac'), d['cpu_baseline']['value'] if d['cpu_baseline'] else None, d['vs_cpu'])"
