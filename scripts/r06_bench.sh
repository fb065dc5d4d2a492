# round 6: the driver's default bench line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
s=$(date +%s)
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $G/bench.log 2>&1 || { tail -20 $G/bench.log; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
tail -1 $G/bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
p = d['pcie_inclusive']
print('bench', d['value'], 'alone', d['launch_ms']['alone'], 'in-flight', d['launch_ms']['in_flight_mean'], 'verified', d['verified']['redo_blocks'], d['verified']['pcm_equal'])
print('pcie', p['value'], 'pipelined', p['pipelined'], p['pipelined_pcm'], 'server', p['pipelined_pcm_2buf'])
print('roofline', json.dumps(d['roofline'])[:300]); print('cpu', json.dumps(d['cpu_baseline'])[:300])"
