# round 6: the whole GPU suite, the driver's bench line, and the pipelined PCM stream probe
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $G/pytest.log 2>&1 || { tail -30 $G/pytest.log; exit 1; }
tail -2 $G/pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $G/bench.log 2>&1 || { tail -20 $G/bench.log; exit 1; }
tail -1 $G/bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('bench', d['value'], 'alone', d['launch_ms']['alone'], 'in-flight', d['launch_ms']['in_flight_mean'], 'verified', d.get('verified'))
print('pcie', json.dumps(d['pcie_inclusive'])[:600])"
