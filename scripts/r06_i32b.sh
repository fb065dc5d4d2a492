# round 6: int32 zeros-only lossless blocks on the lanes -- tests, then the kinds' rates
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 600 python -u -m pytest tests/test_gpu_hybrid_lane.py tests/test_gpu_layout_quirks.py tests/test_gpu_lane.py -m gpu -x -q --timeout 300 --timeout-method thread > $G/t_i32.log 2>&1 || { tail -30 $G/t_i32.log; exit 1; }
tail -1 $G/t_i32.log
timeout -k 10 300 python scripts/r06_i32_probe.py > $G/i32.log 2>&1 || { tail $G/i32.log; exit 1; }
tail -1 $G/i32.log
timeout -k 10 600 python scripts/bench_configs.py hykinds --kernel lane --inflight 20 --lists "lossless,int32" > $G/hykinds2.jsonl 2> $G/hykinds2.err || { tail $G/hykinds2.err; exit 1; }
cut -c1-420 $G/hykinds2.jsonl
