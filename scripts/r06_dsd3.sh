# round 6: DSD mode-3 pair kernel -- its GPU tests, then the 1,024-block stereo batch alone and
# 20 in flight on the pair kernel and on the one-lane kernel (WVG_DSD3_PAIR=0)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsd_lane.py tests/test_gpu_c5.py -m gpu -x -q --timeout 300 --timeout-method thread > $G/t_dsd.log 2>&1 || { tail -30 $G/t_dsd.log; exit 1; }
tail -2 $G/t_dsd.log
timeout -k 10 300 python scripts/bench_configs.py dsd3 --dsd-files 1024 --kernel lane --inflight 20 > $G/dsd3_pair.jsonl 2> $G/dsd3_pair.err || { tail $G/dsd3_pair.err; exit 1; }
WVG_DSD3_PAIR=0 timeout -k 10 300 python scripts/bench_configs.py dsd3 --dsd-files 1024 --kernel lane --inflight 20 > $G/dsd3_one.jsonl 2> $G/dsd3_one.err || { tail $G/dsd3_one.err; exit 1; }
cut -c1-600 $G/dsd3_pair.jsonl $G/dsd3_one.jsonl
# the pipelined PCM request stream: T threads x D-deep rings
timeout -k 10 300 python scripts/pipe2_probe.py --threads 4,8,12 --depth 2,3 --rounds 6 --kernel auto > $G/pipe2.jsonl 2> $G/pipe2.err || { tail $G/pipe2.err; exit 1; }
cut -c1-300 $G/pipe2.jsonl
