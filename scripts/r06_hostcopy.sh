# round 6: parallel blob copy in wvg_batch_add_files -- C2 pipelined stream and the C5 end-to-end leg
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -m gpu -x -q --timeout 300 --timeout-method thread > $G/t_hc.log 2>&1 || { tail -30 $G/t_hc.log; exit 1; }
tail -1 $G/t_hc.log
timeout -k 10 300 python scripts/pipe2_probe.py --threads 8,10,12 --depth 2 --rounds 10 --kernel lane > $G/pipe_hc.jsonl 2> $G/pipe_hc.err || { tail $G/pipe_hc.err; exit 1; }
cut -c1-330 $G/pipe_hc.jsonl
timeout -k 10 900 python bench.py --workload c5 --c5-files 100000 --steps 20 --warmup 2 --no-cpu > $G/c5full2.log 2>&1 || { tail -20 $G/c5full2.log; exit 1; }
tail -1 $G/c5full2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['end_to_end']))"
