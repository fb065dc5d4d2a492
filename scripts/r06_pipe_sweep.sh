# round 6: the pipelined PCM request stream, threads x ring depth, 24 hardware queues (as bench.py)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 300 python scripts/pipe2_probe.py --threads 4,8,12 --depth 2,3,4 --rounds 8 --kernel ${KERNEL:-auto} > $G/pipe_sweep.jsonl 2> $G/pipe_sweep.err || { tail $G/pipe_sweep.err; exit 1; }
cut -c1-330 $G/pipe_sweep.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $G/ptrace2 -o run -- python3 scripts/pipe2_probe.py --threads ${TT:-8} --depth ${TD:-3} --rounds 8 --kernel auto > $G/ptrace2.log 2>&1 || { tail $G/ptrace2.log; exit 1; }
tail -1 $G/ptrace2.log
