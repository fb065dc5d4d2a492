# round 6: kernel + memory-copy trace of the pipelined PCM request stream (8 threads x 2-deep rings)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
GPU_MAX_HW_QUEUES=24 timeout -k 10 300 python scripts/pipe2_probe.py --threads 8 --depth 2,3 --rounds 6 --kernel auto > $G/pipe2_q24.jsonl 2> $G/pipe2_q24.err || { tail $G/pipe2_q24.err; exit 1; }
cut -c1-300 $G/pipe2_q24.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $G/ptrace -o run -- python3 scripts/pipe2_probe.py --threads 8 --depth 2 --rounds 6 --kernel auto > $G/ptrace.log 2>&1 || { tail $G/ptrace.log; exit 1; }
tail -2 $G/ptrace.log
find $G/ptrace -name "*.csv" | head
