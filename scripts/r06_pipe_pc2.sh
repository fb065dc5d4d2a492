# round 6: the producer/consumer server with Python's default GIL switch interval and with 0.1 ms
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 300 python scripts/pipe2_probe.py --threads 1 --depth 2 --rounds 4 --kernel lane --pc 6:1:16,6:2:16 > $G/pipe_pc_a.jsonl 2> $G/pipe_pc_a.err || { tail $G/pipe_pc_a.err; exit 1; }
timeout -k 10 300 python scripts/pipe2_probe.py --threads 1 --depth 2 --rounds 4 --kernel lane --pc 6:1:16,6:2:16 --switch 0.0001 > $G/pipe_pc_b.jsonl 2> $G/pipe_pc_b.err || { tail $G/pipe_pc_b.err; exit 1; }
cat $G/pipe_pc_a.jsonl $G/pipe_pc_b.jsonl
