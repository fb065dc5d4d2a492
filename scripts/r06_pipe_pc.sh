# round 6: producer/consumer request server for the pipelined PCM stream (24 hardware queues)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 400 python scripts/pipe2_probe.py --threads 1 --depth 2 --rounds 4 --kernel lane --pc ${PC:-4:1:12,6:1:16,8:1:16,6:2:16,8:2:20,10:2:20} > $G/pipe_pc.jsonl 2> $G/pipe_pc.err || { tail $G/pipe_pc.err; exit 1; }
cat $G/pipe_pc.jsonl
