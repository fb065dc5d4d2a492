# round 6: async vs blocking pipelined PCM stream on the lane kernel (no AUTO queries), 24 queues
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 300 python scripts/pipe2_probe.py --async-download --threads 4,8,12 --depth 2,3 --rounds 10 --kernel lane > $G/pipe_async_lane.jsonl 2> $G/pipe_async_lane.err || { tail $G/pipe_async_lane.err; exit 1; }
cut -c1-330 $G/pipe_async_lane.jsonl
timeout -k 10 300 python scripts/pipe2_probe.py --threads 8,12 --depth 2,3 --rounds 10 --kernel lane > $G/pipe_sync_lane.jsonl 2> $G/pipe_sync_lane.err || { tail $G/pipe_sync_lane.err; exit 1; }
cut -c1-330 $G/pipe_sync_lane.jsonl
