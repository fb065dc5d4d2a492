# round 6: memory-copy trace of the producer/consumer server (PC=P:C:pool, default 6:1:16; WVG_PCM_DMA=1 for SDMA downloads the trace can see)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $G/ptrace4 -o run -- python3 scripts/pipe2_probe.py --threads 1 --depth 2 --rounds 4 --kernel lane --pc ${PC:-6:1:16} > $G/ptrace4.log 2>&1 || { tail $G/ptrace4.log; exit 1; }
grep producers $G/ptrace4.log
python3 scripts/trace_links.py $G/ptrace4 64
