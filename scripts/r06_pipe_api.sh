# round 6: HIP API trace of the async pipelined stream (which call blocks the request threads)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 300 rocprofv3 --hip-runtime-trace --output-format csv -d $G/papi -o run -- python3 scripts/pipe2_probe.py --async-download --threads 8 --depth 2 --rounds 10 --kernel auto > $G/papi.log 2>&1 || { tail $G/papi.log; exit 1; }
tail -1 $G/papi.log
ls $G/papi
