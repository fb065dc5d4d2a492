# round 6: the async pipelined PCM stream with the copy-to-host kernel (wvg_batch_download_pcm_async)
# against the blocking ring, 24 hardware queues (as bench.py)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k format_epilogue --timeout 120 --timeout-method thread > $G/t_async.log 2>&1 || { tail -20 $G/t_async.log; exit 1; }
tail -1 $G/t_async.log
timeout -k 10 300 python scripts/pipe2_probe.py --async-download --threads 2,4,8 --depth 2,3 --rounds 10 --kernel auto > $G/pipe_async_kern.jsonl 2> $G/pipe_async_kern.err || { tail $G/pipe_async_kern.err; exit 1; }
cut -c1-330 $G/pipe_async_kern.jsonl
timeout -k 10 300 python scripts/pipe2_probe.py --threads 8 --depth 2 --rounds 10 --kernel auto > $G/pipe_sync.jsonl 2> $G/pipe_sync.err || { tail $G/pipe_sync.err; exit 1; }
cut -c1-330 $G/pipe_sync.jsonl
