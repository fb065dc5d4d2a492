# round 6: the pipelined PCM stream with every call of a request issued back to back
# (wvg_batch_download_pcm_async), threads x ring depth, 24 hardware queues (as bench.py)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
export GPU_MAX_HW_QUEUES=24
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k format_epilogue --timeout 120 --timeout-method thread > $G/t_async.log 2>&1 || { tail -20 $G/t_async.log; exit 1; }
tail -1 $G/t_async.log
timeout -k 10 300 python scripts/pipe2_probe.py --async-download --threads 2,4,8 --depth 2,3,4 --rounds 10 --kernel ${KERNEL:-auto} > $G/pipe_async.jsonl 2> $G/pipe_async.err || { tail $G/pipe_async.err; exit 1; }
cut -c1-330 $G/pipe_async.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $G/ptrace3 -o run -- python3 scripts/pipe2_probe.py --async-download --threads ${TT:-4} --depth ${TD:-3} --rounds 10 --kernel auto > $G/ptrace3.log 2>&1 || { tail $G/ptrace3.log; exit 1; }
python3 scripts/trace_links.py $G/ptrace3 40
