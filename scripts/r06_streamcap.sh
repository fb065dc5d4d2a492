# round 6: the stream cap -- env-route tests, the 4,000-file C5 slice at 20 in flight, the 100k C5 bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 600 python -u -m pytest tests/test_gpu_env_routes.py tests/test_gpu_c5.py tests/test_gpu_auto_policy.py -m gpu -x -q --timeout 300 --timeout-method thread > $G/t_cap.log 2>&1 || { tail -30 $G/t_cap.log; exit 1; }
tail -1 $G/t_cap.log
timeout -k 10 300 python scripts/bench_configs.py c5 dsd3 dsd1 --dsd-files 1024 --kernel lane --inflight 20 > $G/c5s_cap.jsonl 2> $G/c5s_cap.err || { tail $G/c5s_cap.err; exit 1; }
cut -c1-120 $G/c5s_cap.jsonl; grep -o '"Mframes_per_s_inflight": [0-9.]*' $G/c5s_cap.jsonl
timeout -k 10 900 python bench.py --workload c5 --c5-files 100000 --steps 20 --warmup 2 --no-cpu --c5-e2e 0 > $G/c5cap.log 2>&1 || { tail -20 $G/c5cap.log; exit 1; }
tail -1 $G/c5cap.log | cut -c1-300
