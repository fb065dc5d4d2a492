# round 6: stream cap A/B on one box (WVG_STREAM_CAP=0 disables it): C5 100k bench and the 4,000-file slice
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
for cap in 1 0 1 0; do
  export WVG_STREAM_CAP=$cap
  timeout -k 10 600 python bench.py --workload c5 --c5-files 100000 --steps 20 --warmup 2 --no-cpu --c5-e2e 0 > $G/c5cap$cap.log 2>&1 || { tail -20 $G/c5cap$cap.log; exit 1; }
  echo "cap $cap c5 100k: $(tail -1 $G/c5cap$cap.log | grep -o '"value": [0-9.]*')"
done
for cap in 1 0; do
  export WVG_STREAM_CAP=$cap
  timeout -k 10 300 python scripts/bench_configs.py c5 --kernel lane --inflight 20 > $G/c5scap$cap.jsonl 2>/dev/null || exit 1
  echo "cap $cap c5 slice: $(grep -o '"Mframes_per_s_inflight": [0-9.]*' $G/c5scap$cap.jsonl)"
done
