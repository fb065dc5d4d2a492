# round 6: the 4,000-file C5 slice at 20 in flight under the stream policies
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
for pol in default 0 1; do
  if [ $pol = default ]; then unset WVG_DSD_STREAM; else export WVG_DSD_STREAM=$pol; fi
  timeout -k 10 300 python scripts/bench_configs.py c5 --kernel lane --inflight 20 > $G/c5s_$pol.jsonl 2> $G/c5s_$pol.err || { tail $G/c5s_$pol.err; exit 1; }
  echo "policy $pol: $(grep -o '"kernel_ms": [0-9.]*\|"Mframes_per_s_inflight": [0-9.]*' $G/c5s_$pol.jsonl | tr '\n' ' ')"
done
