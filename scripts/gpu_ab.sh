# A/B of kernel routes on the config corpora (device-resident rates) + kernel trace
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
CFGS=${CFGS:-"c3 c5"}
for v in 0 1; do
  WVG_PIPE=$v timeout -k 10 600 python3 scripts/bench_configs.py $CFGS > gpurun_out/ab/pipe$v.jsonl 2> gpurun_out/ab/pipe$v.err || { tail -5 gpurun_out/ab/pipe$v.err; exit 1; }
  echo "WVG_PIPE=$v"; cat gpurun_out/ab/pipe$v.jsonl
done
WVG_PIPE=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof -o pipe --output-format csv -- python3 scripts/bench_configs.py c3 > gpurun_out/ab/prof.log 2>&1 || exit 1
find gpurun_out/ab/prof -name "*stats.csv"
