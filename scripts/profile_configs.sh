# Device-resident rates of C1/C3/C4/C5 (+ DSD modes) and their rocprofv3 kernel
# statistics (--kernel-trace --stats only; PMC passes are separate runs).
# Outputs under gpurun_out/prof_cfg; copy the summaries into profiles/<TAG>_*.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/prof_cfg
TAG=${TAG:-r03}
CFGS=${CFGS:-"c1 c3 c4 c5 dsd0 dsd1 dsd3"}
timeout -k 10 900 python3 scripts/bench_configs.py $CFGS --cpu-threads 16 --inflight 3 > gpurun_out/prof_cfg/rates.jsonl 2> gpurun_out/prof_cfg/rates.err
rc=$?; echo "rates rc=$rc"; cat gpurun_out/prof_cfg/rates.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_cfg/rates.err; exit $rc; }
# the PCM configs again on the lane kernel, 20 batches in flight (bench.py's C2 setting)
LANE_CFGS=${LANE_CFGS:-"c1 c3 c4 c5"}
if [ -n "$LANE_CFGS" ]; then
  timeout -k 10 900 python3 scripts/bench_configs.py $LANE_CFGS --kernel lane --inflight 20 > gpurun_out/prof_cfg/rates_lane.jsonl 2>> gpurun_out/prof_cfg/rates.err
  rc=$?; echo "lane rates rc=$rc"; cat gpurun_out/prof_cfg/rates_lane.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_cfg/rates.err; exit $rc; }
fi
for c in $CFGS; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg/$c -o ${TAG}_$c --output-format csv -- python3 scripts/bench_configs.py $c > gpurun_out/prof_cfg/$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_cfg/$c.log; exit $rc; }
done
find gpurun_out/prof_cfg -name "*kernel_stats.csv" | sort
