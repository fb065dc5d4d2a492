# Lane kernel diagnostics: why blocks go back to the two-wave kernel, the lane
# kernel's time alone (WVG_LANE_KERNEL=2: no redo launch), GPU parity with the
# lane kernel on, and C2 at a few in-flight depths (gpu_lane.sh).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/lane
timeout -k 10 300 python scripts/lane_diag.py > gpurun_out/lane/diag.log 2>&1; rc=$?; tail -5 gpurun_out/lane/diag.log; [ $rc -ne 0 ] && exit $rc
WVG_LANE_KERNEL=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lane/prof -o lane --output-format csv -- python3 scripts/lane_diag.py > gpurun_out/lane/prof.log 2>&1; rc=$?
find gpurun_out/lane/prof -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | head -4
[ $rc -ne 0 ] && exit $rc
CFGS="${CFGS:-1:3 1:20 0:3}" bash scripts/gpu_lane.sh
