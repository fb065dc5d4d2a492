# SQ instruction counters of the lane kernel alone (WVG_LANE_KERNEL=2) on C2, then
# GPU parity with the lane kernel on.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
WVG_LANE_KERNEL=2 bash scripts/pmc_sq.sh || exit 1
python3 scripts/pmc_sq_sum.py "wv_pcm_lane<17, 17>"
mkdir -p gpurun_out/lane
WVG_LANE_KERNEL=1 timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lane/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/lane/pytest.log; grep -E "^E  " gpurun_out/lane/pytest.log | head -12
exit $rc
