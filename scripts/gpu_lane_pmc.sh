# SQ instruction counters of the lane kernel alone (WVG_LANE_KERNEL=2) on C2, then
# C2 rates at several in-flight depths for both kernels (24 hardware queues).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
WVG_LANE_KERNEL=2 bash scripts/pmc_sq.sh || exit 1
python3 scripts/pmc_sq_sum.py "wv_pcm_lane<17, 17>"
NO_TESTS=1 CFGS="${CFGS:-1:8 1:16 1:20 0:3 0:6}" bash scripts/gpu_lane.sh
