# round 6: the driver's bench under rocprofv3 (kernel trace + stats; FETCH_SIZE and WRITE_SIZE passes),
# then the SQ instruction counters of the C2 lane kernel
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_sq
TAG=${TAG:-r06} bash scripts/profile.sh || exit 1
bash scripts/pmc_sq.sh > /dev/null || exit 1
python3 scripts/pmc_sq_sum.py "${KSUB:-wv_pcm_lane<false, 0, 17, 17>}" > gpurun_out/prof/pmc_sq_lane.txt && cat gpurun_out/prof/pmc_sq_lane.txt
