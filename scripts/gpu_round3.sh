# Round-3 GPU sequence: smoke, GPU parity (lane tests included), bench, rocprofv3
# kernel trace + FETCH/WRITE PMC of the bench (TAG), SQ counters of the lane kernel.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
TAG=$TAG bash scripts/profile.sh || exit 1
WVG_LANE_KERNEL=2 bash scripts/pmc_sq.sh > /dev/null || exit 1
python3 scripts/pmc_sq_sum.py "wv_pcm_lane<false, 17, 17>" > gpurun_out/pmc_sq_lane.txt; cat gpurun_out/pmc_sq_lane.txt
exit 0
