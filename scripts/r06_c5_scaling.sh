# round 6: C5 predicted strong scaling (per-rank shares timed alone) on the current build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/c5
timeout -k 10 1100 python scripts/c5_scaling.py --ns ${NS:-1,2,4,8} --out gpurun_out/c5/scal_r06c.jsonl > gpurun_out/c5/scal_r06c.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/c5/scal_r06c.log; exit 1; }
grep summary gpurun_out/c5/scal_r06c.jsonl
