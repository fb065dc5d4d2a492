# round 6: the 100,000-file C5 corpus on one GPU (bench.py --workload c5: device-resident steps,
# the end-to-end leg, the CPU baseline on a sample)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 900 python bench.py --workload c5 --c5-files 100000 --steps 20 --warmup 2 > $G/c5full.log 2>&1 || { tail -20 $G/c5full.log; exit 1; }
tail -1 $G/c5full.log | cut -c1-3000
