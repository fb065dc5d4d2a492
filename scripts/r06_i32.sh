cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 300 python scripts/r06_i32_probe.py > $G/i32.log 2>&1 || { tail $G/i32.log; exit 1; }
tail -1 $G/i32.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/i32prof -o run -- python3 scripts/r06_i32_probe.py > $G/i32prof.log 2>&1 || { tail $G/i32prof.log; exit 1; }
find $G/i32prof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 | head -12
