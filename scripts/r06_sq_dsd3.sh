# round 6: SQ counters of the DSD mode-3 pair kernel on the final (iterative-ILP) build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && rm -rf gpurun_out/pmc_sq
PROG=scripts/bench_configs.py ARGS="dsd3 --dsd-files 1024 --kernel lane" bash scripts/pmc_sq.sh > /dev/null || exit 1
mkdir -p gpurun_out/g && python3 scripts/pmc_sq_sum.py "wv_dsd3_pair" > gpurun_out/g/pmc_sq_dsd3pair2.txt && cat gpurun_out/g/pmc_sq_dsd3pair2.txt
