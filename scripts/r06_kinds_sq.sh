# round 6: in-flight rates of the PCM kinds the round-6 lanes added (beside their neighbours),
# then the SQ counters of the DSD mode-3 pair kernel
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 600 python scripts/bench_configs.py hykinds --kernel lane --inflight 20 > $G/hykinds.jsonl 2> $G/hykinds.err || { tail $G/hykinds.err; exit 1; }
cut -c1-420 $G/hykinds.jsonl
rm -rf gpurun_out/pmc_sq
PROG=scripts/bench_configs.py ARGS="dsd3 --dsd-files 1024 --kernel lane" bash scripts/pmc_sq.sh > /dev/null || exit 1
python3 scripts/pmc_sq_sum.py "wv_dsd3_pair" > $G/pmc_sq_dsd3pair.txt && cat $G/pmc_sq_dsd3pair.txt
