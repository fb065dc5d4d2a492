# Instruction-level PMC passes for the bench kernel (one rocprofv3 --pmc run per
# counter group, nothing else traced): SALU/SMEM/VALU instruction counts, wave
# cycles, waits, branches -- per launch in gpurun_out/pmc_sq/<pass>.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc_sq
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU"
B="SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SMEM"
PROG=${PROG:-bench.py}
ARGS=${ARGS:-"--inflight 1 --steps 2 --warmup 0 --no-cpu --timed-only"}
n=0
for grp in "$A" "$B"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_sq/p$n -o p$n --output-format csv -- python3 $PROG $ARGS > gpurun_out/pmc_sq/p$n.log 2>&1 || { echo "pass $n failed"; tail -3 gpurun_out/pmc_sq/p$n.log; exit 1; }
done
find gpurun_out/pmc_sq -name "*counter_collection.csv"
