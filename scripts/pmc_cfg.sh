# SQ instruction counters of one bench_configs.py config, per experiment build:
#   LIBS="build/libwvgpu.so ..." CFG=c4 bash scripts/pmc_cfg.sh
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pc
LIBS=${LIBS:-"build/libwvgpu.so"}
CFG=${CFG:-c4}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_INSTS_LDS"
i=0
for L in $LIBS; do
  i=$((i+1))
  WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -s KILL 300 rocprofv3 --pmc $A -d gpurun_out/pc/p$i -o p$i --output-format csv -- python3 scripts/bench_configs.py $CFG > gpurun_out/pc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pc/p$i.log; exit 1; }
done
find gpurun_out/pc -name "*counter_collection.csv"
