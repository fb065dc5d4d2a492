# PMC probe of the parser wave alone (exp1 build, 1 block).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY"
C2="SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVES SQ_INSTS_SENDMSG"
C3="SQ_IFETCH SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_FLAT"
L=$PWD/wavpackdecoder_amd/build/exp1/libwvgpu.so
WVG_LIB=$L timeout -k 10 240 rocprofv3 --pmc $C1 -d gpurun_out/pmc/a1 -o a1 --output-format csv -- python3 scripts/exp_time.py 1 > gpurun_out/pmc/a1.log 2>&1 && \
WVG_LIB=$L timeout -k 10 240 rocprofv3 --pmc $C2 -d gpurun_out/pmc/a2 -o a2 --output-format csv -- python3 scripts/exp_time.py 1 > gpurun_out/pmc/a2.log 2>&1 && \
WVG_LIB=$L timeout -k 10 240 rocprofv3 --pmc $C3 -d gpurun_out/pmc/a3 -o a3 --output-format csv -- python3 scripts/exp_time.py 1 > gpurun_out/pmc/a3.log 2>&1
rc=$?; echo rc=$rc; tail -3 gpurun_out/pmc/a3.log; exit $rc
