# kernel-time experiments: shipped build, parser-only (exp1), recon-only (exp2), parser counters (exp3)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
B=$PWD/wavpackdecoder_amd/build
timeout -k 10 300 python scripts/exp_time.py 1 256 512 1024 > gpurun_out/exp0.log 2>&1 && \
WVG_LIB=$B/exp1/libwvgpu.so timeout -k 10 200 python scripts/exp_time.py 1 1024 > gpurun_out/exp1.log 2>&1 && \
WVG_LIB=$B/exp2/libwvgpu.so timeout -k 10 200 python scripts/exp_time.py 1 1024 > gpurun_out/exp2.log 2>&1 && \
WVG_PROF=1 WVG_LIB=$B/exp3/libwvgpu.so timeout -k 10 200 python scripts/exp_time.py 1 > gpurun_out/exp3.log 2>&1
rc=$?; cat gpurun_out/exp[0-3].log | grep -v Warn; [ $rc -ne 0 ] && exit $rc
WVG_PROF=4 WVG_LIB=$B/exp4/libwvgpu.so timeout -k 10 200 python scripts/exp_time.py 1024 > gpurun_out/exp4.log 2>&1; cat gpurun_out/exp4.log | grep -v Warn
