# Performance experiments only (no tests): placement/timeline probe + parser counters.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
B=$PWD/wavpackdecoder_amd/build
WVG_LIB=$B/exp5/libwvgpu.so timeout -k 10 200 python scripts/exp_place.py ${NBLK:-1024} > gpurun_out/exp5.log 2>&1; rc=$?
echo "exp5 rc=$rc"; grep -v Warn gpurun_out/exp5.log
[ $rc -ne 0 ] && exit $rc
WVG_PROF=4 WVG_LIB=$B/exp4/libwvgpu.so timeout -k 10 200 python scripts/exp_time.py ${NBLK:-1024} > gpurun_out/exp4.log 2>&1; rc=$?
echo "exp4 rc=$rc"; grep -v Warn gpurun_out/exp4.log
[ $rc -ne 0 ] && exit $rc
for v in $EXTRA; do
  WVG_LIB=$B/$v/libwvgpu.so timeout -k 10 200 python scripts/exp_time.py ${NBLK:-1024} > gpurun_out/$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; grep -v Warn gpurun_out/$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit $rc
