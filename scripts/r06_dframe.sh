# round 6: device framing with the parallel copy and the batched info fetch -- tests, the add_files probe
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 600 python -u -m pytest tests/test_gpu_dframe.py tests/test_gpu_parity.py tests/test_gpu_c5.py -m gpu -x -q --timeout 300 --timeout-method thread > $G/t_df.log 2>&1 || { tail -30 $G/t_df.log; exit 1; }
tail -1 $G/t_df.log
timeout -k 10 300 python scripts/r06_add_probe.py > $G/add_probe.log 2>&1 || { tail $G/add_probe.log; exit 1; }
grep -v amdgpu.ids $G/add_probe.log | tail -5
