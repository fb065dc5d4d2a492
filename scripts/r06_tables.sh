# round 6: DSD mode-1 host tables kept for chained blocks only -- DSD / C5 / parity tests, the add_files phases
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 900 python -u -m pytest tests/test_gpu_dsd_lane.py tests/test_gpu_dsd1_lane.py tests/test_gpu_c5.py tests/test_gpu_parity.py tests/test_gpu_dframe.py tests/test_gpu_c5_full.py -m gpu -x -q --timeout 600 --timeout-method thread > $G/t_tab.log 2>&1 || { tail -30 $G/t_tab.log; exit 1; }
tail -1 $G/t_tab.log
timeout -k 10 300 python scripts/r06_add_probe.py > $G/add_probe.log 2>&1 || { tail $G/add_probe.log; exit 1; }
grep -v amdgpu.ids $G/add_probe.log | tail -4
