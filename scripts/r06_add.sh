cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
timeout -k 10 300 python scripts/r06_add_probe.py > gpurun_out/g/add_probe.log 2>&1; rc=$?; cat gpurun_out/g/add_probe.log | grep -v amdgpu.ids; exit $rc
