cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/micro/pcie_kernel.hip -o gpurun_out/g/pcie_kernel && timeout -k 10 120 gpurun_out/g/pcie_kernel 90 > gpurun_out/g/pcie_kernel.jsonl 2>&1; rc=$?; cat gpurun_out/g/pcie_kernel.jsonl; exit $rc
