# round 6: the decode server's rate beside the same box's PCIe rates (scripts/micro/pcie_kernel.hip),
# so the server is read as a fraction of its own box's link
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/micro/pcie_kernel.hip -o gpurun_out/g/pcie_kernel || exit 1
timeout -k 10 120 gpurun_out/g/pcie_kernel 90 > gpurun_out/g/link.jsonl 2>&1 || exit 1
timeout -k 10 300 python scripts/pipe2_probe.py --threads 1 --depth 2 --kernel lane --rounds 6 --pc "6:2:16,6:2:16" >> gpurun_out/g/link.jsonl 2> gpurun_out/g/link.err || exit 1
cat gpurun_out/g/link.jsonl
