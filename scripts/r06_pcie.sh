# round 6: PCIe rates (SDMA engines vs blit kernels) and the pipelined PCM request stream under each
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g
G=gpurun_out/g
timeout -k 10 120 python scripts/pcie_probe.py > $G/pcie_sdma.json 2>&1 || { tail $G/pcie_sdma.json; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 120 python scripts/pcie_probe.py > $G/pcie_blit.json 2>&1 || { tail $G/pcie_blit.json; exit 1; }
cat $G/pcie_sdma.json $G/pcie_blit.json
HSA_ENABLE_SDMA=0 timeout -k 10 300 python scripts/pipe2_probe.py --threads 4,8 --depth 2,3 --rounds 6 --kernel auto > $G/pipe2_blit.jsonl 2> $G/pipe2_blit.err || { tail $G/pipe2_blit.err; exit 1; }
cut -c1-300 $G/pipe2_blit.jsonl
