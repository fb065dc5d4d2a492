# round 6: the new lane scope and status tests, the 100k-file C5 parity test, a kernel trace
# of the heaviest N=8 C5 share, PCIe bounds and the pipelined end-to-end phases
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6a
G=gpurun_out/r6a
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread ${PROBE_TESTS:-tests/test_gpu_parity.py::test_poison_then_decode_stores_every_status} -m gpu -s > $G/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $G/pytest.log; exit 1; }
grep -E "passed|failed|PARITY" $G/pytest.log | tail -5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o c5s8 -- python3 bench.py --workload c5 --c5-files 100000 --c5-share 8:0 --c5-copies 12 --steps 20 --warmup 2 --no-cpu --c5-e2e 0 > $G/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $G/prof.log; exit 1; }
tail -1 $G/prof.log | cut -c1-200
timeout -k 10 120 python3 scripts/pcie_probe.py > $G/pcie.log 2>&1 || { echo "pcie rc=$?"; tail -5 $G/pcie.log; exit 1; }
cat $G/pcie.log
timeout -k 10 300 python3 scripts/pipe2_probe.py --threads 1,2,4,6 > $G/pipe2.log 2>&1 || { echo "pipe2 rc=$?"; tail -5 $G/pipe2.log; exit 1; }
cat $G/pipe2.log
