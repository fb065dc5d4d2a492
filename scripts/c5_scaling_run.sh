cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/c5
timeout -k 10 900 python scripts/c5_scaling.py --ns 1,2,4,8 --out gpurun_out/c5/scal_default.jsonl > gpurun_out/c5/scal_default.log 2>&1 || { echo "default rc=$?"; tail -20 gpurun_out/c5/scal_default.log; exit 1; }
grep summary gpurun_out/c5/scal_default.jsonl
WVG_DSD_STREAM=0 timeout -k 10 400 python scripts/c5_scaling.py --ns 1,8 --out gpurun_out/c5/scal_off.jsonl > gpurun_out/c5/scal_off.log 2>&1 || { echo "off rc=$?"; tail -20 gpurun_out/c5/scal_off.log; exit 1; }
grep summary gpurun_out/c5/scal_off.jsonl
