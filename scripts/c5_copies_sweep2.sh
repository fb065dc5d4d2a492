# C5: the N=8 share's copies and stream policies, DSD mode 3 on lanes or on the wave kernel
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/c5
O=gpurun_out/c5/copies2.jsonl
run() {  # $1 = label, rest = bench args
  lab=$1; shift
  timeout -k 10 300 python bench.py --workload c5 --c5-files 100000 --steps 20 --warmup 2 --no-cpu "$@" > gpurun_out/c5/run.log 2>&1 || { echo "$lab rc=$?"; tail -5 gpurun_out/c5/run.log; exit 1; }
  tail -1 gpurun_out/c5/run.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r={'label':'$lab','ms_per_step':d['ms_per_step'],'value':d['value'],'kernel_ms':d['kernel_ms'],'copies':d['c5_copies'],'slices':d['config']['slices_rank0'],'redo':d['verified']['redo_blocks']}
print(json.dumps(r)); open('$O','a').write(json.dumps(r)+'\n')"
}
run "n8r0 c12" --c5-share 8:0 --c5-copies 12
WVG_DSD3_WAVE=1 run "n8r0 c12 dsd3wave" --c5-share 8:0 --c5-copies 12
WVG_DSD3_WAVE=1 run "n8r0 c20 dsd3wave" --c5-share 8:0 --c5-copies 20
WVG_DSD_STREAM=1 run "n8r0 c12 own2" --c5-share 8:0 --c5-copies 12
WVG_DSD_STREAM=1 run "n8r0 c20 own2" --c5-share 8:0 --c5-copies 20
run "n8r0 c12 b6250" --c5-share 8:0 --c5-copies 6 --c5-batch 6250
run "n1 b25000 c2" --c5-batch 25000 --c5-copies 2
WVG_DSD3_WAVE=1 run "n1 b25000 c2 dsd3wave" --c5-batch 25000 --c5-copies 2
run "n1 b50000 c2" --c5-batch 50000 --c5-copies 2
run "n1 b25000 c3" --c5-batch 25000 --c5-copies 3
run "n1 b100000 c4" --c5-batch 100000 --c5-copies 4
