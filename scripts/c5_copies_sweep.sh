# C5: copies in flight vs queue budget, N=1 and the heaviest N=8 share (bench.py --c5-share)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/c5
O=gpurun_out/c5/copies.jsonl
run() {  # $1 = label, rest = bench args
  lab=$1; shift
  timeout -k 10 300 python bench.py --workload c5 --c5-files 100000 --steps 20 --warmup 2 --no-cpu "$@" > gpurun_out/c5/run.log 2>&1 || { echo "$lab rc=$?"; tail -5 gpurun_out/c5/run.log; exit 1; }
  tail -1 gpurun_out/c5/run.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r={'label':'$lab','ms_per_step':d['ms_per_step'],'value':d['value'],'kernel_ms':d['kernel_ms'],'copies':d['c5_copies'],'slices':d['config']['slices_rank0'],'redo':d['verified']['redo_blocks']}
print(json.dumps(r)); open('$O','a').write(json.dumps(r)+'\n')"
}
for c in 8 10 12 16 20; do run "n8r0 q24 c$c" --c5-share 8:0 --c5-copies $c; done
for c in 10 16; do WVG_BENCH_HW_QUEUES=32 run "n8r0 q32 c$c" --c5-share 8:0 --c5-copies $c; done
for c in 1 2 3; do run "n1 q24 c$c" --c5-copies $c; done
WVG_BENCH_HW_QUEUES=32 run "n1 q32 c2" --c5-copies 2
run "n1 q24 b25000 c2" --c5-batch 25000 --c5-copies 2
