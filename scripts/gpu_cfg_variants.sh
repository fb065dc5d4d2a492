# bench_configs.py rates for experiment builds (WVG_LIB), e.g.
#   LIBS="build/libwvgpu.so build/exp_x/libwvgpu.so" CFGS="c4" bash scripts/gpu_cfg_variants.sh
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/cv
LIBS=${LIBS:-"build/libwvgpu.so"}
CFGS=${CFGS:-"c4"}
i=0
for L in $LIBS; do
  i=$((i+1))
  WVG_LIB=$GRAFT_REPO_ROOT/wavpackdecoder_amd/$L timeout -k 10 600 python scripts/bench_configs.py $CFGS > gpurun_out/cv/c$i.jsonl 2> gpurun_out/cv/c$i.err || { tail -3 gpurun_out/cv/c$i.err; exit 1; }
  echo "== $L"; cut -c1-200 gpurun_out/cv/c$i.jsonl
done
