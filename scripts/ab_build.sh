# A/B build of one kernel file: reuse build/'s other objects, recompile FILE with the
# extra flags, link into wavpackdecoder_amd/build_ab_<TAG>/libwvgpu.so
#   bash scripts/ab_build.sh <TAG> <file.hip> "<-D flags>" [extra hipcc flags]
set -e
TAG=$1; SRC=$2; DEFS=$3; XF=$4
cd "$(dirname "$0")/../wavpackdecoder_amd"
OUT=build_ab_$TAG
mkdir -p $OUT
base=$(basename "$SRC" .hip)
for o in build/*.o; do [ "$(basename $o .o)" = "$base" ] || cp "$o" $OUT/; done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result \
  -mllvm -structurizecfg-skip-uniform-regions=true $XF $DEFS -c -o $OUT/$base.o csrc/$base.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libwvgpu.so $OUT/*.o
echo $OUT/libwvgpu.so
