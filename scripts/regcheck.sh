# Register budget of every kernel (VGPRs, SGPR spills, scratch) from the gfx950
# device assembly -- run after any kernel change (a spill reloaded in a
# frame loop, or a VGPR count past 256, halves a kernel's occupancy).
set -e
OUT=${1:-/tmp/wv_decode_gfx950.s}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -structurizecfg-skip-uniform-regions=true \
  --cuda-device-only -S -o "$OUT" "$(dirname "$0")/../wavpackdecoder_amd/csrc/wv_decode.hip"
python3 - "$OUT" <<'PY'
import re, sys
s = open(sys.argv[1]).read()
for m in re.finditer(r"\.name:\s+(\S+)(.*?)\.vgpr_spill_count:\s+(\d+)", s, re.S):
    body = m.group(2)
    g = lambda k: re.search(r"\." + k + r":\s+(\d+)", body)
    name = re.sub(r"_ZN3wvg12wv_pcm_2waveIJ(.*)EEEEv.*", lambda x: "wv_pcm_2wave<" + x.group(1) + ">", m.group(1))
    print(f"{name[:90]:90s} vgpr={g('vgpr_count').group(1):>4} sgpr_spill={g('sgpr_spill_count').group(1):>4} "
          f"scratch={g('private_segment_fixed_size').group(1):>5} vgpr_spill={m.group(3)}")
PY
