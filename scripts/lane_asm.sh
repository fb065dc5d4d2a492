# gfx950 assembly of the C2 lane kernel alone (wv_pcm_lane<false, 0, 17, 17>) and a
# per-basic-block instruction census of it (the fast group is the largest block).
# usage: bash scripts/lane_asm.sh [out.s]
set -e
OUT=${1:-/tmp/wv_lane_fast.s}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -structurizecfg-skip-uniform-regions=true -mllvm -amdgpu-sched-strategy=max-ilp \
  -DWV_LANE_ONLY_FAST $LANE_DEFS --cuda-device-only -S -o "$OUT" "$(dirname "$0")/../wavpackdecoder_amd/csrc/wv_lane.hip"
python3 - "$OUT" <<'PY'
import re, sys
lines = open(sys.argv[1]).read().split("\n")
blocks, cur, kinds = [], None, {}
for l in lines:
    m = re.match(r"^(\.LBB\d+_\d+|_Z\w+):", l)
    if m:
        if cur: blocks.append((cur, sum(kinds.values()), dict(kinds)))
        cur, kinds = m.group(1), {}
    elif l.startswith("\t") and l.strip() and not l.strip().startswith((";", ".")):
        op = l.split()[0]
        k = op.split("_")[0] if op.split("_")[0] in ("v", "s", "ds", "global") else "other"
        kinds[k] = kinds.get(k, 0) + 1
if cur: blocks.append((cur, sum(kinds.values()), dict(kinds)))
for b in sorted(blocks, key=lambda b: -b[1])[:6]:
    print(b)
for m in re.finditer(r"\.vgpr_count:\s+(\d+)|\.sgpr_spill_count:\s+(\d+)|\.vgpr_spill_count:\s+(\d+)", open(sys.argv[1]).read()):
    print(m.group(0))
PY
