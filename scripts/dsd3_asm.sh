# gfx950 assembly of the DSD mode-3 lane kernels (wv_dsd_lane.hip) and a per-basic-block
# instruction census of each kernel (the frame loop is the largest block).
# usage: bash scripts/dsd3_asm.sh [out.s]
set -e
OUT=${1:-/tmp/wv_dsd_lane.s}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=${SCHED:-iterative-ilp} \
  --cuda-device-only -S -o "$OUT" "$(dirname "$0")/../wavpackdecoder_amd/csrc/wv_dsd_lane.hip"
python3 - "$OUT" <<'PY'
import re, sys
lines = open(sys.argv[1]).read().split("\n")
blocks, cur, kinds, fn = [], None, {}, None
for l in lines:
    m = re.match(r"^(\.LBB\d+_\d+|_Z\w+):", l)
    if m:
        if cur: blocks.append((fn, cur, sum(kinds.values()), dict(kinds)))
        cur, kinds = m.group(1), {}
        if cur.startswith("_Z"): fn = cur
    elif l.startswith("\t") and l.strip() and not l.strip().startswith((";", ".")):
        op = l.split()[0]
        k = op.split("_")[0] if op.split("_")[0] in ("v", "s", "ds", "global") else "other"
        if op.endswith("_dpp") or "dpp" in l: k = "dpp"
        kinds[k] = kinds.get(k, 0) + 1
if cur: blocks.append((fn, cur, sum(kinds.values()), dict(kinds)))
for b in sorted(blocks, key=lambda b: -b[2])[:4]:
    print(b)
for m in re.finditer(r"\.name:\s+(\S+)|\.vgpr_count:\s+(\d+)|\.sgpr_spill_count:\s+(\d+)|\.vgpr_spill_count:\s+(\d+)", open(sys.argv[1]).read()):
    print(m.group(0))
PY
