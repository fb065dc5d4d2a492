#!/usr/bin/env python3
"""Copy a scripts/profile.sh run (gpurun_out/prof) into profiles/<tag>_*.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
profiles/<tag>_pmc.json: per-launch HBM bytes of the bench kernel from the
separate FETCH_SIZE / WRITE_SIZE passes (unit KiB).  MI355X_MICROARCH.md: on
gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane vector streaming reads
and other widths are uncalibrated.  The bench kernel reads its payload with
scalar s_load_dwordx2 for the two-wave kernel (scale 1: the raw FETCH_SIZE equals
the known bytes it must read) and global_load_dwordx4 for the lane kernels' LDS
staging (FETCH_SCALE=2, the guide's gfx950 correction for 16-B-per-lane reads).
bench.py reports `roofline.traffic` from it.
usage: [FETCH_SCALE=1] python scripts/pmc_to_profile.py <tag> [kernel-substring]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "wv_pcm_2wave"
src = os.path.join(ROOT, "gpurun_out", "prof")
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", f"{tag}_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))


def per_dispatch(path, counter):
    per = collections.defaultdict(float)
    name = None
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name = r["Kernel_Name"]
    return name, sorted(per.values())


name, fetch = per_dispatch(os.path.join(src, "fetch", f"{tag}_fetch_counter_collection.csv"), "FETCH_SIZE")
_, write = per_dispatch(os.path.join(src, "write", f"{tag}_write_counter_collection.csv"), "WRITE_SIZE")
stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(dst, f"{tag}_kernel_stats.csv")))}
st = next(v for k, v in stats.items() if kern in k)
fetch_kib = sum(fetch) / len(fetch)
scale = float(os.environ.get("FETCH_SCALE", "1"))
NOTE_X1 = ("FETCH_SIZE/WRITE_SIZE in KiB. Payload read by scalar s_load_dwordx2 (the two-wave kernel): raw FETCH_SIZE "
           "calibrated against the known read bytes (compressed payload + block descriptors) -> scale 1; WRITE from "
           "dword-per-lane stores equals the int32 output byte count")
NOTE_X2 = ("FETCH_SIZE/WRITE_SIZE in KiB. Payload read by global_load_dwordx4 (16 B per lane: the lane kernels' LDS "
           "staging), which gfx950's FETCH_SIZE counts at half (MI355X_MICROARCH.md) -> scale 2; WRITE from "
           "dword-per-lane stores equals the int32 output byte count")
write_kib = sum(write) / len(write)
out = {
    "kernel": name,
    "rocprof_avg_ns": float(st["AverageNs"]), "rocprof_calls": int(st["Calls"]),
    "dispatches_counted": {"FETCH_SIZE": len(fetch), "WRITE_SIZE": len(write)},
    "fetch_size_kib_per_launch": fetch_kib, "write_size_kib_per_launch": write_kib,
    "fetch_scale": scale,
    "fetch_bytes_per_launch": fetch_kib * 1024 * scale,
    "write_bytes_per_launch": write_kib * 1024,
    "traffic_bytes_per_launch": fetch_kib * 1024 * scale + write_kib * 1024,
    "note": os.environ.get("PMC_NOTE", NOTE_X2 if scale == 2 else NOTE_X1),
}
with open(os.path.join(dst, f"{tag}_pmc.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
