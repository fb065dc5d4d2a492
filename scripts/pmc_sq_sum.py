#!/usr/bin/env python3
"""Sum the pmc_sq.sh counter passes per dispatch of one kernel (substring)."""
import collections, csv, glob, sys
kern = sys.argv[1] if len(sys.argv) > 1 else "wv_pcm_2wave<17, 17>"
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for path in sorted(glob.glob("gpurun_out/pmc_sq/*/*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"]:
            tot[r["Counter_Name"]][(path, r["Dispatch_Id"])] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    vals = list(v.values())
    print(f"{k:24s} per dispatch {sum(vals) / len(vals):16.4e}  (dispatches {len(vals)})")
