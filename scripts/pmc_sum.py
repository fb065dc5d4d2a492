"""Summarise rocprofv3 --pmc csv output: per kernel, first dispatch, counters summed over instances."""
import collections
import csv
import glob
import sys

for path in sorted(glob.glob(sys.argv[1] + "/*/*_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"][:50], int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    seen = set()
    for (name, disp), v in sorted(agg.items(), key=lambda x: x[0][1]):
        if "rocclr" in name or name in seen:
            continue
        seen.add(name)
        print(path.split("/")[-2], name, disp, {k: int(x) for k, x in sorted(v.items())})
