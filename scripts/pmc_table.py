"""Sum per-dispatch PMC counters of kernels matching a name filter, grouped by grid.
usage: pmc_table.py <gpurun_out/tag> <name filter>"""
import collections
import csv
import glob
import sys

root, filt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob(root + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].replace("ghip::(anonymous namespace)::", "")[:40], r.get("Grid_Size", r.get("Grid_Size_X", "")))
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(key, r["Counter_Name"])] += 1
for key, d in agg.items():
    print(key)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:16.4g}  (dispatch rows {n[(key, c)]})")
