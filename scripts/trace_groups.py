"""Per-(kernel, grid) totals of a rocprofv3 kernel trace directory.  usage: trace_groups.py <dir> [n]"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
g = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = (r["Kernel_Name"].replace("ghip::(anonymous namespace)::", "")[:60], r["Grid_Size_X"], r["Grid_Size_Y"])
    g[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:n]:
    print(f"{k[0]:60s} grid {k[1]:>8s}x{k[2]:<5s} calls {len(v):5d} avg {sum(v)/len(v)/1e3:9.1f} us total {sum(v)/1e6:8.2f} ms")
