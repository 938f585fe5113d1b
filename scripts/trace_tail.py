"""Per-kernel average duration over the last fraction of a rocprofv3 kernel trace (steady state)."""
import collections
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
r.sort(key=lambda x: int(x["Start_Timestamp"]))
tail = r[-int(len(r) * frac):]
d = collections.defaultdict(list)
for x in tail:
    d[x["Kernel_Name"][:90]].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
busy = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:90s} {len(v):5d} {sum(v) / len(v):8.2f}")
print(f"span {span:.1f} us, busy {busy:.1f} us, gaps {span - busy:.1f} us over {len(tail)} launches")
