"""Kernel stats (calls, total/avg us) from a rocprofv3 results database (sqlite 'kernels' view).
usage: python scripts/db_stats.py run_results.db [per_token_divisor]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start) from kernels group by {name} "
                 f"order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
for n, cnt, s, a in rows[:25]:
    print(f"{s / 1e3 / div:9.1f} us/tok {cnt / div:6.1f}/tok {a / 1e3:8.2f} us  {n[:110]}")
print(f"total {tot / 1e3 / div:.1f} us per unit")
