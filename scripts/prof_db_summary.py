"""Per-kernel summary of a rocprofv3 SQLite output (rocpd `kernels` view): total / count / average
duration per kernel name, sorted by total.  usage: python scripts/prof_db_summary.py results.db [divisor]
(divisor: e.g. the number of identical passes the profile covered, to print per-pass totals)."""
import sqlite3
import sys

db = sys.argv[1]
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end - start), avg(end - start) from kernels group by name "
                 "order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'total ms':>10} {'count':>7} {'avg us':>9}  kernel")
for name, n, t, avg in rows:
    print(f"{t / 1e6 / div:10.3f} {n / div:7.1f} {avg / 1e3:9.1f}  {name[:120]}")
print(f"{tot / 1e6 / div:10.3f}  all kernels")
