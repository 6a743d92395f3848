"""Per-kernel summary (calls, average and total duration) of a rocprofv3 rocpd database: python tools/rocpd_stats.py DB [N]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
q = ("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1e6 from kernels group by name "
     "order by sum(end-start) desc limit ?")
print(f"{'kernel':70s} {'calls':>7s} {'avg_us':>8s} {'total_ms':>9s}")
for name, n, avg, tot in db.execute(q, (top,)):
    print(f"{name[:70]:70s} {n:7d} {avg:8.2f} {tot:9.2f}")
