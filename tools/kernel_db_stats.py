"""Per-kernel count / total / average duration from a rocprofv3 SQLite output (kernels view), plus the mean gap
between consecutive dispatches on the stream (launch overhead).  usage: kernel_db_stats.py DB [name-filter]"""
import glob
import sqlite3
import sys


def main():
    path = sys.argv[1]
    if not path.endswith(".db"):
        path = glob.glob(path + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end, duration from kernels order by start").fetchall()
    flt = sys.argv[2] if len(sys.argv) > 2 else None
    agg = {}
    for name, s, e, d in rows:
        short = name.split("(")[0].replace("void ", "")
        if flt and flt not in short:
            continue
        a = agg.setdefault(short, [0, 0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':70s} {'calls':>8s} {'total_ms':>10s} {'avg_us':>9s} {'share':>6s}")
    for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[:70]:70s} {n:8d} {d / 1e6:10.3f} {d / n / 1e3:9.2f} {d / tot:6.1%}")
    if len(rows) > 1:
        span = rows[-1][2] - rows[0][1]
        busy = sum(r[3] for r in rows)
        print(f"dispatches {len(rows)}, span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, "
              f"mean gap {(span - busy) / max(1, len(rows) - 1) / 1e3:.2f} us")


if __name__ == "__main__":
    main()
