"""One line per record of a bench.py JSON line: pods/s, ms per step, kernel split (tools/*.sh summaries)."""
import json
import sys

d = json.load(open(sys.argv[1]))
recs = [("main", d)] + [(k, d[k]) for k in ("c5", "c3", "c4", "c2d", "preempt", "c2_replicas") if isinstance(d.get(k), dict)]
for name, r in recs:
    print(name, r["value"], r.get("ms_per_step"), r.get("parity"), r.get("kernel_ms_per_step"),
          (r.get("cpu_baseline") or {}).get("value"))
