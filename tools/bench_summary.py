"""One line per record of a bench.py JSON line: pods/s, ms per step, parity, the §8(d) pass roofline fraction, the
commit kernel's time per pass, the CPU baseline."""
import json
import sys

d = json.load(open(sys.argv[1]))
recs = [("main", d)] + [(k, v) for k, v in d.items() if isinstance(v, dict) and "value" in v]
for name, r in recs:
    roof = r.get("roofline") or {}
    print(name, r["value"], r.get("ms_per_step"), "parity", r.get("parity"), "frac", roof.get("frac"),
          "sweep_frac", roof.get("sweep_frac"), "commit_us", roof.get("commit_us"),
          "cpu", (r.get("cpu_baseline") or {}).get("value"))
