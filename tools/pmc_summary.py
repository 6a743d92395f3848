"""Average PMC counter values per dispatch for kernels whose name contains a filter string.
usage: python tools/pmc_summary.py <rocprofv3 output dir> [name filter]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
sums = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            if filt not in name:
                continue
            short = name.split("(")[0][-60:]
            key = (os.path.dirname(f), row.get("Dispatch_Id"))
            disp[short][row["Counter_Name"]].add(key)
            sums[short][row["Counter_Name"]] += float(row["Counter_Value"])
for k, cs in sums.items():
    print(k, "dispatches", max(len(v) for v in disp[k].values()))
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {v / max(len(disp[k][c]), 1):14.1f} per dispatch")
