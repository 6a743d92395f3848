"""Per-launch HBM bytes of each kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half the bytes of a wide
coalesced read, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Usage: traffic.py OUT_DIR CONFIG
"""
import csv
import hashlib
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(root, counter):
    vals = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                d = int(row["Dispatch_Id"])
                vals[d] += float(row["Counter_Value"])
                names[d] = row["Kernel_Name"]
    return vals, names


def lib_sha256():
    """sha256 of the libkoordgpu.so the profiled bench loaded (bench.py refuses summaries of another build)"""
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "koordinator_amd", "libkoordgpu.so")
    with open(p, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    fetch, names = per_dispatch(root, "FETCH_SIZE")
    write, wnames = per_dispatch(root, "WRITE_SIZE")
    by_kernel = defaultdict(lambda: {"launches": 0, "fetch_kib": 0.0, "launches_w": 0, "write_kib": 0.0})
    for d, v in fetch.items():
        k = names[d].split("(")[0]
        by_kernel[k]["launches"] += 1
        by_kernel[k]["fetch_kib"] += v
    for d, v in write.items():
        k = wnames[d].split("(")[0]
        by_kernel[k]["launches_w"] += 1
        by_kernel[k]["write_kib"] += v
    out = {"config": cfg, "lib_sha256": lib_sha256(), "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
           f"bench.py --config {cfg} --steps 1 --warmup 0; bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch", "kernels": {}}
    for k, a in sorted(by_kernel.items()):
        if not a["launches"] or not a["launches_w"]:
            continue
        f = a["fetch_kib"] / a["launches"]
        w = a["write_kib"] / a["launches_w"]
        out["kernels"][k] = {"launches": a["launches"], "fetch_kib_per_launch": round(f, 3),
                             "write_kib_per_launch": round(w, 3), "hbm_bytes_per_launch": round((2 * f + w) * 1024)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
