"""Per-launch SQ / GRBM counters of each kernel from one rocprofv3 --pmc pass (tools/pmc_valu.sh).

Reports the kernel's VALU instruction count per launch and the time that many wave64 VALU
instructions take at the chip's issue rate (MI355X_MICROARCH.md, per-instruction table: a wave64
v_fma_f32 issues in 2 cycles on a SIMD when several waves share it; 256 CUs x 4 SIMDs), so a
launch time can be compared with its VALU-issue floor.  Usage: valu.py OUT_DIR CONFIG [LAUNCH_US]
(LAUNCH_US: the un-instrumented average launch time of the sweep from bench.py, for the fraction).
"""
import csv
import hashlib
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
CYC_PER_VALU = 2.0
CLOCK_HZ = 2.4e9


def lib_sha256():
    """sha256 of the libkoordgpu.so the profiled bench loaded (bench.py refuses summaries of another build)"""
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "koordinator_amd", "libkoordgpu.so")
    with open(p, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    launch_us = float(sys.argv[3]) if len(sys.argv) > 3 else None
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                d = int(row["Dispatch_Id"])
                per[d][row["Counter_Name"]] += float(row["Counter_Value"])
                names[d] = row["Kernel_Name"].split("(")[0]
    by_kernel = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(int)
    for d, cs in per.items():
        k = names[d]
        launches[k] += 1
        for c, v in cs.items():
            by_kernel[k][c] += v
    out = {"config": cfg, "lib_sha256": lib_sha256(), "method": f"rocprofv3 --pmc (one pass) of bench.py --config {cfg}; per-launch averages; "
           f"VALU floor = SQ_INSTS_VALU x {CYC_PER_VALU} cyc / ({SIMDS} SIMDs x {CLOCK_HZ / 1e9} GHz)", "kernels": {}}
    for k, cs in sorted(by_kernel.items()):
        n = launches[k]
        avg = {c: v / n for c, v in cs.items()}
        e = {"launches": n, **{c: round(v, 1) for c, v in avg.items()}}
        if "SQ_INSTS_VALU" in avg:
            floor_us = avg["SQ_INSTS_VALU"] * CYC_PER_VALU / (SIMDS * CLOCK_HZ) * 1e6
            e["valu_issue_floor_us"] = round(floor_us, 3)
            if "SQ_WAVES" in avg and avg["SQ_WAVES"]:
                e["valu_insts_per_wave"] = round(avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"], 1)
            if launch_us and k.startswith("void sweep_kernel"):
                e["launch_us_unprofiled"] = launch_us
                e["valu_issue_frac"] = round(floor_us / launch_us, 3)
        out["kernels"][k] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
