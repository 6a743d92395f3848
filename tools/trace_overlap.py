#!/usr/bin/env python3
"""Overlap of the pass kernels in a rocprofv3 --kernel-trace CSV (pipelined passes): for each
kernel family its launches, busy time, and how much of the commit kernels' time a sweep / select launch ran
concurrently with.  Usage: trace_overlap.py <kernel_trace.csv> > summary.json"""
import csv
import json
import sys


def family(name: str) -> str:
    for k in ("commit_mono_kernel", "commit_kernel", "sweep_kernel", "select_kernel", "merge_kernel", "prep_pods_kernel"):
        if k in name:
            return k
    return "other"


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b):
    """total length of the intersection of two sorted disjoint interval lists"""
    i = j = 0
    t = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            t += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return t


def main(path):
    fam = {}
    with open(path) as f:
        rd = csv.DictReader(f)
        cols = {c.lower(): c for c in rd.fieldnames}
        cs = next(cols[c] for c in cols if "start" in c)
        ce = next(cols[c] for c in cols if c.startswith("end"))
        cn = next(cols[c] for c in cols if "kernel_name" in c or c == "name")
        cq = cols.get("stream_id") or cols.get("queue_id")
        rows = [(family(r[cn]), int(r[cs]), int(r[ce]), r.get(cq) if cq else None) for r in rd]
    # a sweep_kernel launched on the commit kernels' stream is the patched pipeline's list re-evaluation
    # (DESIGN.md §5a), not a speculative sweep
    commit_streams = {q for f, _, _, q in rows if f.startswith("commit")}
    for f, s, e, q in rows:
        if f == "sweep_kernel" and q is not None and q in commit_streams:
            f = "sweep_kernel (list re-evaluation, commit stream)"
        fam.setdefault(f, []).append((s, e))
    uni = {k: union(v) for k, v in fam.items()}
    commit = union(uni.get("commit_mono_kernel", []) + uni.get("commit_kernel", []))
    ct = sum(e - s for s, e in commit)
    out = {"source": path, "kernels": {}}
    for k, v in fam.items():
        out["kernels"][k] = {"launches": len(v), "busy_ms": round(sum(e - s for s, e in uni[k]) / 1e6, 3),
                             "sum_ms": round(sum(e - s for s, e in v) / 1e6, 3)}
    for k in ("sweep_kernel", "select_kernel"):
        if k in uni and ct:
            ov = overlap(commit, uni[k])
            out[f"commit_time_overlapped_by_{k}"] = {"ms": round(ov / 1e6, 3), "frac_of_commit": round(ov / ct, 4)}
    allk = union([x for v in uni.values() for x in v])
    if allk:
        span = allk[-1][1] - allk[0][0]
        out["span_ms"] = round(span / 1e6, 3)
        out["gpu_busy_ms"] = round(sum(e - s for s, e in allk) / 1e6, 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
