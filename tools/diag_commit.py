"""Diagnostic: per-phase cycle split of the commit kernel (libkoordgpu_diag.so, -DKS_COMMIT_STAMPS) or, with
--cat, per-pod-category cycles (libkoordgpu_cat.so, -DKS_COMMIT_CAT); both built by tools/build_diag.sh.
--seg: the fast pods' iteration split (libkoordgpu_seg.so, -DKS_COMMIT_SEG; monotone commit kernel only).
--split: the slot evaluation's parts timed separately (libkoordgpu_split.so, -DKS_COMMIT_STAMPS -DKS_SLOT_SPLIT).
usage: python tools/diag_commit.py [c2|c3|c4|c5|c2d] [--cat|--seg|--split]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CAT = "--cat" in sys.argv
SEG = "--seg" in sys.argv
SPLIT = "--split" in sys.argv
sys.argv = [a for a in sys.argv if a not in ("--cat", "--seg", "--split")]
os.environ.setdefault("KS_LIB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "koordinator_amd",
                                                  "libkoordgpu_seg.so" if SEG else ("libkoordgpu_cat.so" if CAT else (
                                                      "libkoordgpu_split.so" if SPLIT else "libkoordgpu_diag.so"))))
from koordinator_amd import runtime, synth
which = sys.argv[1] if len(sys.argv) > 1 else "c2"
w = {"c2": synth.c2, "c3": synth.c3, "c4": synth.c4, "c2d": synth.c2_default, "c2s": synth.c2_default,
     "c5": lambda: synth.c5(n_pods=100_000)}[which]()
cfg = w.cfg
cfg.profile = 1
ev = runtime.Evaluator(cfg, w.nodes, **w.tables(copy=False))
ev.stage(w.pods)
ev.checkpoint()
for i in range(3):
    ev.restore(); ev.schedule_staged(); st = ev.stats()
if SPLIT:
    d = st["diag"]
    print(w.name, {k: st[k] for k in ("passes", "commit_ms")})
    for nm, v in zip(("Fit+LoadAware+NUMA none", "NUMA policy path", "DeviceShare Filter/Score", "(DeviceShare hints alone)"), d[:4]):
        print(f"{nm:26s} {v:14d} cycles {v / w.pods.n:10.1f} cyc/pod (slowest lane, re-run ahead of the slot evaluation)")
    sys.exit(0)
if SEG:
    d = st["diag"]
    nf = max(d[7], 1)
    print(w.name, {k: st[k] for k in ("passes", "rescans", "commit_ms")}, "fast", d[7])
    for nm, v in zip(("admission+fast check", "slot assignment", "row reserve", "result+quota"), d[:4]):
        print(f"{nm:22s} {v / nf:9.1f} cyc per fast pod")
    print(f"{'other pods':22s} {d[4] / max(w.pods.n - d[7], 1):9.1f} cyc per pod")
    sys.exit(0)
if CAT:
    d = st["diag"]
    n_fast, n_new, n_old = d[7], d[5], d[6]
    print(w.name, {k: st[k] for k in ("passes", "cut_passes", "rescans", "slot_misses", "commit_ms")})
    for nm, cyc, cnt in (("rejected/unsched", d[0] + d[4], None), ("fast", d[1], n_fast), ("slow->new slot", d[2], n_new),
                         ("slow->touched slot", d[3], n_old)):
        print(f"{nm:20s} {cyc:14d} cycles" + (f"  n={cnt:8d}  {cyc/max(cnt,1):9.1f} cyc/pod" if cnt is not None else ""))
    sys.exit(0)
names = ["prefetch", "lookahead(quota+cands)", "slot_eval", "rescans+cut", "reserve_row", "reserve_rest", "loop_exit"]
tot = sum(st["diag"][:7])
print(w.name, {k: st[k] for k in ("passes", "cut_passes", "rescans", "slot_misses", "sweep_ms", "select_ms", "commit_ms", "total_ms")}, "fast_picks", st["diag"][7])
for n, v in zip(names, st["diag"][:7]):
    print(f"{n:20s} {v:14d} cycles  {100.0*v/max(tot,1):6.2f}%  {v/w.pods.n:10.1f} cyc/pod")
