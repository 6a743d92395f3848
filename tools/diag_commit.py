"""Diagnostic: per-phase cycle split of the commit kernel (needs libkoordgpu_diag.so, -DKS_COMMIT_STAMPS).
usage: python tools/diag_commit.py [c2|c3|c4]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("KS_LIB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "koordinator_amd", "libkoordgpu_diag.so"))
from koordinator_amd import runtime, synth
which = sys.argv[1] if len(sys.argv) > 1 else "c2"
w = {"c2": synth.c2, "c3": synth.c3, "c4": synth.c4}[which]()
cfg = w.cfg
cfg.profile = 1
ev = runtime.Evaluator(cfg, w.nodes, **w.tables(copy=False))
ev.stage(w.pods)
ev.checkpoint()
for i in range(3):
    ev.restore(); ev.schedule_staged(); st = ev.stats()
names = ["prefetch", "lookahead(quota+cands)", "slot_eval", "rescans+cut", "reserve_row", "reserve_rest", "loop_exit"]
tot = sum(st["diag"][:7])
print(w.name, {k: st[k] for k in ("passes", "cut_passes", "rescans", "slot_misses", "sweep_ms", "select_ms", "commit_ms", "total_ms")}, "fast_picks", st["diag"][7])
for n, v in zip(names, st["diag"][:7]):
    print(f"{n:20s} {v:14d} cycles  {100.0*v/max(tot,1):6.2f}%  {v/w.pods.n:10.1f} cyc/pod")
