"""Wall-clock of ks_schedule on c3r with and without device-holding reservations (development A/B aid)."""
import os
import sys
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
from koordinator_amd import runtime as rt, synth  # noqa: E402

for frac in [float(x) for x in sys.argv[1:]] or [0.0, 0.7]:
    w = synth.c3_rsv(dev_rsv_frac=frac)
    ev = rt.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    ev.stage(w.pods)
    ev.checkpoint()
    best = 1e9
    for _ in range(2):
        ev.restore()
        t0 = time.perf_counter()
        ev.schedule_staged()
        best = min(best, time.perf_counter() - t0)
    print(f"dev_rsv_frac={frac}: {w.pods.n / best:.0f} pods/s ({best * 1e3:.1f} ms)", flush=True)
    ev.close()
