import sys; sys.path.insert(0,'.')
from koordinator_amd import runtime, synth
w = synth.c5(n_pods=200_000)
ev = runtime.Evaluator(w.cfg, w.nodes, **w.tables(copy=False))
ev.stage(w.pods); ev.checkpoint()
for i in range(2):
    ev.restore(); ev.schedule_staged(); st = ev.stats()
print({k: st[k] for k in st if k not in ('diag',)})
