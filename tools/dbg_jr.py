# debugging aid: GPU vs oracle eval of one pod after a queue prefix (C3 with joint pods without an RDMA request)
import sys
import numpy as np
sys.path[:0] = [".", "tests"]
from koordinator_amd import synth, runtime
from oracle.oracle import Oracle
seed, k = 56, 183
w = synth.c3(seed=seed, n_nodes=500, n_pods=700)
rng = np.random.Generator(np.random.PCG64(seed))
jr = (w.pods.joint != 0) & (rng.random(w.pods.n) < 0.35)
w.pods.rdma[jr] = 0
ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
o = Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
pre = w.pods.rows(list(range(k)))
g1, o1 = ev.schedule(pre), o.schedule(pre)
print("prefix equal", all(np.array_equal(g1[x], o1[x]) for x in ("node", "status", "score", "gpu_minors", "rdma_minors")))
p = w.pods.rows([k])
rg, sg, tg = ev.eval_pod(p)
ro, so, to = o.eval_pod(p)
bad = np.nonzero((rg != ro) | (tg != to) | (sg != so).any(1))[0]
print("eval differs at", bad[:20].tolist())
for n in bad[:5]:
    print(n, "gpu", hex(rg[n]), tg[n], sg[n].tolist(), "orc", hex(ro[n]), to[n], so[n].tolist())
