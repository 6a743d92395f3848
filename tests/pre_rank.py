"""How often a pod's commit winner is among its snapshot top-M nodes (the nodes reserve_pre_kernel precomputes
Reserve for): replays passes of 64 pods on the CPU oracle, ranking every node for each pod on the state at the pass
start (ko_eval_pod) and placing the pass sequentially (ko_schedule).
usage: python tests/pre_rank.py [c3|c4|c2] [passes]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import synth  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "c3"
npass = int(sys.argv[2]) if len(sys.argv) > 2 else 6
w = {"c3": synth.c3, "c4": synth.c4, "c2": synth.c2}[which](n_pods=64 * npass)
orc = Oracle(w.cfg, w.nodes.copy(), **w.tables())
ranks = []
for p in range(npass):
    idx = np.arange(64 * p, 64 * p + 64)
    keys = []
    for j in idx:
        r, _, tot = orc.eval_pod(w.pods.rows([int(j)]))
        keys.append(np.where(r == 0, (tot + 1) * (1 << 32) + (0xFFFFFFFF - np.arange(w.nodes.n)), 0))
    res = orc.schedule(w.pods.rows(idx))
    for jj in range(64):
        nd = res["node"][jj]
        if res["status"][jj] == 0 and nd >= 0:
            ranks.append(int((keys[jj] > keys[jj][nd]).sum()))
ranks = np.array(ranks)
for m in (1, 2, 4, 8, 16, 32):
    print(f"{which}: winner within the snapshot top-{m}: {np.mean(ranks < m):.3f}")
print("placed pods:", len(ranks))
orc.close()
