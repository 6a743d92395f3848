import sys, time
sys.path.insert(0, '/root/repo')
import numpy as np
from koordinator_amd import synth
from oracle.oracle import Oracle
cfgname = sys.argv[1] if len(sys.argv) > 1 else 'c5'
npass = int(sys.argv[2]) if len(sys.argv) > 2 else 20
w = getattr(synth, cfgname)(n_pods=64 * (npass + 1)) if cfgname == 'c5' else getattr(synth, cfgname)()
cur = Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
lag = Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
def top(o, pod):
    r, s, t = o.eval_pod(pod)
    feas = r == 0
    if not feas.any(): return -1
    tt = np.where(feas, t, -1)
    return int(np.argmax(tt))  # lowest index among max
prev_nodes = set()
fast_np = fast_p = tot = 0
for k in range(npass):
    idx = range(64 * k, 64 * (k + 1))
    P = w.pods.rows(idx)
    tn = [top(cur, w.pods.rows([i])) for i in idx]
    tp = [top(lag, w.pods.rows([i])) for i in idx]
    res = cur.schedule(P)
    nodes = [int(x) for x in res['node']]
    touched = set()
    for j in range(64):
        if res['status'][j] != 0:
            continue
        tot += 1
        if tn[j] >= 0 and tn[j] not in touched: fast_np += 1
        if tp[j] >= 0 and tp[j] not in touched and tp[j] not in prev_nodes: fast_p += 1
        touched.add(nodes[j])
    if k > 0:
        lag.schedule(w.pods.rows(range(64 * (k - 1), 64 * k)))
    prev_nodes = touched
    print(k, fast_np, fast_p, tot, flush=True)
print('fast non-pipelined %.3f pipelined %.3f' % (fast_np / tot, fast_p / tot))
