"""GPU parity under forced sweep launch shapes.

The sweep's grid-stride loop over (chunk, pod group) items must give the same candidates for any
pods-per-wave and block count.  The overrides (KS_SWEEP_PPW / KS_SWEEP_BLOCK_CAP) are read once
per process, so each shape runs in a child process: C2-shaped (ElasticQuota) and C4-shaped
(Reservation) clusters, checked bit-exact against the CPU oracle.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import numpy as np
from koordinator_amd import runtime, synth
from oracle.oracle import Oracle

for w in (synth.c2(n_nodes=900, n_pods=384), synth.c4(n_nodes=700, n_reservations=1500, n_pods=256)):
    q = w.quotas.copy() if w.quotas is not None else None
    rs = w.reservations.copy() if w.reservations is not None else None
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), q, rs)
    got = ev.schedule(w.pods)
    orc = Oracle(w.cfg, w.nodes.copy(), w.quotas.copy() if w.quotas is not None else None, nthreads=4,
                 reservations=w.reservations.copy() if w.reservations is not None else None)
    want = orc.schedule(w.pods)
    for k in ("node", "status", "score", "reservation"):
        assert np.array_equal(got[k], want[k]), (w.name, k)
    gs, ws = ev.read_nodes().as_dict(), orc.read_nodes().as_dict()
    for k in ws:
        assert np.array_equal(gs[k], ws[k]), (w.name, "node state", k)
    ev.close()
    orc.close()
print("SHAPE OK")
"""


@pytest.mark.parametrize("ppw,cap", [(1, 8), (3, 24), (4, 16), (64, 8)])
def test_sweep_shape_invariant(ppw, cap):
    env = dict(os.environ, KS_SWEEP_PPW=str(ppw), KS_SWEEP_BLOCK_CAP=str(cap))
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "SHAPE OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
