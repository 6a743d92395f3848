"""The oracle's per-pod framework mode (ko_assume / ko_unreserve, CPU only): Reserve then Unreserve of every
plugin is an exact round trip -- schedule a queue, unreserve every placed pod in reverse order, and every table
(NodeInfo, assign cache, quota used, reservation allocated / assigned, device used, CPU sets, NUMA-node
allocations) is back to its loaded value; an assume at the node the scheduler would pick equals the schedule."""
import numpy as np
import pytest

from assume_util import assert_states_equal, state, workloads
from koordinator_amd import abi
from oracle.oracle import Oracle


@pytest.mark.parametrize("wi", [0, 1, 2], ids=["c2", "c3", "c4"])
def test_schedule_unreserve_round_trip(wi):
    w = workloads()[wi]
    orc = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    s0 = state(orc, w)
    res = orc.schedule_raw(w.pods)
    cs = orc.fetch_cpusets(w.pods.n)
    placed = np.nonzero(res["status"] == abi.KS_S_SCHEDULED)[0]
    assert placed.size > 50
    for i in placed[::-1]:
        orc.unreserve(w.pods.rows([int(i)]), res[i:i + 1], cs[i], None)
    s1 = state(orc, w)
    # NUMA-node allocations need the per-pod allocation (the assume test covers them); compare the rest
    for k in [k for k in s0 if k.startswith("numa.")]:
        s0.pop(k), s1.pop(k)
    assert_states_equal(s0, s1, w.name)
    orc.close()


@pytest.mark.parametrize("wi", [0, 1, 2], ids=["c2", "c3", "c4"])
def test_assume_at_the_chosen_node_equals_schedule(wi):
    w = workloads()[wi]
    a = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    b = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    nalloc = []
    for i in range(60):
        pod = w.pods.rows([i])
        r = b.schedule_raw(pod)[0]
        if r["status"] != abi.KS_S_SCHEDULED:
            continue
        ra, csa, na = a.assume(pod, int(r["node"]))
        assert ra[0]["status"] == abi.KS_S_SCHEDULED
        for k in ("node", "reservation", "gpu_minors", "rdma_minors"):
            assert ra[0][k] == r[k], (i, k)
        assert np.array_equal(csa, b.fetch_cpusets(1)[0]), i
        nalloc.append((pod, ra, csa, na))
    assert_states_equal(state(a, w), state(b, w), w.name)
    # and the assumes undone in reverse order restore the loaded state exactly (NUMA allocations included)
    c = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    s0 = state(c, w)
    for pod, ra, csa, na in nalloc[::-1]:
        a.unreserve(pod, ra, csa, na)
    assert_states_equal(s0, state(a, w), w.name + " round trip")
    for o in (a, b, c):
        o.close()
