"""GPU parity of the per-pod framework mode: ks_eval_pod (Filter + Score without Reserve, caller buffers),
ks_assume (Reserve of every plugin on the node the framework picked) and ks_unreserve (Unreserve of every plugin
+ ForgetPod), against the oracle's ko_eval_pod / ko_assume / ko_unreserve, on C2 (quota), C3 (devices, cpusets,
SingleNUMANode nodes) and C4 (reservations): placements, reservations, minors, CPUs, NUMA allocations and every
state table after each step; schedule -> unreserve-all returns the loaded state bit for bit."""
import numpy as np
import pytest

from assume_util import assert_states_equal, state, workloads
from koordinator_amd import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


def pick(total):
    """selectHost: the highest total, the lowest index on ties; -1 when no node is feasible"""
    if total.max() < 0:
        return -1
    return int(np.argmax(total))


@pytest.mark.parametrize("wi", [0, 1, 2, 3], ids=["c2", "c3", "c4", "c3rsv"])
def test_eval_pick_assume_matches_oracle(runtime, oracle_lib, wi):
    w = workloads()[wi]
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    placed = 0
    for i in range(80):
        pod = w.pods.rows([i])
        rg, sg, tg = ev.eval_pod(pod)
        ro, so, to = orc.eval_pod(pod)
        assert np.array_equal(rg, ro) and np.array_equal(tg, to), f"pod {i}: eval"
        node = pick(tg)
        if node < 0:
            continue
        a, csa, naa = ev.assume(pod, node)
        b, csb, nab = orc.assume(pod, node)
        for k in ("node", "status", "reservation", "gpu_minors", "rdma_minors"):
            assert a[0][k] == b[0][k], f"pod {i}: {k} {a[0][k]} vs {b[0][k]}"
        assert np.array_equal(csa, csb), f"pod {i}: cpuset"
        assert np.array_equal(naa, nab), f"pod {i}: NUMA allocation"
        placed += int(a[0]["status"] == abi.KS_S_SCHEDULED)
    assert placed > 40
    assert_states_equal(state(ev, w), state(orc, w), w.name)
    ev.close()
    orc.close()


@pytest.mark.parametrize("wi", [0, 1, 2, 3], ids=["c2", "c3", "c4", "c3rsv"])
def test_schedule_then_unreserve(runtime, oracle_lib, wi):
    w = workloads()[wi]
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    s0 = state(ev, w)
    rg = ev.schedule_raw(w.pods)
    ro = orc.schedule_raw(w.pods)
    for k in ("node", "status", "reservation", "gpu_minors", "rdma_minors"):
        assert np.array_equal(rg[k], ro[k]), k
    cs = ev.fetch_cpusets(w.pods.n)
    assert np.array_equal(cs, orc.fetch_cpusets(w.pods.n))
    na = ev.fetch_numa_alloc(w.pods.n) if w.numa_nodes is not None else [None] * w.pods.n
    placed = np.nonzero(rg["status"] == abi.KS_S_SCHEDULED)[0]
    assert placed.size > 50
    # Permit / Bind failures of every other placed pod, latest first
    for i in placed[::-2]:
        pod = w.pods.rows([int(i)])
        ev.unreserve(pod, rg[i:i + 1], cs[i], na[i])
        orc.unreserve(pod, ro[i:i + 1], cs[i], na[i])
    assert_states_equal(state(ev, w), state(orc, w), w.name + " half unreserved")
    rest = sorted(set(placed.tolist()) - set(placed[::-2].tolist()), reverse=True)
    for i in rest:
        ev.unreserve(w.pods.rows([int(i)]), rg[i:i + 1], cs[i], na[i])
    assert_states_equal(state(ev, w), s0, w.name + " all unreserved")
    ev.close()
    orc.close()


def test_read_nodes_leaves_state_alone(runtime, oracle_lib):
    """ks_read_nodes computes the NodeInfo view into scratch: reading never changes a later schedule"""
    w = workloads()[2]
    a = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    b = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    for _ in range(3):
        a.read_nodes()
    ra, rb = a.schedule(w.pods), b.schedule(w.pods)
    for k in ("node", "status", "score", "reservation"):
        assert np.array_equal(ra[k], rb[k]), k
    a.close()
    b.close()


def test_assume_guards(runtime):
    """ks_assume overwrites the batch's cpuset / NUMA buffers (ks_fetch_cpusets refuses until the next schedule),
    and a node holding an assumed device pod refuses ks_update_devices until the pod is unreserved: its Unreserve
    re-derives the per-instance request from the node's device totals."""
    from test_gpu_deltas import dev_rows

    w = workloads()[1]  # C3: devices + cpusets
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    ev.schedule(w.pods.rows(range(20)))
    ev.fetch_cpusets(20)
    gpu = [i for i in range(20, 200) if w.pods.gpu_core[i] > 0 or w.pods.gpu_memory_ratio[i] > 0]
    pod = w.pods.rows([gpu[0]])
    _, _, tot = ev.eval_pod(pod)
    node = pick(tot)
    assert node >= 0
    r, cs, na = ev.assume(pod, node)
    assert r[0]["status"] == abi.KS_S_SCHEDULED and r[0]["gpu_minors"] != 0
    with pytest.raises(runtime.KsError):
        ev.fetch_cpusets(20)
    idx = np.array([node], np.int32)
    with pytest.raises(runtime.KsError):
        ev.update_devices(idx, dev_rows(w.devices, idx))
    ev.update_devices(np.array([(node + 1) % w.nodes.n], np.int32), dev_rows(w.devices, np.array([(node + 1) % w.nodes.n])))
    ev.unreserve(pod, r, cs, na)
    ev.update_devices(idx, dev_rows(w.devices, idx))
    ev.schedule(w.pods.rows(range(20, 40)))
    ev.fetch_cpusets(20)
    ev.close()
